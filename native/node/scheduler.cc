// scheduler.cc — GPU-aware single-cluster scheduler (see node.h).
#include <unistd.h>

#include <algorithm>
#include <set>

#include "apiserver/selector.h"
#include "controllers/common.h"
#include "core/resources.h"
#include "core/util.h"
#include "node/node.h"

namespace kf {

// Quantities were validated by the API server (core/resources.h), so a parse failure here means a
// value the API server never saw (node status, a quota written before validation): it counts 0.
// amd.com/gpu-memory is counted in GiB, as the node advertises it: a unit-suffixed value
// ("300Gi", "322G") is converted, a bare number is already GiB.
double resource_value(const std::string& name, const Json& q) {
  if (q.is_number()) return q.as_double();
  auto v = parse_quantity(q.as_string());
  if (!v) return 0.0;
  if (contains(name, "gpu-memory") && q.as_string().find_first_of("kKMGTPEi") != std::string::npos)
    return *v / (1024.0 * 1024.0 * 1024.0);
  return *v;
}

Json pod_requests(const Json& pod) {
  std::map<std::string, double> sum, init_max;
  // requests (defaulted from limits at admission); restartable init containers (sidecars) run
  // beside the app containers, so their requests add to the app sum
  auto add_container = [](const Json& c, std::map<std::string, double>& into, bool max_mode) {
    std::map<std::string, double> one;
    for (const auto& m : c.at_path({"resources", "limits"}).as_object()) one[m.first] = resource_value(m.first, m.second);
    for (const auto& m : c.at_path({"resources", "requests"}).as_object()) one[m.first] = resource_value(m.first, m.second);
    for (auto& kv : one) into[kv.first] = max_mode ? std::max(into[kv.first], kv.second) : into[kv.first] + kv.second;
  };
  for (const auto& c : pod.at_path({"spec", "containers"}).as_array()) add_container(c, sum, false);
  for (const auto& c : pod.at_path({"spec", "initContainers"}).as_array())
    add_container(c, c["restartPolicy"].as_string() == "Always" ? sum : init_max, c["restartPolicy"].as_string() != "Always");
  Json out = Json::object();
  for (auto& kv : sum) out[kv.first] = std::max(kv.second, init_max[kv.first]);
  for (auto& kv : init_max)
    if (!out.has(kv.first)) out[kv.first] = kv.second;
  // GPUs: exactly what the device plugin will allocate (the shared count, core/resources.h)
  if (auto g = pod_gpu_count(pod, GPU_RESOURCE); g && *g > 0) out[GPU_RESOURCE] = static_cast<double>(*g);
  return out;
}

bool Scheduler::tolerates(const Json& pod, const Json& node) {
  for (const auto& taint : node.at_path({"spec", "taints"}).as_array()) {
    const std::string& effect = taint["effect"].as_string();
    if (effect != "NoSchedule" && effect != "NoExecute") continue;
    bool ok = false;
    for (const auto& t : pod.at_path({"spec", "tolerations"}).as_array()) {
      if (!t["effect"].as_string().empty() && t["effect"].as_string() != effect) continue;
      const std::string op = t["operator"].as_string_or("Equal");
      if (t["key"].as_string().empty() && op == "Exists") {
        ok = true;
        break;
      }
      if (t["key"].as_string() != taint["key"].as_string()) continue;
      if (op == "Exists" || t["value"].as_string() == taint["value"].as_string()) {
        ok = true;
        break;
      }
    }
    if (!ok) return false;
  }
  return true;
}

bool Scheduler::matches_affinity(const Json& pod, const Json& node) {
  const Json& labels = node.at_path({"metadata", "labels"});
  for (const auto& m : pod.at_path({"spec", "nodeSelector"}).as_object())
    if (labels[m.first].as_string() != m.second.as_string()) return false;
  const Json& req = pod.at_path({"spec", "affinity", "nodeAffinity", "requiredDuringSchedulingIgnoredDuringExecution"});
  if (req.is_object()) {
    const Json& terms = req["nodeSelectorTerms"];
    if (terms.is_array() && !terms.empty()) {
      bool any = false;
      for (const auto& t : terms.as_array()) any = any || match_node_selector_term(t, node);
      if (!any) return false;
    }
  }
  return true;
}

int64_t Scheduler::preferred_score(const Json& pod, const Json& node) {
  int64_t s = 0;
  for (const auto& p : pod.at_path({"spec", "affinity", "nodeAffinity", "preferredDuringSchedulingIgnoredDuringExecution"}).as_array())
    if (match_node_selector_term(p["preference"], node)) s += p["weight"].as_int(1);
  return s;
}

Result Scheduler::reconcile(const Request& r, std::string* err) {
  Json pod;
  if (!pods_->get(r.ns, r.name, pod)) return {};
  if (!pod.at_path({"spec", "nodeName"}).as_string().empty()) return {};
  if (pod.at_path({"metadata", "deletionTimestamp"}).is_string()) return {};
  if (pod.at_path({"spec", "schedulerName"}).as_string_or("default-scheduler") != "default-scheduler") return {};
  const Json req = pod_requests(pod);
  std::vector<std::string> reasons;
  std::string best;
  double best_score = -1;
  auto nodes = nodes_->list();
  for (const auto& node : nodes) {
    const std::string name = node.str_at({"metadata", "name"});
    bool ready = false;
    for (const auto& c : node.at_path({"status", "conditions"}).as_array())
      if (c["type"].as_string() == "Ready") ready = c["status"].as_string() == "True";
    if (!ready) {
      reasons.push_back("node(s) were not ready");
      continue;
    }
    if (node.at_path({"spec", "unschedulable"}).as_bool()) {
      reasons.push_back("node(s) were unschedulable");
      continue;
    }
    if (!tolerates(pod, node)) {
      reasons.push_back("node(s) had untolerated taint");
      continue;
    }
    if (!matches_affinity(pod, node)) {
      reasons.push_back("node(s) didn't match Pod's node affinity/selector");
      continue;
    }
    // resource fit: bound pods from the cache + pods this scheduler assumed onto the node whose
    // binding the cache has not shown yet (kube-scheduler's assume cache)
    std::map<std::string, double> used;
    int64_t npods = 0;
    std::set<std::string> cached_bound;
    pods_->visit("", [&](const Json& p) {
      const std::string& bound = p.at_path({"spec", "nodeName"}).as_string();
      if (!bound.empty() && assumed_.count(ns_name(p))) cached_bound.insert(ns_name(p));
      if (bound != name) return;
      const std::string& ph = p.at_path({"status", "phase"}).as_string();
      if (ph == "Succeeded" || ph == "Failed") return;
      npods++;
      const Json req = pod_requests(p);
      for (const auto& m : req.as_object()) used[m.first] += m.second.as_double();
    });
    for (auto it = assumed_.begin(); it != assumed_.end();) {
      Json cur;
      if (cached_bound.count(it->first) || !pods_->get(it->second.ns, it->second.name, cur) ||
          !cur.at_path({"spec", "nodeName"}).as_string().empty()) {
        it = assumed_.erase(it);
        continue;
      }
      if (it->second.node == name) {
        npods++;
        for (const auto& m : it->second.requests.as_object()) used[m.first] += m.second.as_double();
      }
      ++it;
    }
    const Json& alloc = node.at_path({"status", "allocatable"});
    bool fits = true;
    if (alloc.has("pods") && npods + 1 > resource_value("pods", alloc["pods"])) {
      reasons.push_back("Too many pods");
      fits = false;
    }
    double free_frac = 0;
    int counted = 0;
    for (const auto& m : req.as_object()) {
      const double want = m.second.as_double();
      if (want <= 0) continue;
      if (!alloc.has(m.first)) {
        if (m.first == "cpu" || m.first == "memory" || m.first == "ephemeral-storage") continue;
        reasons.push_back("Insufficient " + m.first);
        fits = false;
        break;
      }
      const double cap = resource_value(m.first, alloc[m.first]);
      if (used[m.first] + want > cap + 1e-9) {
        reasons.push_back("Insufficient " + m.first);
        fits = false;
        break;
      }
      free_frac += (cap - used[m.first] - want) / std::max(cap, 1e-9);
      counted++;
    }
    if (!fits) continue;
    double score = static_cast<double>(preferred_score(pod, node)) * 100.0 + (counted ? free_frac / counted : 1.0) * 10.0;
    if (score > best_score) {
      best_score = score;
      best = name;
    }
  }
  if (best.empty()) {
    std::map<std::string, int> counts;
    for (auto& s : reasons) counts[s]++;
    std::string msg = "0/" + std::to_string(nodes.size()) + " nodes are available";
    std::vector<std::string> parts;
    for (auto& kv : counts) parts.push_back(std::to_string(kv.second) + " " + kv.first);
    if (!parts.empty()) msg += ": " + join(parts, ", ");
    msg += ".";
    bool changed = false;
    c_->update_with_retry(
        "v1", "Pod", r.ns, r.name,
        [&](Json& p) {
          Json conds = Json::array();
          for (const auto& c : p.at_path({"status", "conditions"}).as_array())
            if (c["type"].as_string() != "PodScheduled") conds.push_back(c);
          const Json* prev = nullptr;
          for (const auto& c : p.at_path({"status", "conditions"}).as_array())
            if (c["type"].as_string() == "PodScheduled") prev = &c;
          if (prev && (*prev)["message"].as_string() == msg) return false;
          conds.push_back(Json{{"type", "PodScheduled"}, {"status", "False"}, {"reason", "Unschedulable"},
                               {"message", msg}, {"lastProbeTime", Json()}, {"lastTransitionTime", rfc3339_ms_now()}});
          p["status"]["conditions"] = conds;
          changed = true;
          return true;
        },
        true);
    if (changed) rec_->event(pod, "Warning", "FailedScheduling", msg);
    return Result::after(2.0);
  }
  ApiError e = c_->update_with_retry("v1", "Pod", r.ns, r.name, [&](Json& p) {
    if (!p.at_path({"spec", "nodeName"}).as_string().empty()) return false;
    p["spec"]["nodeName"] = best;
    return true;
  });
  if (e) {
    *err = e.message;
    return {};
  }
  c_->update_with_retry(
      "v1", "Pod", r.ns, r.name,
      [&](Json& p) {
        Json conds = Json::array();
        for (const auto& c : p.at_path({"status", "conditions"}).as_array())
          if (c["type"].as_string() != "PodScheduled") conds.push_back(c);
        conds.push_back(Json{{"type", "PodScheduled"}, {"status", "True"}, {"lastProbeTime", Json()},
                             {"lastTransitionTime", rfc3339_ms_now()}});
        p["status"]["conditions"] = conds;
        return true;
      },
      true);
  rec_->event(pod, "Normal", "Scheduled", "Successfully assigned " + r.ns + "/" + r.name + " to " + best);
  // assume the binding so the next decision accounts for this pod's CPU / GPUs / HBM before the
  // watch event reaches our cache (instead of blocking the worker until it does)
  assumed_[r.ns + "/" + r.name] = Assumed{r.ns, r.name, best, req};
  return {};
}

void Scheduler::setup(Manager& mgr) {
  pods_ = &mgr.informer("v1", "Pod");
  nodes_ = &mgr.informer("v1", "Node");
  rec_ = std::make_unique<EventRecorder>(c_, "default-scheduler");
  ctl_ = std::make_shared<Controller>("default-scheduler", [this](const Request& r, std::string* e) { return reconcile(r, e); });
  ctl_->For(*pods_, [](const std::string& type, const Json& p, const Json*) {
    return type != "DELETED" && p.at_path({"spec", "nodeName"}).as_string().empty();
  });
  // capacity changes (node updates, pods finishing) re-trigger pending pods
  auto requeue_pending = [this](const std::string&, const Json&) {
    std::vector<Request> out;
    pods_->visit("", [&](const Json& p) {
      if (p.at_path({"spec", "nodeName"}).as_string().empty())
        out.push_back({p.str_at({"metadata", "namespace"}), p.str_at({"metadata", "name"})});
    });
    return out;
  };
  ctl_->Watches(*nodes_, requeue_pending, [](const std::string& type, const Json& n, const Json* old) {
    return type != "MODIFIED" || !old || n["status"]["allocatable"] != (*old)["status"]["allocatable"] ||
           n.at_path({"spec", "unschedulable"}) != old->at_path({"spec", "unschedulable"});
  });
  ctl_->Watches(*pods_, requeue_pending, [](const std::string& type, const Json& p, const Json*) {
    const std::string& ph = p.at_path({"status", "phase"}).as_string();
    return type == "DELETED" || ph == "Succeeded" || ph == "Failed";
  });
  mgr.add(ctl_);
}

}  // namespace kf
