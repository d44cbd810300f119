// quota.cc — ResourceQuota admission + status controller with MI355X GPU / HBM accounting (K7).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <memory>
#include <mutex>
#include <set>

#include "admission/admission.h"
#include "controllers/common.h"
#include "core/resources.h"
#include "core/util.h"
#include "node/node.h"

namespace kf {

std::map<std::string, double> pod_quota_usage(const Json& pod, int64_t hbm_gib_per_gpu) {
  std::map<std::string, double> use;
  use["pods"] = 1;
  use["count/pods"] = 1;
  auto acc = [&](const Json& list, bool init) {
    std::map<std::string, double> req, lim;
    for (const auto& c : list.as_array()) {
      std::map<std::string, double> r1, l1;
      for (const auto& m : c.at_path({"resources", "limits"}).as_object()) l1[m.first] = resource_value(m.first, m.second);
      for (const auto& m : c.at_path({"resources", "requests"}).as_object()) r1[m.first] = resource_value(m.first, m.second);
      for (auto& kv : l1)
        if (!r1.count(kv.first)) r1[kv.first] = kv.second;  // requests default to limits
      for (auto& kv : r1) req[kv.first] = init ? std::max(req[kv.first], kv.second) : req[kv.first] + kv.second;
      for (auto& kv : l1) lim[kv.first] = init ? std::max(lim[kv.first], kv.second) : lim[kv.first] + kv.second;
    }
    return std::make_pair(req, lim);
  };
  auto app = acc(pod.at_path({"spec", "containers"}), false);
  auto ini = acc(pod.at_path({"spec", "initContainers"}), true);
  for (auto* m : {&app.first, &ini.first})
    for (auto& kv : *m) use["requests." + kv.first] = std::max(use["requests." + kv.first], kv.second);
  for (auto* m : {&app.second, &ini.second})
    for (auto& kv : *m) use["limits." + kv.first] = std::max(use["limits." + kv.first], kv.second);
  // bare cpu / memory quota keys mean requests
  if (use.count("requests.cpu")) use["cpu"] = use["requests.cpu"];
  if (use.count("requests.memory")) use["memory"] = use["requests.memory"];
  // MI355X: GPUs and HBM, charged as the device plugin allocates them. The GPU count is the one
  // normalized count the scheduler and the device plugin use (core/resources.h); the device plugin
  // hands out whole GPUs, so a pod holds gpus x per-GPU HBM however little amd.com/gpu-memory it
  // states: the larger of the two is charged (a 300 GiB budget is one MI355X, not five).
  const std::string G = "amd.com/gpu", M = "amd.com/gpu-memory";
  auto counted = pod_gpu_count(pod, G);
  const double gpus = counted ? static_cast<double>(*counted) : use["requests." + G];
  if (gpus > 0)
    for (const std::string& k : {G, "requests." + G, "limits." + G}) use[k] = std::max(use[k], gpus);
  const double hbm = std::max(use.count("requests." + M) ? use["requests." + M] : 0.0, gpus * static_cast<double>(hbm_gib_per_gpu));
  if (hbm > 0)
    for (const std::string& k : {M, "requests." + M, "limits." + M}) use[k] = std::max(use[k], hbm);
  return use;
}

namespace {
// HBM per schedulable GPU as the nodes advertise it (capacity amd.com/gpu-memory / amd.com/gpu):
// 288 GiB on an SPX/NPS1 MI355X, a share of it per partition in CPX/NPS2 modes. The largest value
// across nodes is charged (conservative when nodes differ); `fallback` when no node has GPUs.
int64_t hbm_per_gpu(Client& c, int64_t fallback) {
  Json nodes;
  if (c.list("v1", "Node", "", ListOptions(), nodes)) return fallback;
  double best = 0;
  for (const auto& n : nodes["items"].as_array()) {
    const double g = resource_value(GPU_RESOURCE, n.at_path({"status", "capacity", GPU_RESOURCE}));
    const double m = resource_value(GPU_MEMORY_RESOURCE, n.at_path({"status", "capacity", GPU_MEMORY_RESOURCE}));
    if (g > 0 && m > 0) best = std::max(best, m / g);
  }
  return best > 0 ? static_cast<int64_t>(std::llround(best)) : fallback;
}

bool pod_counts(const Json& p) {
  const std::string& ph = p.at_path({"status", "phase"}).as_string();
  return ph != "Succeeded" && ph != "Failed" && !p.at_path({"metadata", "deletionTimestamp"}).is_string();
}
// amd.com/gpu-memory quota is expressed in GiB ("2304") or as a quantity ("2304Gi"); resource_value
// normalizes both to GiB
double hard_value(const std::string& key, const Json& q) { return resource_value(key, q); }
std::string fmt_num(double v) {
  char buf[64];
  if (std::fabs(v - std::round(v)) < 1e-9) std::snprintf(buf, sizeof buf, "%.0f", v);
  else std::snprintf(buf, sizeof buf, "%.3f", v);
  return buf;
}
}  // namespace

// Quota admission is check-then-commit, and the commit happens after admission returns. Two
// concurrent creates in one namespace would both see the same committed pods and both pass, so
// each admitted pod holds a reservation in this ledger from its check until it is visible in the
// store: the check and the reservation are one critical section per namespace, and the usage it
// checks against is committed pods + every other live reservation. A reservation ends when the
// request's completion hook fires (in-process API server: committed or not), when the pod shows
// up in the namespace's pod list (webhook mode, where no completion hook exists), or after
// kReservationTtl (a webhook-admitted create that the API server then failed).
// Reservations are keyed by the admission request (AdmissionReview uid, or a ledger sequence number
// in-process), never by pod name: kube-apiserver sends generateName creates (ReplicaSet / Job pods)
// with an EMPTY name, so name keys made concurrent generateName creates overwrite each other
// (ADVICE r2). Landing is matched by name when the request had one, otherwise by generateName: the
// oldest open reservation of that prefix claims one landed pod of the prefix that was NOT listed when
// the reservation was made (a landed pod claims at most one reservation, ever). Name sets rather than
// creationTimestamps (1 s resolution): a pod that landed just before the reservation, and was never
// claimed, could otherwise claim it and drop an in-flight pod's usage from the total.
// Reference quota semantics: profile-controller/controllers/profile_controller.go:559-589
// (the Profile's ResourceQuota) enforced by kube-apiserver's quota admission.
namespace {
constexpr double kReservationTtl = 30.0;

struct LandedPod {
  std::string name, generate_name;
};

struct QuotaLedger {
  struct Reservation {
    std::map<std::string, double> use;
    double expires = 0;
    std::string name, generate_name;
    std::set<std::string> existed;  // pods of generate_name listed at reserve time: never claim this one
    uint64_t seq = 0;
  };
  std::mutex mu;
  std::map<std::string, std::map<std::string, Reservation>> by_ns;  // ns -> request key -> usage
  std::map<std::string, std::set<std::string>> claimed;              // ns -> landed pods that ended one
  std::map<std::string, std::unique_ptr<std::mutex>> ns_locks;
  uint64_t next_seq = 0;

  std::mutex& ns_lock(const std::string& ns) {
    std::lock_guard<std::mutex> g(mu);
    auto& m = ns_locks[ns];
    if (!m) m = std::make_unique<std::mutex>();
    return *m;
  }
  // usage of ns's live reservations whose pod has not landed; drops expired and landed ones
  std::vector<std::map<std::string, double>> live(const std::string& ns, const std::vector<LandedPod>& pods) {
    std::lock_guard<std::mutex> g(mu);
    std::vector<std::map<std::string, double>> out;
    auto& cl = claimed[ns];
    {  // forget claims of pods that are gone (the set only needs the pods still listed)
      std::set<std::string> present;
      for (const auto& p : pods) present.insert(p.name);
      for (auto it = cl.begin(); it != cl.end();) it = present.count(*it) ? std::next(it) : cl.erase(it);
    }
    auto it = by_ns.find(ns);
    if (it == by_ns.end()) return out;
    const double now = now_seconds();
    std::vector<std::pair<uint64_t, std::string>> order;  // oldest reservation first
    for (const auto& r : it->second) order.push_back({r.second.seq, r.first});
    std::sort(order.begin(), order.end());
    for (const auto& o : order) {
      Reservation& r = it->second[o.second];
      bool landed = false;
      if (!r.name.empty()) {
        for (const auto& p : pods)
          if (p.name == r.name && !cl.count(p.name)) {
            landed = true;
            cl.insert(p.name);
            break;
          }
      } else if (!r.generate_name.empty()) {
        for (const auto& p : pods)
          if (p.generate_name == r.generate_name && !cl.count(p.name) && !r.existed.count(p.name)) {
            landed = true;
            cl.insert(p.name);
            break;
          }
      }
      if (landed || r.expires < now) it->second.erase(o.second);
      else out.push_back(r.use);
    }
    return out;
  }
  std::string reserve(const std::string& ns, const std::string& key_hint, const std::string& name,
                      const std::string& generate_name, std::map<std::string, double> use,
                      const std::vector<LandedPod>& listed) {
    std::lock_guard<std::mutex> g(mu);
    const uint64_t seq = ++next_seq;
    const std::string key = key_hint.empty() ? "seq:" + std::to_string(seq) : "uid:" + key_hint;
    Reservation r;
    r.use = std::move(use);
    r.expires = now_seconds() + kReservationTtl;
    r.name = name;
    r.generate_name = generate_name;
    if (!generate_name.empty())
      for (const auto& p : listed)
        if (p.generate_name == generate_name) r.existed.insert(p.name);
    r.seq = seq;
    by_ns[ns][key] = std::move(r);
    return key;
  }
  void release(const std::string& ns, const std::string& key) {
    std::lock_guard<std::mutex> g(mu);
    auto it = by_ns.find(ns);
    if (it != by_ns.end()) it->second.erase(key);
  }
  size_t open(const std::string& ns) {
    std::lock_guard<std::mutex> g(mu);
    auto it = by_ns.find(ns);
    return it == by_ns.end() ? 0 : it->second.size();
  }
};
}  // namespace

AdmissionFn make_quota_plugin(std::shared_ptr<Client> c, int64_t hbm) {
  auto ledger = std::make_shared<QuotaLedger>();
  return [c, hbm, ledger](AdmissionAttrs& a) -> ApiError {
    if (a.operation != "CREATE" || a.res->kind != "Pod" || !a.res->group.empty() || !a.object) return {};
    Json quotas;
    if (c->list("v1", "ResourceQuota", a.ns, ListOptions(), quotas)) return {};
    if (quotas["items"].empty()) return {};
    std::lock_guard<std::mutex> serial(ledger->ns_lock(a.ns));
    const int64_t hbm_dev = hbm_per_gpu(*c, hbm);
    Json pods;
    c->list("v1", "Pod", a.ns, ListOptions(), pods);
    std::map<std::string, double> used;
    std::vector<LandedPod> landed;
    for (const auto& p : pods["items"].as_array()) {
      LandedPod lp;
      lp.name = p.str_at({"metadata", "name"});
      lp.generate_name = p.str_at({"metadata", "generateName"});
      landed.push_back(std::move(lp));
      if (pod_counts(p))
        for (auto& kv : pod_quota_usage(p, hbm_dev)) used[kv.first] += kv.second;
    }
    for (const auto& r : ledger->live(a.ns, landed))
      for (const auto& kv : r) used[kv.first] += kv.second;
    auto want = pod_quota_usage(*a.object, hbm_dev);
    const std::string name = !a.name.empty() ? a.name : a.object->str_at({"metadata", "name"});
    for (const auto& q : quotas["items"].as_array()) {
      std::vector<std::string> exceeded;
      for (const auto& h : q.at_path({"spec", "hard"}).as_object()) {
        auto w = want.find(h.first);
        if (w == want.end() || w->second <= 0) continue;
        const double hard = hard_value(h.first, h.second);
        if (used[h.first] + w->second > hard + 1e-9)
          exceeded.push_back(h.first + "=" + fmt_num(w->second) + ", used: " + h.first + "=" + fmt_num(used[h.first]) +
                             ", limited: " + h.first + "=" + fmt_num(hard));
      }
      if (!exceeded.empty())
        return ApiError{403, "Forbidden", "pods \"" + name + "\" is forbidden: exceeded quota: " + q.str_at({"metadata", "name"}) +
                                              ", requested: " + join(exceeded, "; ")};
    }
    if (a.dry_run) return {};
    const std::string key = ledger->reserve(a.ns, a.uid, name, a.object->str_at({"metadata", "generateName"}),
                                            std::move(want), landed);
    const std::string ns = a.ns;
    // in-process: the pod is in the store (its list entry replaces the reservation) or never will be
    a.on_done.push_back([ledger, ns, key](bool) { ledger->release(ns, key); });
    return {};
  };
}

Result QuotaController::reconcile(const Request& r, std::string* err) {
  Json q;
  ApiError e = c_->get("v1", "ResourceQuota", r.ns, r.name, q);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  std::map<std::string, double> used;
  const int64_t hbm_dev = hbm_per_gpu(*c_, hbm_);
  pods_->visit(r.ns, [&](const Json& p) {
    if (pod_counts(p))
      for (auto& kv : pod_quota_usage(p, hbm_dev)) used[kv.first] += kv.second;
  });
  Json hard = q.at_path({"spec", "hard"});
  Json u = Json::object();
  for (const auto& h : hard.as_object()) u[h.first] = fmt_num(used[h.first]);
  Json status{{"hard", hard}, {"used", u}};
  if (q["status"] != status) {
    q["status"] = status;
    e = c_->update_status(q);
    if (e && e.code != 409) *err = e.message;
  }
  return {};
}

void QuotaController::setup(Manager& mgr) {
  pods_ = &mgr.informer("v1", "Pod");
  Informer& quotas = mgr.informer("v1", "ResourceQuota");
  ctl_ = std::make_shared<Controller>("resourcequota", [this](const Request& r, std::string* e) { return reconcile(r, e); });
  ctl_->For(quotas);
  ctl_->Watches(*pods_, [&quotas](const std::string&, const Json& p) {
    std::vector<Request> out;
    for (const auto& q : quotas.list(p.str_at({"metadata", "namespace"})))
      out.push_back({q.str_at({"metadata", "namespace"}), q.str_at({"metadata", "name"})});
    return out;
  });
  mgr.add(ctl_);
}

// ---- HTTP AdmissionReview server -----------------------------------------------------------------
void AdmissionWebhookServer::add(const std::string& path, AdmissionFn fn, bool mutating, std::shared_ptr<const ResourceInfo> res) {
  routes_[path] = Entry{std::move(fn), mutating, std::move(res)};
}

Json AdmissionWebhookServer::review(const std::string& path, const Json& ar) {
  const Json& req = ar["request"];
  Json resp{{"uid", req["uid"]}, {"allowed", true}};
  auto it = routes_.find(path);
  if (it == routes_.end()) {
    resp["allowed"] = false;
    resp["status"] = Json{{"code", 404}, {"message", "no admission handler at " + path}};
  } else {
    AdmissionAttrs a;
    a.operation = req["operation"].as_string();
    a.res = it->second.res;
    a.subresource = req["subResource"].as_string();
    a.ns = req["namespace"].as_string();
    a.name = req["name"].as_string();
    a.uid = req["uid"].as_string();
    a.version = req.at_path({"kind", "version"}).as_string();
    Json obj = req["object"];
    Json old = req["oldObject"];
    UserInfo u;
    u.username = req.at_path({"userInfo", "username"}).as_string();
    a.object = obj.is_null() ? nullptr : &obj;
    a.old_object = old.is_null() ? nullptr : &old;
    a.user = &u;
    a.dry_run = req["dryRun"].as_bool();
    ApiError e = it->second.fn(a);
    if (e) {
      resp["allowed"] = false;
      resp["status"] = Json{{"code", e.code}, {"message", e.message}, {"reason", e.reason}};
    } else if (it->second.mutating && !req["object"].is_null()) {
      Json patch = diff_json_patch(req["object"], obj);
      if (!patch.empty()) {
        resp["patch"] = base64_encode(patch.dump());
        resp["patchType"] = "JSONPatch";
      }
    }
  }
  return Json{{"apiVersion", "admission.k8s.io/v1"}, {"kind", "AdmissionReview"}, {"response", resp}};
}

std::vector<Json> AdmissionWebhookServer::webhook_configurations(const std::string& base_url, const std::string& name,
                                                                 const std::string& ca_pem) const {
  Json mut = Json::array(), val = Json::array();
  for (const auto& kv : routes_) {
    const auto& res = kv.second.res;
    if (!res) continue;
    Json versions = Json::array();
    for (const auto& v : res->versions) versions.push_back(v);
    std::string hook = kv.first.substr(1);
    for (auto& ch : hook)
      if (ch == '/') ch = '-';
    Json wh{{"name", hook + "." + name + ".kfamd.io"},
            {"clientConfig", Json{{"url", base_url + kv.first}}},
            {"rules", Json::array({Json{{"apiGroups", Json::array({res->group})},
                                        {"apiVersions", versions},
                                        {"operations", Json::array({"CREATE", "UPDATE"})},
                                        {"resources", Json::array({res->plural})}}})},
            {"failurePolicy", "Fail"},
            {"sideEffects", "None"},
            {"admissionReviewVersions", Json::array({"v1"})}};
    if (!ca_pem.empty()) wh["clientConfig"]["caBundle"] = base64_encode(ca_pem);
    if (res->kind == "Pod" && kv.first == "/apply-poddefault")
      wh["namespaceSelector"] = Json{{"matchLabels", Json{{"app.kubernetes.io/part-of", "kubeflow-profile"}}}};
    (kv.second.mutating ? mut : val).push_back(wh);
  }
  std::vector<Json> out;
  if (!mut.empty())
    out.push_back(Json{{"apiVersion", "admissionregistration.k8s.io/v1"}, {"kind", "MutatingWebhookConfiguration"},
                       {"metadata", Json{{"name", name}}}, {"webhooks", mut}});
  if (!val.empty())
    out.push_back(Json{{"apiVersion", "admissionregistration.k8s.io/v1"}, {"kind", "ValidatingWebhookConfiguration"},
                       {"metadata", Json{{"name", name}}}, {"webhooks", val}});
  return out;
}

bool AdmissionWebhookServer::start(const std::string& addr, int port, std::string* err, const TlsServerConfig* tls) {
  srv_ = std::make_unique<HttpServer>();
  if (tls && !srv_->enable_tls(*tls, err)) return false;
  if (!srv_->listen(addr, port, err)) return false;
  srv_->set_handler([this](HttpRequest& req, HttpResponse& resp) {
    if (req.path == "/healthz" || req.path == "/readyz") {
      resp.text(200, "ok");
      return;
    }
    Json ar;
    if (req.method != "POST" || !Json::try_parse(req.body, ar)) {
      resp.json(400, R"({"error":"expected an AdmissionReview"})");
      return;
    }
    resp.json(200, review(req.path, ar).dump());
  });
  srv_->start();
  return true;
}

void AdmissionWebhookServer::stop() {
  if (srv_) srv_->stop();
}

}  // namespace kf
