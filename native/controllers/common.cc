// common.cc — see common.h.
#include "controllers/common.h"

#include <map>

#include "core/util.h"

namespace kf {

bool stop_annotation_is_set(const Json& obj) { return has_annotation(obj, STOP_ANNOTATION); }

namespace {
// "for k, v := range to.Labels { if from.Labels[k] != v {update} }; to.Labels = from.Labels"
bool copy_map_field(const Json& from, Json& to, const char* field) {
  bool update = false;
  const Json& f = from.at_path({"metadata", field});
  const Json& t = to.at_path({"metadata", field});
  for (const auto& m : t.as_object()) {
    const Json* fv = f.find(m.first);
    if (!fv || *fv != m.second) update = true;
  }
  if (f.is_object() && !f.empty()) to["metadata"][field] = f;
  else to["metadata"].erase(field);
  return update;
}
}  // namespace

bool copy_statefulset_fields(const Json& from, Json& to) {
  bool update = copy_map_field(from, to, "labels");
  update = copy_map_field(from, to, "annotations") || update;
  if (from.at_path({"spec", "replicas"}).as_int(1) != to.at_path({"spec", "replicas"}).as_int(1)) {
    to["spec"]["replicas"] = from.at_path({"spec", "replicas"});
    update = true;
  }
  if (to.at_path({"spec", "template", "spec"}) != from.at_path({"spec", "template", "spec"})) update = true;
  to["spec"]["template"]["spec"] = from.at_path({"spec", "template", "spec"});
  return update;
}

bool copy_deployment_fields(const Json& from, Json& to) {
  bool update = copy_map_field(from, to, "labels");
  update = copy_map_field(from, to, "annotations") || update;
  if (from.at_path({"spec", "replicas"}).as_int(1) != to.at_path({"spec", "replicas"}).as_int(1)) {
    to["spec"]["replicas"] = from.at_path({"spec", "replicas"});
    update = true;
  }
  if (to.at_path({"spec", "template", "spec"}) != from.at_path({"spec", "template", "spec"})) update = true;
  to["spec"]["template"]["spec"] = from.at_path({"spec", "template", "spec"});
  return update;
}

bool copy_service_fields(const Json& from, Json& to) {
  bool update = copy_map_field(from, to, "labels");
  update = copy_map_field(from, to, "annotations") || update;
  if (to.at_path({"spec", "selector"}) != from.at_path({"spec", "selector"})) update = true;
  to["spec"]["selector"] = from.at_path({"spec", "selector"});
  // compare ports after normalising the defaulted fields the API server fills in
  Json fp = from.at_path({"spec", "ports"});
  for (auto& p : fp.mut_array()) {
    if (!p.has("protocol")) p["protocol"] = "TCP";
    if (!p.has("targetPort")) p["targetPort"] = p["port"];
  }
  if (to.at_path({"spec", "ports"}) != fp) update = true;
  to["spec"]["ports"] = fp;
  return update;
}

bool copy_virtual_service(const Json& from, Json& to) {
  const Json* fs = from.find("spec");
  if (!fs) return false;
  if (!to.has("spec")) {
    to["spec"] = *fs;
    return true;
  }
  if (to["spec"] != *fs) {
    to["spec"] = *fs;
    return true;
  }
  return false;
}

ApiError reconcile_owned(Client& c, const Json& desired, CopyKind kind, Json* live, bool* created) {
  const std::string av = desired["apiVersion"].as_string(), k = desired["kind"].as_string();
  const std::string ns = desired.str_at({"metadata", "namespace"}), name = desired.str_at({"metadata", "name"});
  Json found;
  ApiError e = c.get(av, k, ns, name, found);
  if (created) *created = false;
  if (e.code == 404) {
    Json obj = desired;
    e = c.create(obj);
    if (!e) {
      if (live) *live = obj;
      if (created) *created = true;
    }
    return e;
  }
  if (e) return e;
  bool need = false;
  switch (kind) {
    case CopyKind::StatefulSet: need = copy_statefulset_fields(desired, found); break;
    case CopyKind::Deployment: need = copy_deployment_fields(desired, found); break;
    case CopyKind::Service: need = copy_service_fields(desired, found); break;
    case CopyKind::VirtualService: need = copy_virtual_service(desired, found); break;
    case CopyKind::Generic:
      for (const auto& m : desired.as_object()) {
        if (m.first == "metadata" || m.first == "status" || m.first == "apiVersion" || m.first == "kind") continue;
        if (found.get(m.first) != m.second) {
          found[m.first] = m.second;
          need = true;
        }
      }
      need = copy_map_field(desired, found, "labels") || need;
      break;
  }
  if (need) e = c.update(found);
  if (!e && live) *live = found;
  return e;
}

std::shared_ptr<NotebookMetrics> NotebookMetrics::install(std::shared_ptr<Client> c) {
  auto m = std::make_shared<NotebookMetrics>();
  auto& reg = Registry::global();
  m->create_total = reg.counter("notebook_create_total", "Total times of creating notebooks", {"namespace"});
  m->create_failed_total = reg.counter("notebook_create_failed_total", "Total failure times of creating notebooks", {"namespace"});
  m->culling_total = reg.counter("notebook_culling_total", "Total times of culling notebooks", {"namespace", "name"});
  m->last_culling_timestamp = reg.gauge("last_notebook_culling_timestamp_seconds", "Timestamp of the last notebook culling in seconds",
                                        {"namespace", "name"});
  m->cold_start_seconds = reg.histogram(
      "notebook_cold_start_seconds",
      "Notebook first start by phase: observed->statefulset, statefulset->scheduled, scheduled->initialized "
      "(in-pod GPU readiness op), initialized->ready, total (observed->notebook ready)",
      {"phase"}, HistogramVec::exponential(0.001, 2, 18));
  reg.add_collector(std::make_shared<CollectorFamily>(
      "notebook_running", "Current running notebooks in the cluster", "gauge", std::vector<std::string>{"namespace"},
      [c]() {
        std::vector<std::pair<Labels, double>> out;
        Json lst;
        if (c->list("apps/v1", "StatefulSet", "", ListOptions(), lst)) return out;
        std::map<std::string, double> per_ns;
        for (const auto& sts : lst["items"].as_array()) {
          if (sts.at_path({"spec", "template", "metadata", "labels", "notebook-name"}).as_string() ==
              sts.str_at({"metadata", "name"}))
            per_ns[sts.str_at({"metadata", "namespace"})] += 1;
        }
        for (auto& kv : per_ns) out.push_back({{kv.first}, kv.second});
        return out;
      }));
  return m;
}

}  // namespace kf
