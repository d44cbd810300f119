// culling.cc — N3 CullingReconciler (reference notebook-controller/controllers/culling_controller.go).
//
// Every IDLENESS_CHECK_PERIOD the culler GETs the Jupyter /api/kernels and /api/terminals of the
// notebook (through its Service, resolved by the embedded API server, or through the API server's
// service proxy in DEV mode), maintains notebooks.kubeflow.org/last-activity (never moving it
// backwards) and sets kubeflow-resource-stopped once idle for CULL_IDLE_TIME minutes.
// Q2 deviation: the reference never emits notebook_culling_total / last_notebook_culling_timestamp
// (the CullingReconciler is built without Metrics); here they are emitted.
#include <algorithm>

#include "controllers/notebook.h"
#include "core/util.h"

namespace kf {

CullingOptions CullingOptions::from_env() {
  CullingOptions o;
  const std::string idle = getenv_or("CULL_IDLE_TIME", "1440");
  char* end = nullptr;
  long v = std::strtol(idle.c_str(), &end, 10);
  o.cull_idle_minutes = (end && *end == 0 && !idle.empty()) ? v : 1440;
  const std::string per = getenv_or("IDLENESS_CHECK_PERIOD", "1");
  long p = std::strtol(per.c_str(), &end, 10);
  o.check_period_minutes = (end && *end == 0 && !per.empty()) ? p : 1;
  o.dev = getenv_or("DEV", "false") != "false";
  o.proxy_url = getenv_or("KUBE_PROXY_URL", "http://localhost:8001");
  o.cluster_domain = getenv_or("CLUSTER_DOMAIN", "cluster.local");
  o.mesh_url = getenv_or("MESH_URL", "");
  o.mesh_token_file = getenv_or("MESH_TOKEN_FILE", "/var/run/secrets/kubernetes.io/serviceaccount/token");
  const std::string ps = getenv_or("IDLENESS_CHECK_PERIOD_SECONDS", "");
  if (!ps.empty()) o.period_seconds_override = std::atof(ps.c_str());
  return o;
}

bool all_kernels_are_idle(const Json& kernels) {
  for (const auto& k : kernels.as_array())
    if (k["execution_state"].as_string() != "idle") return false;
  return true;
}

std::string notebook_recent_time(const std::vector<std::string>& times) {
  if (times.empty()) return "";
  auto first = parse_rfc3339_ms(times[0]);
  if (!first) return "";
  int64_t best = *first;
  for (size_t i = 1; i < times.size(); ++i) {
    auto t = parse_rfc3339_ms(times[i]);
    if (!t) return "";
    best = std::max(best, *t);
  }
  return rfc3339_from_ms(best);
}

namespace {
// compareAnnotationTimeToResource: false when the annotation is newer than the resource time
bool resource_not_older(const Json& ann, const std::string& resource_time) {
  auto a = parse_rfc3339_ms(ann[LAST_ACTIVITY_ANNOTATION].as_string());
  auto t = parse_rfc3339_ms(resource_time);
  if (!a || !t) return false;
  // RFC3339 second precision, like time.Parse(RFC3339) + After()
  return !(*a / 1000 > *t / 1000);
}
}  // namespace

bool update_timestamp_from_kernels_activity(Json& ann, const Json& kernels) {
  if (!kernels.is_array() || kernels.empty()) return false;
  if (!all_kernels_are_idle(kernels)) {
    ann[LAST_ACTIVITY_ANNOTATION] = rfc3339_now();  // a busy kernel means activity now
    return false;
  }
  std::vector<std::string> arr;
  for (const auto& k : kernels.as_array()) arr.push_back(k["last_activity"].as_string());
  std::string t = notebook_recent_time(arr);
  if (t.empty() || !resource_not_older(ann, t)) return false;
  ann[LAST_ACTIVITY_ANNOTATION] = t;
  return true;
}

bool update_timestamp_from_terminals_activity(Json& ann, const Json& terminals) {
  if (!terminals.is_array() || terminals.empty()) return false;
  std::vector<std::string> arr;
  for (const auto& k : terminals.as_array()) arr.push_back(k["last_activity"].as_string());
  std::string t = notebook_recent_time(arr);
  if (t.empty() || !resource_not_older(ann, t)) return false;
  ann[LAST_ACTIVITY_ANNOTATION] = t;
  return true;
}

bool notebook_is_idle(const Json& nb, int64_t cull_idle_minutes, int64_t now_ms) {
  if (stop_annotation_is_set(nb)) return false;
  auto last = parse_rfc3339_ms(annotation(nb, LAST_ACTIVITY_ANNOTATION));
  if (!last) return false;
  return now_ms > *last + cull_idle_minutes * 60000;
}

bool culling_check_period_has_passed(const Json& nb, double period_s, int64_t now_ms) {
  if (!has_annotation(nb, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION)) return false;
  auto stored = parse_rfc3339_ms(annotation(nb, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION));
  int64_t base = stored ? *stored : 0;  // Go's zero time on parse error -> always passed
  return base + static_cast<int64_t>(period_s * 1000) < now_ms;
}

void set_stop_annotation(Json& nb, NotebookMetrics* m) {
  const int64_t now = now_unix_ms();
  set_annotation(nb, STOP_ANNOTATION, rfc3339_from_ms(now));
  if (m) {
    Labels l{nb.str_at({"metadata", "namespace"}), nb.str_at({"metadata", "name"})};
    m->culling_total->inc(l);
    m->last_culling_timestamp->set(l, static_cast<double>(now / 1000));
  }
}

CullingReconciler::CullingReconciler(std::shared_ptr<Client> c, CullingOptions o, std::shared_ptr<NotebookMetrics> m)
    : c_(std::move(c)), o_(std::move(o)), m_(std::move(m)) {}

bool CullingReconciler::fetch(const std::string& nm, const std::string& ns, const std::string& what, Json& out) {
  std::string url = "http://" + nm + "." + ns + ".svc." + o_.cluster_domain + "/notebook/" + ns + "/" + nm + "/api/" + what;
  if (o_.dev)
    url = o_.proxy_url + "/api/v1/namespaces/" + ns + "/services/" + nm + ":http-" + nm + "/proxy/notebook/" + ns + "/" + nm +
          "/api/" + what;
  Headers h;
  const std::string mesh = o_.mesh_url_fn ? o_.mesh_url_fn() : o_.mesh_url;
  // through the mesh (with the culler's workload identity) only into mesh members: in any other
  // namespace the reference's plain GET comes from the controller's own namespace, which is what
  // ODH's <nb>-ctrl-np admits on :8888
  bool member = false;
  if (!o_.dev && !mesh.empty()) {
    Json n;
    member = !c_->get("v1", "Namespace", "", ns, n) && n.at_path({"metadata", "labels", "istio-injection"}).as_string() == "enabled";
  }
  if (member) {
    h["Host"] = nm + "." + ns + ".svc." + o_.cluster_domain;
    std::string token;
    if (o_.peer_token_fn) token = o_.peer_token_fn();
    else if (read_file(o_.mesh_token_file, token)) token = trim(token);
    if (!token.empty()) h["X-Kfamd-Peer-Token"] = token;
    url = mesh + "/notebook/" + ns + "/" + nm + "/api/" + what;
  }
  HttpResult r = http_request("GET", url, "", h, 10000);
  if (r.status != 200) {
    KF_INFO("culler", "Warning: GET to " + url + ": " + (r.status ? std::to_string(r.status) : r.error));
    return false;
  }
  if (!Json::try_parse(r.body, out) || !out.is_array()) {
    KF_ERROR("culler", "Error parsing JSON response for Notebook API " + what);
    return false;
  }
  return true;
}

Result CullingReconciler::reconcile(const Request& req, std::string* err) {
  Json nb;
  ApiError e = c_->get("kubeflow.org/v1beta1", "Notebook", req.ns, req.name, nb);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  auto remove_annotations = [](Json& o) {
    bool changed = o["metadata"]["annotations"].erase(LAST_ACTIVITY_ANNOTATION);
    changed = o["metadata"]["annotations"].erase(LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION) || changed;
    return changed;
  };
  if (stop_annotation_is_set(nb)) {
    if (remove_annotations(nb)) {
      e = c_->update(nb);
      if (e) *err = e.message;
    }
    return {};
  }
  Json pod;
  e = c_->get("v1", "Pod", req.ns, req.name + "-0", pod);
  if (e.code == 404) {
    if (remove_annotations(nb)) {
      e = c_->update(nb);
      if (e) *err = e.message;
    }
    return {};
  }
  if (e) {
    *err = e.message;
    return {};
  }
  if (!has_annotation(nb, LAST_ACTIVITY_ANNOTATION) || !has_annotation(nb, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION)) {
    const std::string t = rfc3339_now();
    set_annotation(nb, LAST_ACTIVITY_ANNOTATION, t);
    set_annotation(nb, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION, t);
    e = c_->update(nb);
    if (e) {
      *err = e.message;
      return {};
    }
  }
  const int64_t now = now_unix_ms();
  if (!culling_check_period_has_passed(nb, o_.period_seconds(), now)) return Result::after(o_.period_seconds());

  Json kernels, terminals;
  bool have_k = fetch(req.name, req.ns, "kernels", kernels);
  bool have_t = fetch(req.name, req.ns, "terminals", terminals);
  Json& ann = nb["metadata"]["annotations"];
  if (have_k || have_t) {
    if (have_k) update_timestamp_from_kernels_activity(ann, kernels);
    if (have_t) update_timestamp_from_terminals_activity(ann, terminals);
  }
  ann[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION] = rfc3339_now();
  e = c_->update(nb);
  if (e) {
    *err = e.message;
    return {};
  }
  if (notebook_is_idle(nb, o_.cull_idle_minutes, now_unix_ms())) {
    KF_INFO("culler", "Notebook " + req.str() + " needs culling. Updating Notebook CR Annotations...");
    set_stop_annotation(nb, m_.get());
    e = c_->update(nb);
    if (e) {
      *err = e.message;
      return {};
    }
  }
  return Result::after(o_.period_seconds());
}

void CullingReconciler::setup(Manager& mgr) {
  ctl_ = std::make_shared<Controller>("Culler", [this](const Request& r, std::string* err) { return reconcile(r, err); });
  ctl_->For(mgr.informer("kubeflow.org/v1beta1", "Notebook"));
  mgr.add(ctl_);
}

}  // namespace kf
