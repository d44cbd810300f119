// tensorboard.cc — N16 Tensorboard reconciler + N17 PVCViewer (see tensorboard.h).
#include "controllers/tensorboard.h"

#include "controllers/common.h"
#include "core/util.h"
#include "core/yaml.h"

namespace kf {

// ---- Tensorboard helpers ---------------------------------------------------------------------
bool tb_is_gcs_path(const std::string& p) { return starts_with(p, "gs://"); }
bool tb_is_cloud_path(const std::string& p) { return tb_is_gcs_path(p) || starts_with(p, "s3://") || starts_with(p, "/cns/"); }
bool tb_is_pvc_path(const std::string& p) { return starts_with(p, "pvc://"); }
std::string tb_extract_pvc_name(const std::string& p) {
  std::string t = starts_with(p, "pvc://") ? p.substr(6) : p;
  size_t e = t.find('/');
  return e == std::string::npos ? t : t.substr(0, e);
}
std::string tb_extract_pvc_subpath(const std::string& p) {
  std::string t = starts_with(p, "pvc://") ? p.substr(6) : p;
  size_t s = t.find('/');
  if (s == std::string::npos || t.size() == s + 1) return "";
  return t.substr(s + 1);
}

Json preferred_node_affinity(const std::string& node) {
  if (node.empty()) return Json::object();
  return Json{{"nodeAffinity",
               Json{{"preferredDuringSchedulingIgnoredDuringExecution",
                     Json::array({Json{{"weight", 100},
                                       {"preference", Json{{"matchExpressions",
                                                            Json::array({Json{{"key", "kubernetes.io/hostname"},
                                                                              {"operator", "In"},
                                                                              {"values", Json::array({node})}}})}}}}})}}}};
}

Json tb_generate_deployment(const Json& tb, const std::string& image, const Json& affinity) {
  const std::string name = tb.str_at({"metadata", "name"});
  const std::string ns = tb.str_at({"metadata", "namespace"});
  const std::string logs = tb.at_path({"spec", "logspath"}).as_string();
  std::string mountpath = logs, subpath;
  Json mounts = Json::array(), volumes = Json::array();
  if (!tb_is_cloud_path(logs)) {
    std::string pvc;
    if (tb_is_pvc_path(logs)) {
      pvc = tb_extract_pvc_name(logs);
      mountpath = "/tensorboard_logs/";
      subpath = tb_extract_pvc_subpath(logs);
    } else {
      pvc = "tb-volume";
    }
    Json m{{"name", "tbpd"}, {"readOnly", true}, {"mountPath", mountpath}};
    if (!subpath.empty()) m["subPath"] = subpath;
    mounts.push_back(m);
    volumes.push_back(Json{{"name", "tbpd"}, {"persistentVolumeClaim", Json{{"claimName", pvc}}}});
  } else if (tb_is_gcs_path(logs)) {
    mounts.push_back(Json{{"name", "gcp-creds"}, {"readOnly", true}, {"mountPath", "/secret/gcp"}});
    volumes.push_back(Json{{"name", "gcp-creds"}, {"secret", Json{{"secretName", "user-gcp-sa"}}}});
  }
  Json labels = tb.at_path({"metadata", "labels"}).is_object() ? tb.at_path({"metadata", "labels"}) : Json::object();
  labels["app"] = name;
  Json container{{"name", "tensorboard"},
                 {"image", image},
                 {"imagePullPolicy", "IfNotPresent"},
                 {"command", Json::array({"/usr/local/bin/tensorboard"})},
                 {"workingDir", "/"},
                 {"args", Json::array({"--logdir=" + mountpath, "--bind_all"})},
                 {"ports", Json::array({Json{{"containerPort", 6006}}})}};
  if (!mounts.empty()) container["volumeMounts"] = mounts;
  Json pod_spec{{"affinity", affinity.is_object() ? affinity : Json::object()},
                {"restartPolicy", "Always"},
                {"containers", Json::array({container})}};
  if (!volumes.empty()) pod_spec["volumes"] = volumes;
  return Json{{"apiVersion", "apps/v1"},
              {"kind", "Deployment"},
              {"metadata", Json{{"name", name}, {"namespace", ns}}},
              {"spec", Json{{"replicas", 1},
                            {"selector", Json{{"matchLabels", Json{{"app", name}}}}},
                            {"template", Json{{"metadata", Json{{"labels", labels}}}, {"spec", pod_spec}}}}}};
}

Json tb_generate_service(const Json& tb) {
  const std::string name = tb.str_at({"metadata", "name"});
  return Json{{"apiVersion", "v1"},
              {"kind", "Service"},
              {"metadata", Json{{"name", name}, {"namespace", tb.str_at({"metadata", "namespace"})}}},
              {"spec", Json{{"type", "ClusterIP"},
                            {"selector", Json{{"app", name}}},
                            {"ports", Json::array({Json{{"name", "http-" + name}, {"port", 80}, {"targetPort", 6006}}})}}}};
}

Json tb_generate_virtual_service(const Json& tb, const std::string& gateway, const std::string& host) {
  const std::string name = tb.str_at({"metadata", "name"});
  const std::string ns = tb.str_at({"metadata", "namespace"});
  Json http{{"match", Json::array({Json{{"uri", Json{{"prefix", "/tensorboard/" + ns + "/" + name + "/"}}}}})},
            {"rewrite", Json{{"uri", "/"}}},
            {"route", Json::array({Json{{"destination", Json{{"host", name + "." + ns + ".svc.cluster.local"},
                                                             {"port", Json{{"number", 80}}}}}}})},
            {"timeout", "300s"}};
  return Json{{"apiVersion", "networking.istio.io/v1alpha3"},
              {"kind", "VirtualService"},
              {"metadata", Json{{"name", name}, {"namespace", ns}}},
              {"spec", Json{{"hosts", Json::array({host})}, {"gateways", Json::array({gateway})}, {"http", Json::array({http})}}}};
}

bool tb_copy_deployment_fields(const Json& from, Json& to) {
  bool update = false;
  const Json& fl = from.at_path({"metadata", "labels"});
  for (const auto& kv : to.at_path({"metadata", "labels"}).as_object())
    if (fl[kv.first] != kv.second) update = true;
  if (fl.is_object()) to["metadata"]["labels"] = fl;
  else to["metadata"].erase("labels");
  if (from.at_path({"spec", "replicas"}) != to.at_path({"spec", "replicas"})) {
    to["spec"]["replicas"] = from.at_path({"spec", "replicas"});
    update = true;
  }
  const Json& fa = from.at_path({"spec", "template", "spec", "affinity"});
  const Json& ta = to.at_path({"spec", "template", "spec", "affinity"});
  // an empty affinity object and an absent one are the same thing after a round trip
  auto norm = [](const Json& a) { return a.is_object() && !a.empty() ? a : Json(); };
  if (norm(fa) != norm(ta)) update = true;
  to["spec"]["template"]["spec"]["affinity"] = fa.is_object() ? fa : Json::object();
  return update;
}

Json tb_status(const Json& tb, const Json& dep) {
  Json st = tb["status"].is_object() ? tb["status"] : Json::object();
  if (!st["conditions"].is_array()) st["conditions"] = Json::array();
  const Json& dc = dep.at_path({"status", "conditions"});
  if (dc.is_array() && !dc.empty()) {
    Json cond{{"deploymentState", dc[0]["type"]}, {"lastProbeTime", dc[0]["lastUpdateTime"]}};
    const auto& cs = st["conditions"].as_array();
    if (cs.empty() || cs.back()["deploymentState"] != cond["deploymentState"]) st["conditions"].push_back(cond);
  }
  st["readyReplicas"] = dep.at_path({"status", "readyReplicas"}).as_int(0);
  return st;
}

TensorboardOptions TensorboardOptions::from_env(std::string* err) {
  TensorboardOptions o;
  o.image = getenv_or("TENSORBOARD_IMAGE", o.image);
  o.istio_gateway = getenv_or("ISTIO_GATEWAY", o.istio_gateway);
  o.istio_host = getenv_or("ISTIO_HOST", o.istio_host);
  const std::string rwo = getenv_or("RWO_PVC_SCHEDULING", "false");
  if (rwo == "true" || rwo == "True" || rwo == "TRUE") o.rwo_pvc_scheduling = true;
  else if (!(rwo == "false" || rwo == "False" || rwo == "FALSE") && err) *err = "Invalid value for 'RWO_PVC_SCEDULING' env var.";
  return o;
}

Json TensorboardReconciler::node_affinity_for_pvc(const std::string& ns, const std::string& pvc_name, std::string* err) {
  Json pvc;
  ApiError e = c_->get("v1", "PersistentVolumeClaim", ns, pvc_name, pvc);
  if (e) {
    *err = "Get PersistentVolumeClaim error: " + e.message;
    return Json();
  }
  const Json& am = pvc.at_path({"status", "accessModes"});
  if (!am.is_array() || am.empty() || am[0].as_string() != "ReadWriteOnce") return Json::object();
  // field index spec.volumes.persistentvolumeclaim.claimname -> first Running pod's node
  for (const auto& p : pods_->by_index("pvc", ns + "/" + pvc_name))
    if (p.at_path({"status", "phase"}).as_string() == "Running") return preferred_node_affinity(p.at_path({"spec", "nodeName"}).as_string());
  return Json::object();
}

Result TensorboardReconciler::reconcile(const Request& r, std::string* err) {
  Json tb;
  ApiError e = c_->get("tensorboard.kubeflow.org/v1alpha1", "Tensorboard", r.ns, r.name, tb);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  // the web app deletes with foreground propagation: do nothing while terminating
  if (tb.at_path({"metadata", "deletionTimestamp"}).is_string()) return {};
  Json affinity = Json::object();
  const std::string logs = tb.at_path({"spec", "logspath"}).as_string();
  if (!tb_is_cloud_path(logs) && o_.rwo_pvc_scheduling) {
    const std::string pvc = tb_is_pvc_path(logs) ? tb_extract_pvc_name(logs) : "tb-volume";
    affinity = node_affinity_for_pvc(r.ns, pvc, err);
    if (!err->empty()) return {};
  }
  Json dep = tb_generate_deployment(tb, o_.image, affinity);
  set_controller_reference(tb, dep);
  Json found;
  e = c_->get("apps/v1", "Deployment", r.ns, r.name, found);
  if (e.code == 404) {
    KF_INFO("tensorboard-controller", "Creating Deployment", Json{{"namespace", r.ns}, {"name", r.name}});
    Json d = dep;
    e = c_->create(d);
    if (e) {
      *err = "unable to create deployment: " + e.message;
      return {};
    }
  } else if (e) {
    *err = e.message;
    return {};
  } else if (tb_copy_deployment_fields(dep, found)) {
    KF_INFO("tensorboard-controller", "Updating Deployment", Json{{"namespace", r.ns}, {"name", r.name}});
    e = c_->update(found);
    if (e) {
      *err = "unable to update deployment: " + e.message;
      return {};
    }
  }
  Json svc = tb_generate_service(tb);
  set_controller_reference(tb, svc);
  if ((e = reconcile_owned(*c_, svc, CopyKind::Service))) {
    *err = e.message;
    return {};
  }
  Json vs = tb_generate_virtual_service(tb, o_.istio_gateway, o_.istio_host);
  set_controller_reference(tb, vs);
  if ((e = reconcile_owned(*c_, vs, CopyKind::VirtualService))) {
    *err = e.message;
    return {};
  }
  Json live;
  if (!c_->get("apps/v1", "Deployment", r.ns, r.name, live)) {
    Json st = tb_status(tb, live);
    if (st != tb["status"]) {
      tb["status"] = st;
      e = c_->update_status(tb);
      if (e) *err = e.message;
    }
  }
  return {};
}

void TensorboardReconciler::setup(Manager& mgr, int workers) {
  pods_ = &mgr.informer("v1", "Pod");
  pods_->add_index("pvc", [](const Json& p) {
    std::vector<std::string> out;
    const std::string ns = p.str_at({"metadata", "namespace"});
    for (const auto& v : p.at_path({"spec", "volumes"}).as_array()) {
      const Json& pvc = v["persistentVolumeClaim"];
      if (pvc.is_object()) out.push_back(ns + "/" + pvc["claimName"].as_string());
    }
    return out;
  });
  ctl_ = std::make_shared<Controller>("tensorboard-controller", [this](const Request& r, std::string* e) { return reconcile(r, e); },
                                      workers);
  ctl_->For(mgr.informer("tensorboard.kubeflow.org/v1alpha1", "Tensorboard"));
  ctl_->Owns(mgr.informer("apps/v1", "Deployment"), "Tensorboard");
  mgr.add(ctl_);
}

// ---- PVCViewer ---------------------------------------------------------------------------------
Json pvcviewer_default(const Json& viewer, const Json& default_pod_spec) {
  Json v = viewer;
  const Json& ps = v.at_path({"spec", "podSpec"});
  if (ps.is_object() && !ps.empty()) return v;
  const std::string name = v.str_at({"metadata", "name"});
  const std::string ns = v.str_at({"metadata", "namespace"});
  Json spec;
  if (default_pod_spec.is_object() && !default_pod_spec.empty()) {
    spec = default_pod_spec;
  } else {
    const std::string base = v.at_path({"spec", "networking", "basePrefix"}).as_string();
    Json env = Json::array({Json{{"name", "FB_ADDRESS"}, {"value", "0.0.0.0"}}, Json{{"name", "FB_PORT"}, {"value", "8080"}},
                            Json{{"name", "FB_DATABASE"}, {"value", "/tmp/filebrowser.db"}},
                            Json{{"name", "FB_NOAUTH"}, {"value", "true"}},
                            Json{{"name", "FB_BASEURL"}, {"value", base + "/" + ns + "/" + name + "/"}}});
    spec = Json{{"containers", Json::array({Json{{"name", "pvcviewer"},
                                                 {"image", "filebrowser/filebrowser:latest"},
                                                 {"ports", Json::array({Json{{"containerPort", 8080}, {"protocol", "TCP"}}})},
                                                 {"env", env},
                                                 {"workingDir", "/data"},
                                                 {"volumeMounts", Json::array({Json{{"name", "viewer-volume"}, {"mountPath", "/data"}}})}}})}};
  }
  spec["volumes"].push_back(Json{{"name", "viewer-volume"},
                                 {"persistentVolumeClaim", Json{{"claimName", v.at_path({"spec", "pvc"}).as_string()}}}});
  v["spec"]["podSpec"] = spec;
  return v;
}

std::string pvcviewer_validate(const Json& viewer) {
  const std::string pvc = viewer.at_path({"spec", "pvc"}).as_string();
  if (pvc.empty()) return "PVC name must be specified";
  const Json& ps = viewer.at_path({"spec", "podSpec"});
  if (!ps.is_object() || ps.empty()) return "PodSpec must be specified";
  for (const auto& v : ps["volumes"].as_array())
    if (v.at_path({"persistentVolumeClaim", "claimName"}).as_string() == pvc) return "";
  return "PVC " + pvc + " must be used in the podSpec";
}

Json pvcviewer_common_labels(const Json& viewer) {
  const std::string name = viewer.str_at({"metadata", "name"});
  return Json{{"app.kubernetes.io/name", name},
              {"app.kubernetes.io/instance", std::string(PVCVIEWER_PREFIX) + name},
              {"app.kubernetes.io/part-of", "pvc-viewer"}};
}

Json pvcviewer_generate_deployment(const Json& viewer, const Json& affinity) {
  Json labels = pvcviewer_common_labels(viewer);
  Json ps = viewer.at_path({"spec", "podSpec"});
  if (affinity.is_object() && !affinity.empty()) ps["affinity"] = affinity;
  return Json{{"apiVersion", "apps/v1"},
              {"kind", "Deployment"},
              {"metadata", Json{{"name", std::string(PVCVIEWER_PREFIX) + viewer.str_at({"metadata", "name"})},
                                {"namespace", viewer.str_at({"metadata", "namespace"})},
                                {"labels", labels}}},
              {"spec", Json{{"replicas", 1},
                            {"selector", Json{{"matchLabels", labels}}},
                            {"strategy", Json{{"type", "Recreate"}}},
                            {"template", Json{{"metadata", Json{{"labels", labels}}}, {"spec", ps}}}}}};
}

Json pvcviewer_generate_service(const Json& viewer) {
  Json labels = pvcviewer_common_labels(viewer);
  return Json{{"apiVersion", "v1"},
              {"kind", "Service"},
              {"metadata", Json{{"name", std::string(PVCVIEWER_PREFIX) + viewer.str_at({"metadata", "name"})},
                                {"namespace", viewer.str_at({"metadata", "namespace"})},
                                {"labels", labels}}},
              {"spec", Json{{"type", "ClusterIP"},
                            {"selector", labels},
                            {"ports", Json::array({Json{{"name", "http"}, {"port", 80},
                                                        {"targetPort", viewer.at_path({"spec", "networking", "targetPort"})}}})}}}};
}

Json pvcviewer_generate_virtual_service(const Json& viewer, const std::string& gateway) {
  const std::string name = viewer.str_at({"metadata", "name"});
  const std::string ns = viewer.str_at({"metadata", "namespace"});
  const Json& net = viewer.at_path({"spec", "networking"});
  const std::string prefix = net["basePrefix"].as_string() + "/" + ns + "/" + name + "/";
  const std::string rewrite = net["rewrite"].as_string().empty() ? prefix : net["rewrite"].as_string();
  Json http{{"match", Json::array({Json{{"uri", Json{{"prefix", prefix}}}}})},
            {"rewrite", Json{{"uri", rewrite}}},
            {"route", Json::array({Json{{"destination", Json{{"host", std::string(PVCVIEWER_PREFIX) + name + "." + ns + ".svc.cluster.local"},
                                                             {"port", Json{{"number", 80}}}}}}})}};
  if (!net["timeout"].as_string().empty()) http["timeout"] = net["timeout"];
  return Json{{"apiVersion", "networking.istio.io/v1alpha3"},
              {"kind", "VirtualService"},
              {"metadata", Json{{"name", std::string(PVCVIEWER_PREFIX) + name}, {"namespace", ns}, {"labels", pvcviewer_common_labels(viewer)}}},
              {"spec", Json{{"hosts", Json::array({"*"})}, {"gateways", Json::array({gateway})}, {"http", Json::array({http})}}}};
}

std::string pvcviewer_rwo_node(const Json& pvc, const std::vector<Json>& pods) {
  const Json& am = pvc.at_path({"spec", "accessModes"});
  if (!am.is_array() || am.size() != 1 || am[0].as_string() != "ReadWriteOnce") return "";
  const std::string claim = pvc.str_at({"metadata", "name"});
  std::string node;
  for (const auto& p : pods) {
    if (label(p, "app.kubernetes.io/part-of") == "pvc-viewer") continue;
    for (const auto& v : p.at_path({"spec", "volumes"}).as_array()) {
      if (v.at_path({"persistentVolumeClaim", "claimName"}).as_string() != claim) continue;
      const std::string n = p.at_path({"spec", "nodeName"}).as_string();
      if (n.empty()) return "";               // RWO volume on a pod without nodeName
      if (!node.empty() && node != n) return "";  // RWO volume on multiple nodes
      node = n;
    }
  }
  return node;
}

namespace {
bool pvcviewer_networking_set(const Json& v) {
  const Json& n = v.at_path({"spec", "networking"});
  if (!n.is_object()) return false;
  for (const auto& kv : n.as_object())
    if (!kv.second.is_null() && !(kv.second.is_string() && kv.second.as_string().empty()) &&
        !(kv.second.is_number() && kv.second.as_int() == 0))
      return true;
  return false;
}

Json load_default_pod_spec() {
  const std::string path = getenv_or("DEFAULT_POD_SPEC_PATH", "");
  if (path.empty()) return Json();
  std::string text;
  if (!read_file(path, text)) {
    KF_ERROR("pvcviewer-resource", "Failed to read podSpec defaults from file " + path);
    return Json();
  }
  Json out;
  std::string err;
  if (!Json::try_parse(text, out) && !parse_yaml(text, out, &err)) {
    KF_ERROR("pvcviewer-resource", "Failed to unmarshal podSpec defaults file " + path, Json{{"error", err}});
    return Json();
  }
  return out;
}
}  // namespace

AdmissionFn make_pvcviewer_defaulter() {
  return [](AdmissionAttrs& a) -> ApiError {
    if (!a.object || a.res->kind != "PVCViewer" || (a.operation != "CREATE" && a.operation != "UPDATE")) return {};
    Json& v = *a.object;
    if (v.str_at({"metadata", "namespace"}).empty()) v["metadata"]["namespace"] = a.ns;
    v = pvcviewer_default(v, load_default_pod_spec());
    return {};
  };
}

AdmissionFn make_pvcviewer_validator() {
  return [](AdmissionAttrs& a) -> ApiError {
    if (!a.object || a.res->kind != "PVCViewer" || (a.operation != "CREATE" && a.operation != "UPDATE")) return {};
    const std::string msg = pvcviewer_validate(*a.object);
    if (!msg.empty()) return ApiError::Forbidden("admission webhook \"vpvcviewer.kb.io\" denied the request: " + msg);
    return {};
  };
}

ApiError PVCViewerReconciler::reconcile_status(const std::string& ns, const std::string& name) {
  Json v;
  ApiError e = c_->get("kubeflow.org/v1alpha1", "PVCViewer", ns, name, v);
  if (e) return e;
  Json st = v["status"].is_object() ? v["status"] : Json::object();
  if (pvcviewer_networking_set(v)) st["url"] = v.at_path({"spec", "networking", "basePrefix"}).as_string() + "/" + ns + "/" + name + "/";
  else st.erase("url");
  Json dep;
  if (c_->get("apps/v1", "Deployment", ns, std::string(PVCVIEWER_PREFIX) + name, dep)) {
    st["ready"] = false;
  } else {
    st["ready"] = dep.at_path({"spec", "replicas"}).as_int(1) == dep.at_path({"status", "readyReplicas"}).as_int(0);
    const Json& dc = dep.at_path({"status", "conditions"});
    if (dc.is_array() && !dc.empty()) {
      if (!st["conditions"].is_array()) st["conditions"] = Json::array();
      const auto& cs = st["conditions"].as_array();
      if (cs.empty() || cs.back() != dc[0]) st["conditions"].push_back(dc[0]);
    }
  }
  if (st == v["status"]) return {};
  v["status"] = st;
  return c_->update_status(v);
}

Result PVCViewerReconciler::reconcile(const Request& r, std::string* err) {
  Json v;
  ApiError e = c_->get("kubeflow.org/v1alpha1", "PVCViewer", r.ns, r.name, v);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  if (v.at_path({"metadata", "deletionTimestamp"}).is_string()) {
    e = reconcile_status(r.ns, r.name);
    if (e && e.code != 404) *err = e.message;
    return {};
  }
  // ---- deployment (affinity decided only when creating)
  const std::string dname = std::string(PVCVIEWER_PREFIX) + r.name;
  Json found;
  e = c_->get("apps/v1", "Deployment", r.ns, dname, found);
  const bool create = e.code == 404;
  if (e && !create) {
    *err = e.message;
    return {};
  }
  Json affinity = create ? Json::object() : found.at_path({"spec", "template", "spec", "affinity"});
  if (create && v.at_path({"spec", "rwoScheduling"}).as_bool()) {
    Json pvc;
    ApiError pe = c_->get("v1", "PersistentVolumeClaim", r.ns, v.at_path({"spec", "pvc"}).as_string(), pvc);
    if (pe && pe.code != 404) {
      *err = pe.message;
      return {};
    }
    if (!pe) {
      Json pods;
      c_->list("v1", "Pod", r.ns, ListOptions(), pods);
      std::vector<Json> pl(pods["items"].as_array().begin(), pods["items"].as_array().end());
      affinity = preferred_node_affinity(pvcviewer_rwo_node(pvc, pl));
    }
  }
  Json dep = pvcviewer_generate_deployment(v, affinity);
  set_controller_reference(v, dep);
  if (create) {
    e = c_->create(dep);
  } else {
    found["metadata"]["labels"] = dep.at_path({"metadata", "labels"});
    found["spec"]["selector"] = dep.at_path({"spec", "selector"});
    found["spec"]["template"] = dep.at_path({"spec", "template"});
    found["spec"]["strategy"] = dep.at_path({"spec", "strategy"});
    Json cur;
    c_->get("apps/v1", "Deployment", r.ns, dname, cur);
    e = cur == found ? ApiError{} : c_->update(found);
  }
  if (e) {
    *err = "Error while reconciling deployment: " + e.message;
    return {};
  }
  // ---- service + virtual service only with networking
  if (pvcviewer_networking_set(v)) {
    Json svc = pvcviewer_generate_service(v);
    set_controller_reference(v, svc);
    if ((e = reconcile_owned(*c_, svc, CopyKind::Service))) {
      *err = "Error while reconciling service: " + e.message;
      return {};
    }
    Json vs = pvcviewer_generate_virtual_service(v, getenv_or("ISTIO_GATEWAY", "kubeflow/kubeflow-gateway"));
    set_controller_reference(v, vs);
    if ((e = reconcile_owned(*c_, vs, CopyKind::VirtualService))) {
      *err = "Error while reconciling virtual service: " + e.message;
      return {};
    }
  }
  e = reconcile_status(r.ns, r.name);
  if (e && e.code != 409) *err = "Error while reconciling status: " + e.message;
  return {};
}

void PVCViewerReconciler::setup(Manager& mgr, int workers) {
  ctl_ = std::make_shared<Controller>("pvcviewer-controller", [this](const Request& r, std::string* e) { return reconcile(r, e); },
                                      workers);
  ctl_->For(mgr.informer("kubeflow.org/v1alpha1", "PVCViewer"));
  ctl_->Owns(mgr.informer("apps/v1", "Deployment"), "PVCViewer");
  ctl_->Owns(mgr.informer("v1", "Service"), "PVCViewer");
  ctl_->Owns(mgr.informer("networking.istio.io/v1alpha3", "VirtualService"), "PVCViewer");
  mgr.add(ctl_);
}

}  // namespace kf
