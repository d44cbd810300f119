// notebook.cc — N2 NotebookReconciler (reference notebook-controller/controllers/notebook_controller.go).
#include <cmath>

#include "controllers/notebook.h"

#include "core/util.h"

namespace kf {

NotebookOptions NotebookOptions::from_env() {
  NotebookOptions o;
  o.use_istio = getenv_or("USE_ISTIO", "false") == "true";
  o.istio_gateway = getenv_or("ISTIO_GATEWAY", "");
  if (o.istio_gateway.empty()) o.istio_gateway = "kubeflow/kubeflow-gateway";
  o.istio_host = getenv_or("ISTIO_HOST", "");
  if (o.istio_host.empty()) o.istio_host = "*";
  o.cluster_domain = getenv_or("CLUSTER_DOMAIN", "cluster.local");
  const char* fs = std::getenv("ADD_FSGROUP");
  o.add_fsgroup = !fs || std::string(fs) == "true";
  return o;
}

Json generate_statefulset(const Json& nb, const NotebookOptions& o) {
  const std::string name = nb.str_at({"metadata", "name"}), ns = nb.str_at({"metadata", "namespace"});
  const int replicas = stop_annotation_is_set(nb) ? 0 : 1;
  Json labels{{"statefulset", name}, {"notebook-name", name}, {WORKBENCH_LABEL, "true"}};
  for (const auto& m : nb.at_path({"metadata", "labels"}).as_object()) labels[m.first] = m.second;
  Json annotations = Json::object();
  // Q1: annotations whose key contains "kubectl" or "notebook" are not copied to the pod
  for (const auto& m : nb.at_path({"metadata", "annotations"}).as_object())
    if (!contains(m.first, "kubectl") && !contains(m.first, "notebook")) annotations[m.first] = m.second;
  Json spec = nb.at_path({"spec", "template", "spec"});
  if (!spec.is_object()) spec = Json::object();
  Json& containers = spec["containers"];
  if (containers.is_array() && !containers.empty()) {
    Json& c = containers[0];
    if (c["workingDir"].as_string().empty()) c["workingDir"] = "/home/jovyan";
    if (!c["ports"].is_array())
      c["ports"] = Json::array({Json{{"containerPort", DEFAULT_CONTAINER_PORT}, {"name", "notebook-port"}, {"protocol", "TCP"}}});
    // setPrefixEnvVar — note: the reference mutates a copy inside its range loop, so an existing
    // NB_PREFIX is left untouched (and not duplicated); same here.
    bool found = false;
    for (const auto& e : c["env"].as_array()) found = found || e["name"].as_string() == PREFIX_ENV_VAR;
    if (!found) c["env"].push_back(Json{{"name", PREFIX_ENV_VAR}, {"value", "/notebook/" + ns + "/" + name}});
  }
  if (o.add_fsgroup && !spec.has("securityContext")) spec["securityContext"] = Json{{"fsGroup", DEFAULT_FS_GROUP}};
  return Json{{"apiVersion", "apps/v1"},
              {"kind", "StatefulSet"},
              {"metadata", Json{{"name", name}, {"namespace", ns}}},
              {"spec", Json{{"replicas", replicas},
                            {"selector", Json{{"matchLabels", Json{{"statefulset", name}}}}},
                            {"serviceName", ""},
                            {"template", Json{{"metadata", Json{{"labels", labels}, {"annotations", annotations}}},
                                              {"spec", spec}}}}}};
}

Json generate_service(const Json& nb) {
  const std::string name = nb.str_at({"metadata", "name"}), ns = nb.str_at({"metadata", "namespace"});
  int64_t port = DEFAULT_CONTAINER_PORT;
  const Json& ports = nb.at_path({"spec", "template", "spec", "containers"})[0]["ports"];
  if (ports.is_array() && !ports.empty()) port = ports[0]["containerPort"].as_int(DEFAULT_CONTAINER_PORT);
  return Json{{"apiVersion", "v1"},
              {"kind", "Service"},
              {"metadata", Json{{"name", name}, {"namespace", ns}}},
              {"spec", Json{{"type", "ClusterIP"},
                            {"selector", Json{{"statefulset", name}}},
                            {"ports", Json::array({Json{{"name", "http-" + name}, {"port", DEFAULT_SERVING_PORT},
                                                        {"targetPort", port}, {"protocol", "TCP"}}})}}}};
}

std::string virtual_service_name(const std::string& name, const std::string& ns) { return "notebook-" + ns + "-" + name; }

Json generate_virtual_service(const Json& nb, const NotebookOptions& o) {
  const std::string name = nb.str_at({"metadata", "name"}), ns = nb.str_at({"metadata", "namespace"});
  const std::string prefix = "/notebook/" + ns + "/" + name + "/";
  std::string rewrite = annotation(nb, ANNOTATION_REWRITE_URI);
  if (rewrite.empty()) rewrite = prefix;
  Json headers = Json::object();
  std::string hs = annotation(nb, ANNOTATION_HEADERS_REQUEST_SET);
  if (!hs.empty()) {
    Json parsed;
    if (Json::try_parse(hs, parsed) && parsed.is_object()) {
      bool all_str = true;
      for (const auto& m : parsed.as_object()) all_str = all_str && m.second.is_string();
      if (all_str) headers = parsed;  // invalid JSON or non-string values -> empty map (reference behaviour)
    }
  }
  const std::string service = name + "." + ns + ".svc." + o.cluster_domain;
  Json http = Json::array({Json{{"headers", Json{{"request", Json{{"set", headers}}}}},
                                {"match", Json::array({Json{{"uri", Json{{"prefix", prefix}}}}})},
                                {"rewrite", Json{{"uri", rewrite}}},
                                {"route", Json::array({Json{{"destination", Json{{"host", service},
                                                                                 {"port", Json{{"number", DEFAULT_SERVING_PORT}}}}}}})}}});
  return Json{{"apiVersion", "networking.istio.io/v1alpha3"},
              {"kind", "VirtualService"},
              {"metadata", Json{{"name", virtual_service_name(name, ns)}, {"namespace", ns}}},
              {"spec", Json{{"hosts", Json::array({o.istio_host})}, {"gateways", Json::array({o.istio_gateway})}, {"http", http}}}};
}

Json pod_cond_to_notebook_cond(const Json& pc) {
  Json c = Json::object();
  if (!pc["type"].as_string().empty()) c["type"] = pc["type"];
  if (!pc["status"].as_string().empty()) c["status"] = pc["status"];
  if (!pc["message"].as_string().empty()) c["message"] = pc["message"];
  if (!pc["reason"].as_string().empty()) c["reason"] = pc["reason"];
  c["lastProbeTime"] = pc["lastProbeTime"].as_string().empty() ? Json(rfc3339_now()) : pc["lastProbeTime"];
  c["lastTransitionTime"] = pc["lastTransitionTime"].as_string().empty() ? Json(rfc3339_now()) : pc["lastTransitionTime"];
  return c;
}

Json create_notebook_status(const Json& nb, const Json& sts, const Json& pod) {
  Json status{{"conditions", Json::array()},
              {"readyReplicas", sts.at_path({"status", "readyReplicas"}).as_int(0)},
              {"containerState", Json::object()}};
  const Json& ps = pod["status"];
  if (!ps.is_object() || ps.empty()) return status;
  const std::string name = nb.str_at({"metadata", "name"});
  const Json& prev = nb.at_path({"status", "containerState"});
  for (const auto& cs : ps["containerStatuses"].as_array()) {
    if (cs["name"].as_string() != name) continue;
    status["containerState"] = cs["state"].is_object() ? cs["state"] : (prev.is_object() ? prev : Json::object());
    break;
  }
  Json conds = Json::array();
  for (const auto& pc : ps["conditions"].as_array()) conds.push_back(pod_cond_to_notebook_cond(pc));
  status["conditions"] = conds;
  return status;
}

bool nb_name_from_involved_object(Client& c, const Json& involved, std::string& out) {
  const std::string& kind = involved["kind"].as_string();
  if (kind == "StatefulSet") {
    out = involved["name"].as_string();
    return true;
  }
  if (kind == "Pod") {
    Json pod;
    if (c.get("v1", "Pod", involved["namespace"].as_string(), involved["name"].as_string(), pod)) return false;
    std::string nb = label(pod, "notebook-name");
    if (nb.empty()) return false;
    out = nb;
    return true;
  }
  return false;
}

NotebookReconciler::NotebookReconciler(std::shared_ptr<Client> c, NotebookOptions o, std::shared_ptr<NotebookMetrics> m)
    : c_(std::move(c)), o_(std::move(o)), m_(std::move(m)), rec_(std::make_unique<EventRecorder>(c_, "notebook-controller")) {}

Result NotebookReconciler::reemit_event(const Json& event, std::string* err) {
  std::string nb_name;
  if (!nb_name_from_involved_object(*c_, event["involvedObject"], nb_name)) {
    *err = "object isn't related to a Notebook";
    return {};
  }
  Json nb;
  ApiError e = c_->get("kubeflow.org/v1beta1", "Notebook", event.str_at({"metadata", "namespace"}), nb_name, nb);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  rec_->event(nb, event["type"].as_string(), event["reason"].as_string(),
              "Reissued from " + to_lower(event.str_at({"involvedObject", "kind"})) + "/" +
                  event.str_at({"involvedObject", "name"}) + ": " + event["message"].as_string());
  return {};
}

Result NotebookReconciler::reconcile(const Request& req, std::string* err) {
  // Q15: Events and Notebooks share one queue; a request is first tried as an Event.
  Json event;
  ApiError e = c_->get("v1", "Event", req.ns, req.name, event);
  if (!e) return reemit_event(event, err);
  if (e.code != 404) {
    *err = e.message;
    return {};
  }
  Json nb;
  e = c_->get("kubeflow.org/v1beta1", "Notebook", req.ns, req.name, nb);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  // foreground deletion by the JWA: do nothing while terminating
  if (nb.at_path({"metadata", "deletionTimestamp"}).is_string()) {
    std::lock_guard<std::mutex> g(cs_mu_);
    cold_.erase(nb.str_at({"metadata", "uid"}));
    return {};
  }
  if (annotation(nb, ANNOTATION_COLD_START).empty() && nb.at_path({"status", "readyReplicas"}).as_int(0) != 1) {
    std::lock_guard<std::mutex> g(cs_mu_);
    auto& cs = cold_[nb.str_at({"metadata", "uid"})];
    if (cs.seen == 0) cs.seen = now_unix_ms() / 1000.0;  // wall clock: compared with pod condition times
  }

  // ---- StatefulSet
  Json ss = generate_statefulset(nb, o_);
  set_controller_reference(nb, ss);
  Json found;
  e = c_->get("apps/v1", "StatefulSet", req.ns, req.name, found);
  bool just_created = false;
  if (e.code == 404) {
    KF_INFO("notebook-controller", "Creating StatefulSet", Json{{"namespace", req.ns}, {"name", req.name}});
    m_->create_total->inc({req.ns});
    Json obj = ss;
    e = c_->create(obj);
    just_created = true;
    if (e) {
      m_->create_failed_total->inc({req.ns});
      *err = "unable to create Statefulset: " + e.message;
      // the reference only logs this; a user of kfctl / the JWA would never see why nothing runs
      // (e.g. the API server refused a pod template asking for "0.5" GPUs)
      rec_->event(nb, "Warning", "FailedCreate", "unable to create StatefulSet: " + e.message);
      return {};
    }
    found = obj;
    std::lock_guard<std::mutex> g(cs_mu_);
    auto it = cold_.find(nb.str_at({"metadata", "uid"}));
    if (it != cold_.end()) it->second.sts = now_unix_ms() / 1000.0;
  } else if (e) {
    *err = e.message;
    return {};
  }
  if (!just_created && copy_statefulset_fields(ss, found)) {
    KF_INFO("notebook-controller", "Updating StatefulSet", Json{{"namespace", req.ns}, {"name", req.name}});
    // the pod-template labels are not in CopyStatefulSetFields; the reference copies them when
    // replicas change, we keep them in sync always (so PodDefault selectors follow the CR labels)
    found["spec"]["template"]["metadata"]["labels"] = ss.at_path({"spec", "template", "metadata", "labels"});
    found["spec"]["template"]["metadata"]["annotations"] = ss.at_path({"spec", "template", "metadata", "annotations"});
    e = c_->update(found);
    if (e) {
      *err = "unable to update Statefulset: " + e.message;
      return {};
    }
  }
  // ---- Service
  Json svc = generate_service(nb);
  set_controller_reference(nb, svc);
  e = reconcile_owned(*c_, svc, CopyKind::Service);
  if (e) {
    *err = "unable to reconcile Service: " + e.message;
    return {};
  }
  // ---- VirtualService
  if (o_.use_istio) {
    Json vs = generate_virtual_service(nb, o_);
    set_controller_reference(nb, vs);
    e = reconcile_owned(*c_, vs, CopyKind::VirtualService);
    if (e) {
      *err = "unable to reconcile VirtualService: " + e.message;
      return {};
    }
  }
  // ---- status
  Json pod;
  e = c_->get("v1", "Pod", req.ns, req.name + "-0", pod);
  if (e && e.code != 404) {
    *err = e.message;
    return {};
  }
  Json status = create_notebook_status(nb, found, e ? Json::object() : pod);
  if (!e) {
    // MI355X extension: surface the in-pod GPU readiness op result + cold-start phases
    const std::string gr = annotation(pod, ANNOTATION_GPU_READINESS);
    if (!gr.empty()) {
      Json g;
      if (Json::try_parse(gr, g)) status["gpuReadiness"] = g;
    }
    // the gpu-readiness init container's termination message (kfamd-readiness JSON summary)
    for (const auto& ics : pod.at_path({"status", "initContainerStatuses"}).as_array()) {
      if (ics["name"].as_string() != "gpu-readiness") continue;
      const Json& t = ics.at_path({"state", "terminated"}).is_object() ? ics.at_path({"state", "terminated"})
                                                                       : ics.at_path({"lastState", "terminated"});
      Json g;
      if (t.is_object() && Json::try_parse(t["message"].as_string(), g)) status["gpuReadiness"] = g;
    }
    if (pod.at_path({"metadata", "annotations"}).has(ANNOTATION_GPU_IDS))
      status["gpus"] = annotation(pod, ANNOTATION_GPU_IDS);
  }
  if (nb["status"] != status) {
    Json upd = nb;
    upd["status"] = status;
    e = c_->update_status(upd);
    if (e) {
      *err = "unable to update Notebook status: " + e.message;
      return {};
    }
    nb = upd;
  }
  track_cold_start(nb, pod, status);
  // ---- restart annotation: delete the pod once, then clear the annotation
  if (annotation(nb, ANNOTATION_NOTEBOOK_RESTART) == "true") {
    KF_INFO("notebook-controller", "Annotation restart-pod is set, restarting the pod", Json{{"notebook", req.str()}});
    ApiError de = c_->remove("v1", "Pod", req.ns, req.name + "-0");
    if (de && de.code != 404) {
      *err = de.message;
      return {};
    }
    e = c_->update_with_retry("kubeflow.org/v1beta1", "Notebook", req.ns, req.name, [](Json& o) {
      if (!o["metadata"]["annotations"].has(ANNOTATION_NOTEBOOK_RESTART)) return false;
      o["metadata"]["annotations"].erase(ANNOTATION_NOTEBOOK_RESTART);
      return true;
    });
    if (e) {
      *err = e.message;
      return {};
    }
  }
  return {};
}

// the cold-start phases of a Notebook's first start, from the controller's own
// observations (first reconcile, StatefulSet create, Ready) and the pod's condition transition
// times (the kubelet stamps them with ms precision). Exported as the notebook_cold_start_seconds
// histogram and as the kfamd.io/cold-start annotation on the Notebook.
void NotebookReconciler::track_cold_start(const Json& nb, const Json& pod, const Json& status) {
  const std::string uid = nb.str_at({"metadata", "uid"});
  ColdStart cs;
  {
    std::lock_guard<std::mutex> g(cs_mu_);
    auto it = cold_.find(uid);
    if (it == cold_.end()) return;
    if (status["readyReplicas"].as_int(0) != 1) return;
    cs = it->second;
    cold_.erase(it);
  }
  const double now = now_unix_ms() / 1000.0;
  auto cond_time = [&](const std::string& type) -> double {
    for (const auto& c : pod.at_path({"status", "conditions"}).as_array())
      if (c["type"].as_string() == type && c["status"].as_string() == "True") {
        auto ms = parse_rfc3339_ms(c["lastTransitionTime"].as_string());
        if (ms) return static_cast<double>(*ms) / 1000.0;
      }
    return 0;
  };
  const double sched = cond_time("PodScheduled"), init = cond_time("Initialized"), ready = cond_time("Ready");
  Json phases = Json::object();
  auto phase = [&](const char* name, double a, double b) {
    if (a <= 0 || b <= 0 || b < a) return;
    m_->cold_start_seconds->observe({name}, b - a);
    phases[std::string(name) + "_ms"] = std::round((b - a) * 1e4) / 10.0;
  };
  phase("observed_to_statefulset", cs.seen, cs.sts);
  phase("statefulset_to_scheduled", cs.sts, sched);
  phase("scheduled_to_initialized", sched, init);
  phase("initialized_to_ready", init, ready);
  phase("total", cs.seen, now);
  const std::string val = phases.dump();
  ApiError e = c_->update_with_retry("kubeflow.org/v1beta1", "Notebook", nb.str_at({"metadata", "namespace"}),
                                     nb.str_at({"metadata", "name"}), [&val](Json& o) {
                                       if (!o["metadata"]["annotations"].is_object()) o["metadata"]["annotations"] = Json::object();
                                       if (o["metadata"]["annotations"].has(ANNOTATION_COLD_START)) return false;
                                       o["metadata"]["annotations"][ANNOTATION_COLD_START] = val;
                                       return true;
                                     });
  if (e) KF_WARN("notebook-controller", "cannot record cold-start phases", Json{{"error", e.message}});
}

void NotebookReconciler::setup(Manager& mgr, int workers) {
  ctl_ = std::make_shared<Controller>("notebook-controller",
                                      [this](const Request& r, std::string* err) { return reconcile(r, err); }, workers);
  ctl_->For(mgr.informer("kubeflow.org/v1beta1", "Notebook"));
  ctl_->Owns(mgr.informer("apps/v1", "StatefulSet"), "Notebook");
  ctl_->Owns(mgr.informer("v1", "Service"), "Notebook");
  // Pods carrying the notebook-name label
  ctl_->Watches(
      mgr.informer("v1", "Pod"),
      [](const std::string&, const Json& pod) {
        return std::vector<Request>{{pod.str_at({"metadata", "namespace"}), label(pod, "notebook-name")}};
      },
      [](const std::string&, const Json& pod, const Json*) { return !label(pod, "notebook-name").empty(); });
  // Events about Pods / StatefulSets of existing notebooks (never on delete)
  auto c = c_;
  Informer& nbs = mgr.informer("kubeflow.org/v1beta1", "Notebook");
  ctl_->Watches(
      mgr.informer("v1", "Event"),
      [](const std::string&, const Json& ev) {
        return std::vector<Request>{{ev.str_at({"metadata", "namespace"}), ev.str_at({"metadata", "name"})}};
      },
      [c, &nbs](const std::string& type, const Json& ev, const Json*) {
        if (type == "DELETED") return false;
        const std::string& kind = ev.str_at({"involvedObject", "kind"});
        if (kind != "Pod" && kind != "StatefulSet") return false;
        std::string nb;
        if (!nb_name_from_involved_object(*c, ev["involvedObject"], nb)) return false;
        Json tmp;
        return nbs.get(ev.str_at({"metadata", "namespace"}), nb, tmp);
      });
  if (o_.use_istio) ctl_->Owns(mgr.informer("networking.istio.io/v1alpha3", "VirtualService"), "Notebook");
  mgr.add(ctl_);
}

}  // namespace kf
