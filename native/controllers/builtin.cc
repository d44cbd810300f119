// builtin.cc — StatefulSet, Deployment, ReplicaSet and PVC-binder controllers (see builtin.h).
#include "controllers/builtin.h"

#include <algorithm>
#include <map>

#include "core/util.h"

namespace kf {

std::string pod_template_hash(const Json& t) {
  uint32_t h = 2166136261u;
  for (unsigned char ch : t.dump()) {
    h ^= ch;
    h *= 16777619u;
  }
  static const char* alpha = "bcdfghjklmnpqrstvwxz2456789";
  std::string out;
  for (int i = 0; i < 10; ++i) {
    out += alpha[h % 27];
    h = h / 27 + (h * 2654435761u >> 7);
  }
  return out;
}

bool pod_is_ready(const Json& pod) {
  for (const auto& c : pod.at_path({"status", "conditions"}).as_array())
    if (c["type"].as_string() == "Ready") return c["status"].as_string() == "True";
  return false;
}

bool pod_is_terminal(const Json& pod) {
  const std::string& ph = pod.at_path({"status", "phase"}).as_string();
  return ph == "Succeeded" || ph == "Failed";
}

namespace {
bool being_deleted(const Json& o) { return o.at_path({"metadata", "deletionTimestamp"}).is_string(); }

std::vector<Json> owned_pods(Informer* pods, const Json& owner) {
  std::vector<Json> out;
  pods->visit(owner.str_at({"metadata", "namespace"}), [&](const Json& p) {
    if (is_controlled_by(p, owner)) out.push_back(p);
  });
  return out;
}

int ordinal_of(const std::string& sts, const std::string& pod) {
  if (!starts_with(pod, sts + "-")) return -1;
  std::string s = pod.substr(sts.size() + 1);
  if (s.empty() || s.find_first_not_of("0123456789") != std::string::npos) return -1;
  return std::atoi(s.c_str());
}
}  // namespace

Json BuiltinControllers::make_pod(const Json& owner, const Json& tmpl, const std::string& name, const Json& extra_labels) {
  Json pod{{"apiVersion", "v1"}, {"kind", "Pod"},
           {"metadata", Json{{"name", name}, {"namespace", owner.str_at({"metadata", "namespace"})}}},
           {"spec", tmpl["spec"]}};
  Json labels = tmpl.at_path({"metadata", "labels"});
  if (!labels.is_object()) labels = Json::object();
  for (const auto& m : extra_labels.as_object()) labels[m.first] = m.second;
  pod["metadata"]["labels"] = labels;
  if (tmpl.at_path({"metadata", "annotations"}).is_object() && !tmpl.at_path({"metadata", "annotations"}).empty())
    pod["metadata"]["annotations"] = tmpl.at_path({"metadata", "annotations"});
  set_controller_reference(owner, pod);
  return pod;
}

// ---- StatefulSet -------------------------------------------------------------------------------
Result BuiltinControllers::reconcile_statefulset(const Request& r, std::string* err) {
  Json sts;
  ApiError e = c_->get("apps/v1", "StatefulSet", r.ns, r.name, sts);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  if (being_deleted(sts)) return {};
  const int64_t replicas = sts.at_path({"spec", "replicas"}).as_int(1);
  const Json& tmpl = sts.at_path({"spec", "template"});
  const std::string rev = r.name + "-" + pod_template_hash(tmpl);
  const bool ordered = sts.at_path({"spec", "podManagementPolicy"}).as_string_or("OrderedReady") == "OrderedReady";
  std::map<int, Json> by_ord;
  for (auto& p : owned_pods(pods_, sts)) {
    int o = ordinal_of(r.name, p.str_at({"metadata", "name"}));
    if (o >= 0) by_ord[o] = p;
  }
  bool waiting = false;
  // replace terminal pods, create missing ones in ordinal order
  for (int64_t i = 0; i < replicas; ++i) {
    auto it = by_ord.find(static_cast<int>(i));
    if (it != by_ord.end()) {
      if (pod_is_terminal(it->second) && !being_deleted(it->second)) {
        c_->remove("v1", "Pod", r.ns, it->second.str_at({"metadata", "name"}), "", 0);
        waiting = true;
        if (ordered) break;
      }
      if (ordered && (!pod_is_ready(it->second) || being_deleted(it->second))) {
        waiting = true;
        break;
      }
      continue;
    }
    const std::string pname = r.name + "-" + std::to_string(i);
    Json extra{{"statefulset.kubernetes.io/pod-name", pname}, {"controller-revision-hash", rev},
               {"apps.kubernetes.io/pod-index", std::to_string(i)}};
    Json pod = make_pod(sts, tmpl, pname, extra);
    pod["spec"]["hostname"] = pname;
    if (!sts.at_path({"spec", "serviceName"}).as_string().empty()) pod["spec"]["subdomain"] = sts.at_path({"spec", "serviceName"});
    for (const auto& vct : sts.at_path({"spec", "volumeClaimTemplates"}).as_array()) {
      const std::string claim = vct.str_at({"metadata", "name"}) + "-" + pname;
      Json pvc{{"apiVersion", "v1"}, {"kind", "PersistentVolumeClaim"},
               {"metadata", Json{{"name", claim}, {"namespace", r.ns}, {"labels", tmpl.at_path({"metadata", "labels"})}}},
               {"spec", vct["spec"]}};
      ApiError pe = c_->create(pvc);
      if (pe && pe.code != 409) {
        *err = "pvc " + claim + ": " + pe.message;
        return {};
      }
      Json& vols = pod["spec"]["volumes"];
      bool have = false;
      for (const auto& v : vols.as_array()) have = have || v["name"].as_string() == vct.str_at({"metadata", "name"});
      if (!have) vols.push_back(Json{{"name", vct.str_at({"metadata", "name"})}, {"persistentVolumeClaim", Json{{"claimName", claim}}}});
    }
    e = c_->create(pod);
    if (e && e.code != 409) {
      *err = "create pod " + pname + ": " + e.message;
      if (sts_rec_)
        sts_rec_->event(sts, "Warning", "FailedCreate",
                        "create Pod " + pname + " in StatefulSet " + r.name + " failed error: " + e.message);
      return Result::after(5.0);
    }
    if (!e && sts_rec_)
      sts_rec_->event(sts, "Normal", "SuccessfulCreate", "create Pod " + pname + " in StatefulSet " + r.name + " successful");
    waiting = true;
    if (ordered) break;
  }
  // scale down: highest ordinal first
  for (auto it = by_ord.rbegin(); it != by_ord.rend(); ++it) {
    if (it->first < replicas) break;
    if (!being_deleted(it->second)) c_->remove("v1", "Pod", r.ns, it->second.str_at({"metadata", "name"}));
    if (ordered) break;
  }
  // rolling update (highest ordinal first, one at a time, only when everything is ready)
  if (!waiting && sts.at_path({"spec", "updateStrategy", "type"}).as_string_or("RollingUpdate") == "RollingUpdate") {
    bool all_ready = true;
    for (int64_t i = 0; i < replicas; ++i) {
      auto it = by_ord.find(static_cast<int>(i));
      all_ready = all_ready && it != by_ord.end() && pod_is_ready(it->second) && !being_deleted(it->second);
    }
    int64_t partition = sts.at_path({"spec", "updateStrategy", "rollingUpdate", "partition"}).as_int(0);
    for (int64_t i = replicas - 1; i >= partition; --i) {
      auto it = by_ord.find(static_cast<int>(i));
      if (it == by_ord.end()) continue;
      if (label(it->second, "controller-revision-hash") != rev) {
        if (all_ready || !ordered) {
          if (!being_deleted(it->second)) c_->remove("v1", "Pod", r.ns, it->second.str_at({"metadata", "name"}));
        }
        break;
      }
    }
  }
  // status
  int64_t count = 0, ready = 0, updated = 0;
  for (auto& kv : by_ord) {
    if (being_deleted(kv.second) && pod_is_terminal(kv.second)) continue;
    count++;
    if (pod_is_ready(kv.second)) ready++;
    if (label(kv.second, "controller-revision-hash") == rev) updated++;
  }
  Json status{{"observedGeneration", sts.at_path({"metadata", "generation"}).as_int(1)},
              {"replicas", count},
              {"readyReplicas", ready},
              {"currentReplicas", updated},
              {"updatedReplicas", updated},
              {"availableReplicas", ready},
              {"currentRevision", rev},
              {"updateRevision", rev},
              {"collisionCount", 0}};
  if (ready == 0) status.erase("readyReplicas");  // omitempty, like the real API
  if (sts["status"] != status) {
    sts["status"] = status;
    e = c_->update_status(sts);
    if (e && e.code != 409) *err = e.message;
  }
  return {};
}

// ---- Deployment ---------------------------------------------------------------------------------
Result BuiltinControllers::reconcile_deployment(const Request& r, std::string* err) {
  Json dep;
  ApiError e = c_->get("apps/v1", "Deployment", r.ns, r.name, dep);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  if (being_deleted(dep)) return {};
  const int64_t desired = dep.at_path({"spec", "replicas"}).as_int(1);
  const Json& tmpl = dep.at_path({"spec", "template"});
  const std::string hash = pod_template_hash(tmpl);
  Json rs_list;
  e = c_->list("apps/v1", "ReplicaSet", r.ns, ListOptions(), rs_list);
  if (e) {
    *err = e.message;
    return {};
  }
  std::vector<Json> owned;
  Json new_rs;
  for (const auto& rs : rs_list["items"].as_array()) {
    if (!is_controlled_by(rs, dep)) continue;
    if (label(rs, "pod-template-hash") == hash) new_rs = rs;
    else owned.push_back(rs);
  }
  const bool recreate = dep.at_path({"spec", "strategy", "type"}).as_string() == "Recreate";
  int64_t old_pods = 0;
  for (auto& rs : owned) old_pods += rs.at_path({"status", "replicas"}).as_int(0);
  if (new_rs.is_null()) {
    Json t = tmpl;
    t["metadata"]["labels"]["pod-template-hash"] = hash;
    Json sel = dep.at_path({"spec", "selector"});
    sel["matchLabels"]["pod-template-hash"] = hash;
    new_rs = Json{{"apiVersion", "apps/v1"}, {"kind", "ReplicaSet"},
                  {"metadata", Json{{"name", r.name + "-" + hash}, {"namespace", r.ns},
                                    {"labels", t.at_path({"metadata", "labels"})},
                                    {"annotations", Json{{"deployment.kubernetes.io/revision", std::to_string(owned.size() + 1)}}}}},
                  {"spec", Json{{"replicas", (recreate && old_pods > 0) ? 0 : desired}, {"selector", sel}, {"template", t}}}};
    set_controller_reference(dep, new_rs);
    e = c_->create(new_rs);
    if (e && e.code != 409) {
      *err = e.message;
      return {};
    }
    return Result::after(0.05);
  }
  int64_t new_ready = new_rs.at_path({"status", "readyReplicas"}).as_int(0);
  // scale the new RS
  int64_t want_new = desired;
  if (recreate && old_pods > 0) want_new = 0;
  if (new_rs.at_path({"spec", "replicas"}).as_int(-1) != want_new) {
    c_->update_with_retry("apps/v1", "ReplicaSet", r.ns, new_rs.str_at({"metadata", "name"}), [&](Json& o) {
      o["spec"]["replicas"] = want_new;
      return true;
    });
  }
  // scale old RSs down (Recreate: immediately; RollingUpdate: as new pods become ready)
  for (auto& rs : owned) {
    int64_t cur = rs.at_path({"spec", "replicas"}).as_int(0);
    int64_t target = recreate ? 0 : std::max<int64_t>(0, std::min(cur, desired - new_ready));
    if (cur != target)
      c_->update_with_retry("apps/v1", "ReplicaSet", r.ns, rs.str_at({"metadata", "name"}), [&](Json& o) {
        o["spec"]["replicas"] = target;
        return true;
      });
  }
  // revision history cleanup
  int64_t limit = dep.at_path({"spec", "revisionHistoryLimit"}).as_int(10);
  int64_t idle_old = 0;
  for (auto& rs : owned)
    if (rs.at_path({"spec", "replicas"}).as_int(0) == 0 && rs.at_path({"status", "replicas"}).as_int(0) == 0) {
      if (++idle_old > limit) c_->remove("apps/v1", "ReplicaSet", r.ns, rs.str_at({"metadata", "name"}));
    }
  // status
  int64_t total = new_rs.at_path({"status", "replicas"}).as_int(0), ready = new_ready,
          avail = new_rs.at_path({"status", "availableReplicas"}).as_int(0);
  for (auto& rs : owned) {
    total += rs.at_path({"status", "replicas"}).as_int(0);
    ready += rs.at_path({"status", "readyReplicas"}).as_int(0);
    avail += rs.at_path({"status", "availableReplicas"}).as_int(0);
  }
  const bool available = avail >= desired;
  Json conds = Json::array();
  auto cond = [&](const char* type, bool ok, const char* reason, const std::string& msg) {
    std::string ts = rfc3339_now();
    for (const auto& c : dep.at_path({"status", "conditions"}).as_array())
      if (c["type"].as_string() == type && c["status"].as_string() == (ok ? "True" : "False")) ts = c["lastTransitionTime"].as_string();
    conds.push_back(Json{{"type", type}, {"status", ok ? "True" : "False"}, {"reason", reason}, {"message", msg},
                         {"lastUpdateTime", ts}, {"lastTransitionTime", ts}});
  };
  cond("Available", available, available ? "MinimumReplicasAvailable" : "MinimumReplicasUnavailable",
       available ? "Deployment has minimum availability." : "Deployment does not have minimum availability.");
  cond("Progressing", true, new_rs.at_path({"status", "readyReplicas"}).as_int(0) == desired ? "NewReplicaSetAvailable" : "ReplicaSetUpdated",
       "ReplicaSet \"" + new_rs.str_at({"metadata", "name"}) + "\" is progressing.");
  Json status{{"observedGeneration", dep.at_path({"metadata", "generation"}).as_int(1)},
              {"replicas", total},
              {"updatedReplicas", new_rs.at_path({"status", "replicas"}).as_int(0)},
              {"readyReplicas", ready},
              {"availableReplicas", avail},
              {"unavailableReplicas", std::max<int64_t>(0, desired - avail)},
              {"conditions", conds}};
  if (ready == 0) status.erase("readyReplicas");
  if (dep["status"] != status) {
    dep["status"] = status;
    e = c_->update_status(dep);
    if (e && e.code != 409) *err = e.message;
  }
  if (recreate && old_pods > 0) return Result::after(0.2);
  return {};
}

// ---- ReplicaSet ---------------------------------------------------------------------------------
Result BuiltinControllers::reconcile_replicaset(const Request& r, std::string* err) {
  Json rs;
  ApiError e = c_->get("apps/v1", "ReplicaSet", r.ns, r.name, rs);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  if (being_deleted(rs)) return {};
  const int64_t want = rs.at_path({"spec", "replicas"}).as_int(1);
  std::vector<Json> active;
  for (auto& p : owned_pods(pods_, rs)) {
    if (being_deleted(p)) continue;
    if (pod_is_terminal(p)) {
      c_->remove("v1", "Pod", r.ns, p.str_at({"metadata", "name"}), "", 0);
      continue;
    }
    active.push_back(p);
  }
  const int64_t have = static_cast<int64_t>(active.size());
  for (int64_t i = have; i < want; ++i) {
    Json pod = make_pod(rs, rs.at_path({"spec", "template"}), r.name + "-" + random_alnum(5), Json::object());
    e = c_->create(pod);
    if (e && e.code != 409) {
      *err = e.message;
      if (rs_rec_) rs_rec_->event(rs, "Warning", "FailedCreate", "Error creating: " + e.message);
      return Result::after(5.0);
    }
    if (!e && rs_rec_)
      rs_rec_->event(rs, "Normal", "SuccessfulCreate", "Created pod: " + pod.str_at({"metadata", "name"}));
  }
  if (have > want) {
    // delete not-ready first, then the newest
    std::sort(active.begin(), active.end(), [](const Json& a, const Json& b) {
      bool ra = pod_is_ready(a), rb = pod_is_ready(b);
      if (ra != rb) return !ra;
      return a.str_at({"metadata", "creationTimestamp"}) > b.str_at({"metadata", "creationTimestamp"});
    });
    for (int64_t i = 0; i < have - want; ++i) c_->remove("v1", "Pod", r.ns, active[i].str_at({"metadata", "name"}));
  }
  int64_t ready = 0;
  for (auto& p : active) ready += pod_is_ready(p) ? 1 : 0;
  Json status{{"replicas", have}, {"fullyLabeledReplicas", have}, {"readyReplicas", ready}, {"availableReplicas", ready},
              {"observedGeneration", rs.at_path({"metadata", "generation"}).as_int(1)}};
  if (rs["status"] != status) {
    rs["status"] = status;
    e = c_->update_status(rs);
    if (e && e.code != 409) *err = e.message;
  }
  return {};
}

// ---- PVC binder (hostpath provisioner) ----------------------------------------------------------
Result BuiltinControllers::reconcile_pvc(const Request& r, std::string* err) {
  Json pvc;
  ApiError e = c_->get("v1", "PersistentVolumeClaim", r.ns, r.name, pvc);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  if (being_deleted(pvc) || pvc.at_path({"status", "phase"}).as_string() == "Bound") return {};
  std::string sc_name = pvc.at_path({"spec", "storageClassName"}).as_string();
  Json sc;
  if (sc_name.empty()) {
    Json scs;
    c_->list("storage.k8s.io/v1", "StorageClass", "", ListOptions(), scs);
    for (const auto& s : scs["items"].as_array())
      if (annotation(s, "storageclass.kubernetes.io/is-default-class") == "true") sc = s;
  } else {
    c_->get("storage.k8s.io/v1", "StorageClass", "", sc_name, sc);
  }
  if (sc.is_null() && !sc_name.empty()) return {};  // no provisioner for this class: stays Pending
  if (sc["volumeBindingMode"].as_string() == "WaitForFirstConsumer") {
    bool consumer = false;
    pods_->visit(r.ns, [&](const Json& p) {
      if (p.at_path({"spec", "nodeName"}).as_string().empty()) return;
      for (const auto& v : p.at_path({"spec", "volumes"}).as_array())
        consumer = consumer || v.at_path({"persistentVolumeClaim", "claimName"}).as_string() == r.name;
    });
    if (!consumer) return {};
  }
  const std::string pv_name = "pvc-" + pvc.str_at({"metadata", "uid"});
  Json cap = pvc.at_path({"spec", "resources", "requests"});
  Json pv{{"apiVersion", "v1"}, {"kind", "PersistentVolume"},
          {"metadata", Json{{"name", pv_name}, {"annotations", Json{{"pv.kubernetes.io/provisioned-by", "kflite.io/hostpath"}}}}},
          {"spec", Json{{"capacity", Json{{"storage", cap["storage"].as_string_or("1Gi")}}},
                        {"accessModes", pvc.at_path({"spec", "accessModes"})},
                        {"persistentVolumeReclaimPolicy", "Delete"},
                        {"storageClassName", sc.str_at({"metadata", "name"})},
                        {"hostPath", Json{{"path", "pv/" + r.ns + "/" + r.name}}},
                        {"claimRef", Json{{"kind", "PersistentVolumeClaim"}, {"namespace", r.ns}, {"name", r.name},
                                          {"uid", pvc.at_path({"metadata", "uid"})}}}}},
          {"status", Json{{"phase", "Bound"}}}};
  e = c_->create(pv);
  if (e && e.code != 409) {
    *err = e.message;
    return {};
  }
  e = c_->update_with_retry("v1", "PersistentVolumeClaim", r.ns, r.name, [&](Json& o) {
    if (o.at_path({"spec", "volumeName"}).as_string() == pv_name) return false;
    o["spec"]["volumeName"] = pv_name;
    if (o.at_path({"spec", "storageClassName"}).as_string().empty()) o["spec"]["storageClassName"] = sc.str_at({"metadata", "name"});
    return true;
  });
  if (e) {
    *err = e.message;
    return {};
  }
  e = c_->update_with_retry(
      "v1", "PersistentVolumeClaim", r.ns, r.name,
      [&](Json& o) {
        o["status"] = Json{{"phase", "Bound"},
                           {"accessModes", o.at_path({"spec", "accessModes"})},
                           {"capacity", Json{{"storage", cap["storage"].as_string_or("1Gi")}}}};
        return true;
      },
      true);
  if (e) *err = e.message;
  return {};
}

void BuiltinControllers::setup(Manager& mgr, int workers) {
  pods_ = &mgr.informer("v1", "Pod");
  sts_rec_ = std::make_unique<EventRecorder>(c_, "statefulset-controller");
  rs_rec_ = std::make_unique<EventRecorder>(c_, "replicaset-controller");
  sts_ = std::make_shared<Controller>("statefulset", [this](const Request& r, std::string* e) { return reconcile_statefulset(r, e); }, workers);
  sts_->For(mgr.informer("apps/v1", "StatefulSet"));
  sts_->Owns(*pods_, "StatefulSet");
  mgr.add(sts_);
  rs_ = std::make_shared<Controller>("replicaset", [this](const Request& r, std::string* e) { return reconcile_replicaset(r, e); }, workers);
  rs_->For(mgr.informer("apps/v1", "ReplicaSet"));
  rs_->Owns(*pods_, "ReplicaSet");
  mgr.add(rs_);
  dep_ = std::make_shared<Controller>("deployment", [this](const Request& r, std::string* e) { return reconcile_deployment(r, e); }, workers);
  dep_->For(mgr.informer("apps/v1", "Deployment"));
  dep_->Owns(mgr.informer("apps/v1", "ReplicaSet"), "Deployment");
  mgr.add(dep_);
  pvc_ = std::make_shared<Controller>("persistentvolume-binder", [this](const Request& r, std::string* e) { return reconcile_pvc(r, e); });
  pvc_->For(mgr.informer("v1", "PersistentVolumeClaim"));
  pvc_->Watches(*pods_, [](const std::string&, const Json& p) {
    std::vector<Request> out;
    if (p.at_path({"spec", "nodeName"}).as_string().empty()) return out;
    for (const auto& v : p.at_path({"spec", "volumes"}).as_array())
      if (v.at_path({"persistentVolumeClaim", "claimName"}).is_string())
        out.push_back({p.str_at({"metadata", "namespace"}), v.at_path({"persistentVolumeClaim", "claimName"}).as_string()});
    return out;
  });
  mgr.add(pvc_);
  sa_ = std::make_shared<Controller>("serviceaccount-pull-secrets",
                                     [this](const Request& r, std::string* e) { return reconcile_service_account(r, e); });
  sa_->For(mgr.informer("v1", "ServiceAccount"));
  mgr.add(sa_);
}

// OpenShift's service-account controller gives every ServiceAccount a dockercfg pull secret; the
// ODH reconciler waits for it before releasing its reconciliation lock, so kube-lite emulates it.
Result BuiltinControllers::reconcile_service_account(const Request& r, std::string* err) {
  Json sa;
  ApiError e = c_->get("v1", "ServiceAccount", r.ns, r.name, sa);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  if (!sa["imagePullSecrets"].empty() || sa.at_path({"metadata", "deletionTimestamp"}).is_string()) return {};
  std::string sname = r.name + "-dockercfg-" + random_hex(3).substr(0, 5);
  Json sec{{"apiVersion", "v1"},
           {"kind", "Secret"},
           {"metadata", Json{{"name", sname}, {"namespace", r.ns},
                             {"annotations", Json{{"kubernetes.io/service-account.name", r.name}}}}},
           {"type", "kubernetes.io/dockercfg"},
           {"data", Json{{".dockercfg", base64_encode("{}")}}}};
  set_controller_reference(sa, sec);
  e = c_->create(sec);
  if (e && e.code != 409) {
    *err = e.message;
    return {};
  }
  e = c_->update_with_retry("v1", "ServiceAccount", r.ns, r.name, [&](Json& o) {
    if (!o["imagePullSecrets"].empty()) return false;
    o["imagePullSecrets"] = Json::array({Json{{"name", sname}}});
    o["secrets"].push_back(Json{{"name", sname}});
    return true;
  });
  if (e && e.code != 404) *err = e.message;
  return {};
}

}  // namespace kf
