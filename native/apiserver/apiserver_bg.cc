// apiserver_bg.cc — kube-lite background controllers (ownerReference garbage collection,
// namespace lifecycle, event TTL, ClusterRole aggregation), RBAC authorization, HTTP admission
// webhooks, authentication and Service -> endpoint resolution.
#include <unistd.h>

#include <algorithm>
#include <chrono>

#include "apiserver/apiserver.h"
#include "core/util.h"

namespace kf {

// ---- background loop ----------------------------------------------------------------------------
void ApiServer::background_loop() {
  int64_t last_ttl = 0;
  while (running_) {
    {
      std::unique_lock<std::mutex> g(bg_mu_);
      bg_cv_.wait_for(g, std::chrono::milliseconds(500), [&] { return bg_kick_; });
      bg_kick_ = false;
    }
    if (!running_) break;
    try {
      gc_pass();
      namespace_pass();
      if (now_unix_ms() - last_ttl > 60000) {
        event_ttl_pass();
        last_ttl = now_unix_ms();
      }
    } catch (const std::exception& e) {
      KF_ERROR("apiserver.gc", "background pass failed", Json{{"error", e.what()}});
    }
  }
}

void ApiServer::gc_pass() {
  struct Item {
    std::shared_ptr<const ResourceInfo> res;
    std::string ns, name;
    std::string action;  // delete | orphan-strip | finalize-foreground | finalize-orphan
    std::vector<std::string> dead_owner_uids;
  };
  std::vector<Item> work;
  {
    std::lock_guard<std::mutex> g(mu_);
    // dependents index: owner uid -> list of (res key, key)
    std::map<std::string, std::vector<std::pair<std::string, std::string>>> deps;
    for (const auto& rk : data_)
      for (const auto& kv : rk.second)
        for (const auto& ref : kv.second.at_path({"metadata", "ownerReferences"}).as_array())
          deps[ref["uid"].as_string()].emplace_back(rk.first, kv.first);
    for (const auto& rk : data_) {
      auto res = [&]() -> std::shared_ptr<const ResourceInfo> {
        size_t s = rk.first.find('/');
        return reg_.by_plural(rk.first.substr(0, s), rk.first.substr(s + 1));
      }();
      if (!res) continue;
      for (const auto& kv : rk.second) {
        const Json& md = kv.second["metadata"];
        const std::string& ns = md["namespace"].as_string();
        const std::string& name = md["name"].as_string();
        // owners gone?
        const Json& refs = md["ownerReferences"];
        if (refs.is_array() && !refs.empty() && !md["deletionTimestamp"].is_string()) {
          bool any_alive = false;
          std::vector<std::string> dead;
          for (const auto& ref : refs.as_array()) {
            auto u = uid_index_.find(ref["uid"].as_string());
            if (u != uid_index_.end()) {
              // owner being deleted in the foreground still counts as alive until it finishes
              any_alive = true;
            } else {
              dead.push_back(ref["uid"].as_string());
            }
          }
          if (!any_alive) work.push_back({res, ns, name, "delete", dead});
          else if (!dead.empty()) work.push_back({res, ns, name, "strip", dead});
        }
        // foreground / orphan finalizers on objects being deleted
        if (md["deletionTimestamp"].is_string()) {
          for (const auto& f : md["finalizers"].as_array()) {
            const std::string uid = md["uid"].as_string();
            auto d = deps.find(uid);
            bool has_deps = d != deps.end() && !d->second.empty();
            if (f.as_string() == "foregroundDeletion") {
              if (!has_deps) work.push_back({res, ns, name, "finalize-foreground", {}});
              else
                for (const auto& dep : d->second) {
                  size_t s = dep.first.find('/');
                  auto dres = reg_.by_plural(dep.first.substr(0, s), dep.first.substr(s + 1));
                  size_t sl = dep.second.find('/');
                  if (dres) work.push_back({dres, dep.second.substr(0, sl), dep.second.substr(sl + 1), "delete-fg", {}});
                }
            } else if (f.as_string() == "orphan") {
              if (has_deps)
                for (const auto& dep : d->second) {
                  size_t s = dep.first.find('/');
                  auto dres = reg_.by_plural(dep.first.substr(0, s), dep.first.substr(s + 1));
                  size_t sl = dep.second.find('/');
                  if (dres) work.push_back({dres, dep.second.substr(0, sl), dep.second.substr(sl + 1), "strip", {uid}});
                }
              work.push_back({res, ns, name, "finalize-orphan", {}});
            }
          }
        }
      }
    }
  }
  WriteOptions sys;
  for (auto& w : work) {
    if (w.action == "delete" || w.action == "delete-fg") {
      DeleteOptions d;
      d.propagation = w.action == "delete-fg" ? "Foreground" : "Background";
      r_delete(w.res, w.ns, w.name, d);
    } else if (w.action == "strip") {
      Json cur;
      if (r_get(w.res, "", w.ns, w.name, cur)) continue;
      Json refs = Json::array();
      for (const auto& r : cur.at_path({"metadata", "ownerReferences"}).as_array()) {
        bool dead = std::find(w.dead_owner_uids.begin(), w.dead_owner_uids.end(), r["uid"].as_string()) != w.dead_owner_uids.end();
        if (!dead) refs.push_back(r);
      }
      if (refs.empty()) cur["metadata"].erase("ownerReferences");
      else cur["metadata"]["ownerReferences"] = refs;
      r_update(w.res, "", w.ns, w.name, cur, sys, "");
    } else {
      const char* fin = w.action == "finalize-foreground" ? "foregroundDeletion" : "orphan";
      Json cur;
      if (r_get(w.res, "", w.ns, w.name, cur)) continue;
      Json fins = Json::array();
      for (const auto& f : cur.at_path({"metadata", "finalizers"}).as_array())
        if (f.as_string() != fin) fins.push_back(f);
      cur["metadata"]["finalizers"] = fins;
      r_update(w.res, "", w.ns, w.name, cur, sys, "");
    }
  }
}

void ApiServer::namespace_pass() {
  std::vector<std::string> terminating;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& kv : data_["/namespaces"])
      if (kv.second.at_path({"metadata", "deletionTimestamp"}).is_string())
        terminating.push_back(kv.second.str_at({"metadata", "name"}));
  }
  auto ns_res = reg_.by_plural("", "namespaces");
  for (const auto& ns : terminating) {
    std::vector<std::pair<std::shared_ptr<const ResourceInfo>, std::string>> victims;
    bool remaining = false;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& rk : data_) {
        size_t s = rk.first.find('/');
        auto res = reg_.by_plural(rk.first.substr(0, s), rk.first.substr(s + 1));
        if (!res || !res->namespaced) continue;
        for (auto it = rk.second.lower_bound(ns + "/"); it != rk.second.end() && starts_with(it->first, ns + "/"); ++it) {
          remaining = true;
          if (!it->second.at_path({"metadata", "deletionTimestamp"}).is_string())
            victims.emplace_back(res, it->first.substr(ns.size() + 1));
        }
      }
    }
    for (auto& v : victims) {
      DeleteOptions d;
      d.propagation = "Background";
      r_delete(v.first, ns, v.second, d);
    }
    if (!remaining) {
      std::lock_guard<std::mutex> g(mu_);
      commit_delete(ns_res, "/" + ns);
    }
  }
}

void ApiServer::event_ttl_pass() {
  int64_t cutoff = now_unix_ms() - cfg_.event_ttl_seconds * 1000;
  std::vector<std::pair<std::string, std::string>> old;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& kv : data_["/events"]) {
      auto t = parse_rfc3339_ms(kv.second["lastTimestamp"].as_string());
      if (t && *t < cutoff) old.emplace_back(kv.second.str_at({"metadata", "namespace"}), kv.second.str_at({"metadata", "name"}));
    }
  }
  auto res = reg_.by_plural("", "events");
  for (auto& o : old) r_delete(res, o.first, o.second, DeleteOptions{});
}

// ---- RBAC -----------------------------------------------------------------------------------------
namespace {
bool match_list(const Json& list, const std::string& v) {
  for (const auto& x : list.as_array())
    if (x.as_string() == "*" || x.as_string() == v) return true;
  return false;
}
bool rule_allows(const Json& rule, const std::string& verb, const std::string& group, const std::string& resource,
                 const std::string& subresource, const std::string& name, bool non_resource) {
  if (!match_list(rule["verbs"], verb)) return false;
  if (non_resource) {
    for (const auto& u : rule["nonResourceURLs"].as_array()) {
      const std::string& p = u.as_string();
      if (p == "*" || p == resource || (ends_with(p, "*") && starts_with(resource, p.substr(0, p.size() - 1)))) return true;
    }
    return false;
  }
  if (!match_list(rule["apiGroups"], group)) return false;
  std::string full = subresource.empty() ? resource : resource + "/" + subresource;
  bool res_ok = false;
  for (const auto& r : rule["resources"].as_array()) {
    const std::string& s = r.as_string();
    if (s == "*" || s == full || (s == resource + "/*" && !subresource.empty()) || (s == "*/" + subresource && !subresource.empty()))
      res_ok = true;
  }
  if (!res_ok) return false;
  if (rule["resourceNames"].is_array() && !rule["resourceNames"].empty()) return !name.empty() && match_list(rule["resourceNames"], name);
  return true;
}
bool subject_matches(const Json& subj, const UserInfo& u) {
  const std::string& kind = subj["kind"].as_string();
  const std::string& name = subj["name"].as_string();
  if (kind == "User") return name == u.username;
  if (kind == "Group") return std::find(u.groups.begin(), u.groups.end(), name) != u.groups.end();
  if (kind == "ServiceAccount")
    return u.username == "system:serviceaccount:" + subj["namespace"].as_string() + ":" + name;
  return false;
}
}  // namespace

bool ApiServer::authorize(const UserInfo& u, const std::string& verb, const std::string& group, const std::string& resource,
                          const std::string& subresource, const std::string& ns, const std::string& name, std::string* reason) {
  if (std::find(u.groups.begin(), u.groups.end(), "system:masters") != u.groups.end()) {
    if (reason) *reason = "system:masters";
    return true;
  }
  bool non_resource = !resource.empty() && resource[0] == '/';
  std::lock_guard<std::mutex> g(mu_);
  auto rules_of = [&](const std::string& kind, const std::string& rns, const std::string& rname) -> Json {
    const std::string rk = kind == "ClusterRole" ? "rbac.authorization.k8s.io/clusterroles" : "rbac.authorization.k8s.io/roles";
    auto& m = data_[rk];
    auto it = m.find((kind == "ClusterRole" ? "" : rns) + "/" + rname);
    return it == m.end() ? Json::array() : it->second["rules"];
  };
  for (const auto& kv : data_["rbac.authorization.k8s.io/clusterrolebindings"]) {
    const Json& b = kv.second;
    bool subj = false;
    for (const auto& s : b["subjects"].as_array()) subj = subj || subject_matches(s, u);
    if (!subj) continue;
    const Json rules = rules_of("ClusterRole", "", b.str_at({"roleRef", "name"}));
    for (const auto& rule : rules.as_array())
      if (rule_allows(rule, verb, group, resource, subresource, name, non_resource)) {
        if (reason) *reason = "RBAC: allowed by ClusterRoleBinding \"" + b.str_at({"metadata", "name"}) + "\"";
        return true;
      }
  }
  if (!ns.empty()) {
    auto& rbs = data_["rbac.authorization.k8s.io/rolebindings"];
    for (auto it = rbs.lower_bound(ns + "/"); it != rbs.end() && starts_with(it->first, ns + "/"); ++it) {
      const Json& b = it->second;
      bool subj = false;
      for (const auto& s : b["subjects"].as_array()) subj = subj || subject_matches(s, u);
      if (!subj) continue;
      const Json rules = rules_of(b.str_at({"roleRef", "kind"}), ns, b.str_at({"roleRef", "name"}));
      for (const auto& rule : rules.as_array())
        if (rule_allows(rule, verb, group, resource, subresource, name, non_resource)) {
          if (reason) *reason = "RBAC: allowed by RoleBinding \"" + b.str_at({"metadata", "name"}) + "/" + ns + "\"";
          return true;
        }
    }
  }
  if (reason) *reason = "";
  return false;
}

void ApiServer::aggregate_clusterroles() {
  std::vector<Json> updates;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& roles = data_["rbac.authorization.k8s.io/clusterroles"];
    for (const auto& kv : roles) {
      const Json& agg = kv.second["aggregationRule"];
      if (!agg.is_object()) continue;
      Json rules = Json::array();
      for (const auto& sel : agg["clusterRoleSelectors"].as_array()) {
        LabelSelector ls = LabelSelector::from_json(sel, true);
        for (const auto& kv2 : roles) {
          if (kv2.first == kv.first) continue;
          if (!ls.matches(kv2.second.at_path({"metadata", "labels"}))) continue;
          for (const auto& r : kv2.second["rules"].as_array()) {
            bool dup = false;
            for (const auto& x : rules.as_array()) dup = dup || x == r;
            if (!dup) rules.push_back(r);
          }
        }
      }
      if (kv.second["rules"] != rules) {
        Json u = kv.second;
        u["rules"] = rules;
        updates.push_back(u);
      }
    }
  }
  auto res = reg_.by_plural("rbac.authorization.k8s.io", "clusterroles");
  for (auto& u : updates) {
    std::string name = u.str_at({"metadata", "name"});
    std::lock_guard<std::mutex> g(mu_);
    commit_put(res, "/" + name, u, "MODIFIED");
  }
}

void ApiServer::bootstrap_rbac() {
  auto cr = [](const std::string& name, Json rules, Json labels = Json(), Json agg = Json()) {
    Json o{{"apiVersion", "rbac.authorization.k8s.io/v1"}, {"kind", "ClusterRole"}, {"metadata", Json{{"name", name}}}};
    if (labels.is_object()) o["metadata"]["labels"] = labels;
    o["rules"] = rules;
    if (agg.is_array()) o["aggregationRule"] = Json{{"clusterRoleSelectors", agg}};
    return o;
  };
  auto rule = [](std::vector<std::string> groups, std::vector<std::string> res, std::vector<std::string> verbs) {
    Json g = Json::array(), r = Json::array(), v = Json::array();
    for (auto& x : groups) g.push_back(x);
    for (auto& x : res) r.push_back(x);
    for (auto& x : verbs) v.push_back(x);
    return Json{{"apiGroups", g}, {"resources", r}, {"verbs", v}};
  };
  const std::vector<std::string> rw = {"get", "list", "watch", "create", "update", "patch", "delete", "deletecollection"};
  const std::vector<std::string> ro = {"get", "list", "watch"};
  std::vector<Json> roles = {
      cr("cluster-admin", Json::array({Json{{"apiGroups", Json::array({"*"})}, {"resources", Json::array({"*"})}, {"verbs", Json::array({"*"})}},
                                       Json{{"nonResourceURLs", Json::array({"*"})}, {"verbs", Json::array({"*"})}}})),
      cr("admin", Json::array({rule({"", "apps", "networking.k8s.io", "rbac.authorization.k8s.io"},
                                    {"*"}, rw)}), Json{{"rbac.authorization.k8s.io/aggregate-to-admin", "true"}}),
      cr("edit", Json::array({rule({"", "apps", "networking.k8s.io"},
                                   {"pods", "pods/log", "services", "configmaps", "secrets", "persistentvolumeclaims", "events",
                                    "statefulsets", "deployments", "replicasets", "serviceaccounts", "networkpolicies"},
                                   rw)})),
      cr("view", Json::array({rule({"", "apps", "networking.k8s.io"},
                                   {"pods", "pods/log", "services", "configmaps", "persistentvolumeclaims", "events",
                                    "statefulsets", "deployments", "replicasets", "serviceaccounts", "networkpolicies"},
                                   ro)})),
      // kubeflow/manifests aggregation roots (the reference binds profiles to these, §2.5)
      cr("kubeflow-admin", Json::array(), Json(),
         Json::array({Json{{"matchLabels", Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-admin", "true"}}}}})),
      cr("kubeflow-edit", Json::array(), Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-admin", "true"}},
         Json::array({Json{{"matchLabels", Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-edit", "true"}}}}})),
      cr("kubeflow-view", Json::array(), Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-edit", "true"}},
         Json::array({Json{{"matchLabels", Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-view", "true"}}}}})),
      cr("kubeflow-kubernetes-admin",
         Json::array({rule({"", "apps", "rbac.authorization.k8s.io", "networking.k8s.io"}, {"*"}, rw)}),
         Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-admin", "true"}}),
      cr("kubeflow-kubernetes-edit",
         Json::array({rule({"", "apps", "networking.k8s.io"},
                           {"pods", "pods/log", "pods/attach", "pods/exec", "services", "configmaps", "secrets",
                            "persistentvolumeclaims", "events", "statefulsets", "deployments", "replicasets",
                            "serviceaccounts"},
                           rw),
                      rule({"storage.k8s.io"}, {"storageclasses"}, ro)}),
         Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-edit", "true"}}),
      cr("kubeflow-kubernetes-view",
         Json::array({rule({"", "apps"},
                           {"pods", "pods/log", "services", "configmaps", "persistentvolumeclaims", "events",
                            "statefulsets", "deployments", "replicasets", "namespaces", "nodes"},
                           ro),
                      rule({"storage.k8s.io"}, {"storageclasses"}, ro)}),
         Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-view", "true"}}),
      // notebook-controller/config/rbac/user_cluster_roles.yaml equivalents
      cr("kubeflow-notebooks-admin", Json::array(),
         Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-admin", "true"}},
         Json::array({Json{{"matchLabels", Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-notebooks-admin", "true"}}}}})),
      cr("kubeflow-notebooks-edit",
         Json::array({rule({"kubeflow.org"}, {"notebooks", "notebooks/status", "poddefaults", "pvcviewers"}, rw),
                      rule({"tensorboard.kubeflow.org"}, {"tensorboards", "tensorboards/status"}, rw)}),
         Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-edit", "true"},
              {"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-notebooks-admin", "true"}}),
      cr("kubeflow-notebooks-view",
         Json::array({rule({"kubeflow.org"}, {"notebooks", "notebooks/status", "poddefaults", "pvcviewers"}, ro),
                      rule({"tensorboard.kubeflow.org"}, {"tensorboards", "tensorboards/status"}, ro)}),
         Json{{"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-view", "true"}}),
  };
  WriteOptions sys;
  for (auto& r : roles) {
    Json existing;
    if (get("rbac.authorization.k8s.io/v1", "ClusterRole", "", r.str_at({"metadata", "name"}), existing).ok()) continue;
    create(r, sys);
  }
  Json crb{{"apiVersion", "rbac.authorization.k8s.io/v1"}, {"kind", "ClusterRoleBinding"},
           {"metadata", Json{{"name", "cluster-admin"}}},
           {"roleRef", Json{{"apiGroup", "rbac.authorization.k8s.io"}, {"kind", "ClusterRole"}, {"name", "cluster-admin"}}},
           {"subjects", Json::array({Json{{"apiGroup", "rbac.authorization.k8s.io"}, {"kind", "Group"}, {"name", "system:masters"}}})}};
  Json existing;
  if (!get("rbac.authorization.k8s.io/v1", "ClusterRoleBinding", "", "cluster-admin", existing).ok()) create(crb, sys);
  aggregate_clusterroles();
}

// ---- authentication ---------------------------------------------------------------------------
bool ApiServer::authenticate_token(const std::string& token, UserInfo& out) const {
  auto it = cfg_.tokens.find(token);
  if (it != cfg_.tokens.end()) {
    out = it->second;
    return true;
  }
  SaToken t;
  {
    std::lock_guard<std::mutex> g(tok_mu_);
    auto st = sa_tokens_.find(token);
    if (st == sa_tokens_.end()) return false;
    t = st->second;
  }
  if (t.expires < static_cast<double>(now_unix_ms()) / 1000.0) return false;
  Json sa;
  // bound to the ServiceAccount object: deleting (or re-creating) it invalidates the token
  if (!const_cast<ApiServer*>(this)->get("v1", "ServiceAccount", t.ns, t.name, sa).ok() ||
      sa.str_at({"metadata", "uid"}) != t.uid)
    return false;
  out.username = "system:serviceaccount:" + t.ns + ":" + t.name;
  out.groups = {"system:serviceaccounts", "system:serviceaccounts:" + t.ns, "system:authenticated"};
  return true;
}

ApiError ApiServer::issue_sa_token(const std::string& ns, const std::string& sa_name, int64_t expiration_s,
                                   std::string& token, double& expires_unix) {
  Json sa;
  ApiError e = get("v1", "ServiceAccount", ns, sa_name, sa);
  if (e) return e;
  expiration_s = std::min<int64_t>(std::max<int64_t>(expiration_s, 600), 48 * 3600);
  token = "kfsa." + secure_random_hex(24);
  expires_unix = static_cast<double>(now_unix_ms()) / 1000.0 + static_cast<double>(expiration_s);
  std::lock_guard<std::mutex> g(tok_mu_);
  const double now = static_cast<double>(now_unix_ms()) / 1000.0;
  for (auto it = sa_tokens_.begin(); it != sa_tokens_.end();) it = it->second.expires < now ? sa_tokens_.erase(it) : std::next(it);
  sa_tokens_[token] = SaToken{ns, sa_name, sa.str_at({"metadata", "uid"}), expires_unix};
  return {};
}

bool ApiServer::authenticate(const HttpRequest& req, UserInfo& out) const {
  std::string auth = req.header("Authorization");
  if (starts_with(auth, "Bearer ")) {
    if (!authenticate_token(auth.substr(7), out)) return false;
  } else if (!cfg_.tokens.empty() && cfg_.authz_rbac) {
    out = UserInfo{"system:anonymous", {"system:unauthenticated"}};
  } else {
    out = UserInfo{};
  }
  // impersonation (allowed for masters only)
  std::string imp = req.header("Impersonate-User");
  if (!imp.empty() && std::find(out.groups.begin(), out.groups.end(), "system:masters") != out.groups.end()) {
    UserInfo u;
    u.username = imp;
    u.groups = {"system:authenticated"};
    for (const auto& g : split(req.header("Impersonate-Group"), ',', true)) u.groups.push_back(trim(g));
    out = u;
  }
  return true;
}

// ---- HTTP admission webhooks ------------------------------------------------------------------
ApiError ApiServer::call_webhooks(AdmissionAttrs& a, bool mutating) {
  const std::string rk = mutating ? "admissionregistration.k8s.io/mutatingwebhookconfigurations"
                                  : "admissionregistration.k8s.io/validatingwebhookconfigurations";
  std::vector<Json> configs;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = data_.find(rk);
    if (it == data_.end()) return {};
    for (const auto& kv : it->second) configs.push_back(kv.second);
  }
  Json ns_obj;
  if (!a.ns.empty()) r_get(reg_.by_plural("", "namespaces"), "", "", a.ns, ns_obj);
  for (const auto& cfg : configs) {
    for (const auto& wh : cfg["webhooks"].as_array()) {
      bool match = false;
      for (const auto& rule : wh["rules"].as_array()) {
        if (!match_list(rule["operations"], a.operation)) continue;
        if (!match_list(rule["apiGroups"], a.res->group)) continue;
        std::string full = a.subresource.empty() ? a.res->plural : a.res->plural + "/" + a.subresource;
        if (!match_list(rule["resources"], full)) continue;
        match = true;
      }
      if (!match) continue;
      if (wh["namespaceSelector"].is_object() && !a.ns.empty() &&
          !LabelSelector::from_json(wh["namespaceSelector"]).matches(ns_obj.at_path({"metadata", "labels"})))
        continue;
      const Json& target = a.object ? *a.object : (a.old_object ? *a.old_object : Json());
      if (wh["objectSelector"].is_object() &&
          !LabelSelector::from_json(wh["objectSelector"]).matches(target.at_path({"metadata", "labels"})))
        continue;
      std::string url = wh.at_path({"clientConfig", "url"}).as_string();
      const std::string ca_b64 = wh.at_path({"clientConfig", "caBundle"}).as_string();
      if (url.empty() && wh.at_path({"clientConfig", "service"}).is_object()) {
        // kube-apiserver calls service webhooks over HTTPS; kube-lite keeps plain HTTP for a
        // service webhook registered without a caBundle (development manifests)
        const Json& svc = wh.at_path({"clientConfig", "service"});
        url = std::string(ca_b64.empty() ? "http://" : "https://") + svc["name"].as_string() + "." +
              svc["namespace"].as_string() + ".svc:" + std::to_string(svc["port"].as_int(443)) + svc["path"].as_string();
      }
      TlsClientOptions tls;
      if (!ca_b64.empty()) tls.ca_pem = base64_decode(ca_b64);
      const std::string uid = uuid4();
      Json review{{"apiVersion", "admission.k8s.io/v1"}, {"kind", "AdmissionReview"},
                  {"request", Json{{"uid", uid},
                                   {"kind", Json{{"group", a.res->group}, {"version", a.version}, {"kind", a.res->kind}}},
                                   {"resource", Json{{"group", a.res->group}, {"version", a.version}, {"resource", a.res->plural}}},
                                   {"subResource", a.subresource},
                                   {"name", a.name},
                                   {"namespace", a.ns},
                                   {"operation", a.operation},
                                   {"userInfo", Json{{"username", a.user ? a.user->username : ""}}},
                                   {"object", a.object ? *a.object : Json()},
                                   {"oldObject", a.old_object ? *a.old_object : Json()},
                                   {"dryRun", a.dry_run}}}};
      int timeout = static_cast<int>(wh["timeoutSeconds"].as_int(10)) * 1000;
      const double t0 = now_seconds();
      HttpResult r = http_request("POST", url, review.dump(), {{"Content-Type", "application/json"}}, timeout,
                                  ca_b64.empty() ? nullptr : &tls);
      bool fail_closed = wh["failurePolicy"].as_string_or("Fail") != "Ignore";
      Json resp;
      const bool parsed = r.ok() && Json::try_parse(r.body, resp);
      const bool rejected = !parsed ? fail_closed : !resp.at_path({"response", "allowed"}).as_bool();
      admission_latency(true)->observe({wh["name"].as_string(), a.operation, mutating ? "admit" : "validate",
                                        rejected ? "true" : "false"}, now_seconds() - t0);
      if (!parsed) {
        if (fail_closed)
          return ApiError::Internal("Internal error occurred: failed calling webhook \"" + wh["name"].as_string() +
                                    "\": " + (r.error.empty() ? "HTTP " + std::to_string(r.status) : r.error));
        continue;
      }
      const Json& rr = resp["response"];
      if (!rr["allowed"].as_bool()) {
        std::string msg = rr.at_path({"status", "message"}).as_string();
        int code = static_cast<int>(rr.at_path({"status", "code"}).as_int(403));
        return ApiError{code, "Forbidden", "admission webhook \"" + wh["name"].as_string() + "\" denied the request: " + msg};
      }
      if (mutating && a.object && rr["patch"].is_string()) {
        Json ops;
        if (Json::try_parse(base64_decode(rr["patch"].as_string()), ops)) {
          try {
            *a.object = apply_json_patch(*a.object, ops);
          } catch (const JsonError& e) {
            if (fail_closed) return ApiError::Internal(std::string("webhook patch failed: ") + e.what());
          }
        }
      }
    }
  }
  return {};
}

// ---- service resolution -----------------------------------------------------------------------
bool ApiServer::resolve_service(const std::string& host, int port, std::string& ip, int& out_port) {
  // <svc>.<ns>.svc.<domain> | <svc>.<ns>.svc | <svc>.<ns>
  auto parts = split(host, '.');
  if (parts.size() < 2) return false;
  if (parts.size() > 2 && parts[2] != "svc") return false;
  if (host == "localhost" || starts_with(host, "127.")) return false;
  const std::string svc = parts[0], ns = parts[1];
  Json s;
  if (r_get(reg_.by_plural("", "services"), "", ns, svc, s)) return false;
  // map service port -> targetPort
  Json target = Json();
  for (const auto& p : s.at_path({"spec", "ports"}).as_array())
    if (p["port"].as_int() == port || s.at_path({"spec", "ports"}).size() == 1) target = p["targetPort"];
  if (target.is_null()) target = port;
  LabelSelector sel = LabelSelector::from_json(Json{{"matchLabels", s.at_path({"spec", "selector"})}}, true);
  if (s.at_path({"spec", "selector"}).empty()) return false;
  Json pods;
  ListOptions lo;
  r_list(reg_.by_plural("", "pods"), "", ns, lo, pods);
  for (const auto& p : pods["items"].as_array()) {
    if (!sel.matches(p.at_path({"metadata", "labels"}))) continue;
    if (p.at_path({"metadata", "deletionTimestamp"}).is_string()) continue;
    const std::string& pip = p.at_path({"status", "podIP"}).as_string();
    if (pip.empty()) continue;
    bool ready = false;
    for (const auto& c : p.at_path({"status", "conditions"}).as_array())
      if (c["type"].as_string() == "Ready" && c["status"].as_string() == "True") ready = true;
    if (!ready) continue;
    int tp = 0;
    if (target.is_number()) {
      tp = static_cast<int>(target.as_int());
    } else {
      for (const auto& c : p.at_path({"spec", "containers"}).as_array())
        for (const auto& cp : c["ports"].as_array())
          if (cp["name"].as_string() == target.as_string()) tp = static_cast<int>(cp["containerPort"].as_int());
    }
    if (tp == 0) continue;
    ip = pip;
    out_port = tp;
    return true;
  }
  return false;
}

}  // namespace kf
