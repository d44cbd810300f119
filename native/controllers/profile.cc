// profile.cc — N12 ProfileReconciler, N13 plugins, N14 monitoring (see profile.h).
#include "controllers/profile.h"

#include <sys/inotify.h>
#include <poll.h>
#include <unistd.h>

#include <algorithm>

#include "core/util.h"

namespace kf {

// ---- monitoring ---------------------------------------------------------------------------------
namespace {
std::string trunc30(const std::string& s) { return s.size() > 30 ? s.substr(0, 30) : s; }
}  // namespace

// One family per metric name for the whole process (kflite hosts profile controller + KFAM):
// the label set is the union of both components' (monitoring.go of each), unused ones empty.
namespace {
std::shared_ptr<CounterVec> request_family() {
  static auto c = Registry::global().counter("request_kf", "Number of request_counter",
                                             {"component", "kind", "request_user", "action", "path"});
  return c;
}
std::shared_ptr<CounterVec> request_failure_family() {
  static auto c = Registry::global().counter("request_kf_failure", "Number of request_failure_counter",
                                             {"component", "kind", "request_user", "action", "path", "severity"});
  return c;
}
}  // namespace

void inc_request_counter(const std::string& kind, const std::string& component) {
  request_family()->inc({component, trunc30(kind), "", "", ""});
}
void inc_request_error_counter(const std::string& kind, const std::string& severity, const std::string& component) {
  request_failure_family()->inc({component, trunc30(kind), "", "", "", severity});
}
void inc_request_counter_full(const std::string& component, const std::string& kind, const std::string& user,
                              const std::string& action, const std::string& path) {
  request_family()->inc({component, trunc30(kind), user, action, path});
}
void inc_request_error_counter_full(const std::string& component, const std::string& kind, const std::string& user,
                                    const std::string& action, const std::string& path, const std::string& severity) {
  request_failure_family()->inc({component, trunc30(kind), user, action, path, severity});
}
Heartbeat::Heartbeat(std::string component, double period_s, std::string severity)
    : component_(std::move(component)), severity_(std::move(severity)) {
  static auto hb = Registry::global().counter("service_heartbeat", "Heartbeat signal every 10 seconds", {"component", "severity"});
  th_ = std::thread([this, period_s] {
    while (run_) {
      hb->inc({component_, severity_});
      for (int i = 0; i < static_cast<int>(period_s * 10) && run_; ++i) ::usleep(100000);
    }
  });
}
Heartbeat::~Heartbeat() {
  run_ = false;
  if (th_.joinable()) th_.join();
}

// ---- YAML flat map / namespace labels ----------------------------------------------------------------
std::map<std::string, std::string> parse_flat_yaml_map(const std::string& text, bool* ok) {
  std::map<std::string, std::string> out;
  bool good = true;
  for (auto line : split(text, '\n')) {
    size_t hash = std::string::npos;
    bool in_s = false, in_d = false;
    for (size_t i = 0; i < line.size(); ++i) {
      if (line[i] == '\'' && !in_d) in_s = !in_s;
      if (line[i] == '"' && !in_s) in_d = !in_d;
      if (line[i] == '#' && !in_s && !in_d && (i == 0 || std::isspace(static_cast<unsigned char>(line[i - 1])))) {
        hash = i;
        break;
      }
    }
    if (hash != std::string::npos) line = line.substr(0, hash);
    line = trim(line);
    if (line.empty() || line == "---") continue;
    size_t colon = line.find(": ");
    if (colon == std::string::npos && ends_with(line, ":")) colon = line.size() - 1;
    if (colon == std::string::npos) {
      good = false;
      continue;
    }
    std::string k = trim(line.substr(0, colon)), v = trim(line.substr(colon + 1));
    auto unq = [](std::string s) {
      if (s.size() >= 2 && ((s.front() == '"' && s.back() == '"') || (s.front() == '\'' && s.back() == '\'')))
        return s.substr(1, s.size() - 2);
      return s;
    };
    out[unq(k)] = unq(v);
  }
  if (ok) *ok = good;
  return out;
}

void set_namespace_labels(Json& ns, const std::map<std::string, std::string>& labels) {
  Json& l = ns["metadata"]["labels"];
  if (!l.is_object()) l = Json::object();
  for (const auto& kv : labels) {
    const bool exists = l.has(kv.first);
    if (kv.second.empty()) {
      if (exists) l.erase(kv.first);
    } else if (!exists) {
      l[kv.first] = kv.second;
    }
  }
}

// ---- AWS / GCP plugin helpers ------------------------------------------------------------------------
std::string get_issuer_url_from_provider_arn(const std::string& arn) {
  size_t p = arn.find('/');
  return p == std::string::npos ? arn : arn.substr(p + 1);
}
std::string get_iam_role_name_from_iam_role_arn(const std::string& arn) {
  size_t p = arn.rfind('/');
  return p == std::string::npos ? arn : arn.substr(p + 1);
}

namespace {
Json make_assume_role_doc(const std::string& provider_arn, const Json& condition) {
  Json stmt{{"Effect", "Allow"}, {"Action", "sts:AssumeRoleWithWebIdentity"},
            {"Principal", Json{{"Federated", provider_arn}}}, {"Condition", condition}};
  return Json{{"Version", "2012-10-17"}, {"Statement", Json::array({stmt})}};
}
}  // namespace

bool add_service_account_in_assume_role_policy(const std::string& doc, const std::string& ns, const std::string& sa,
                                               std::string& out, bool* exists) {
  if (exists) *exists = false;
  Json d;
  if (!Json::try_parse(doc, d)) return false;
  const std::string provider = d["Statement"][0].at_path({"Principal", "Federated"}).as_string();
  const std::string issuer = get_issuer_url_from_provider_arn(provider);
  const std::string key = issuer + ":sub";
  const std::string trust = "system:serviceaccount:" + ns + ":" + sa;
  Json ids = Json::array();
  const Json& cur = d["Statement"][0].at_path({"Condition", "StringEquals"})[key];
  std::vector<Json> existing;
  if (cur.is_array()) existing.assign(cur.as_array().begin(), cur.as_array().end());
  else if (cur.is_string()) existing.push_back(cur);
  for (const auto& i : existing) {
    if (i.as_string() == trust) {
      out = doc;
      if (exists) *exists = true;
      return false;
    }
    ids.push_back(i);
  }
  ids.push_back(trust);
  Json cond{{"StringEquals", Json{{issuer + ":aud", Json::array({"sts.amazonaws.com"})}, {key, ids}}}};
  out = make_assume_role_doc(provider, cond).dump();
  return true;
}

bool remove_service_account_in_assume_role_policy(const std::string& doc, const std::string& ns, const std::string& sa,
                                                  std::string& out) {
  Json d;
  if (!Json::try_parse(doc, d)) return false;
  const std::string provider = d["Statement"][0].at_path({"Principal", "Federated"}).as_string();
  const std::string issuer = get_issuer_url_from_provider_arn(provider);
  const std::string key = issuer + ":sub";
  const std::string trust = "system:serviceaccount:" + ns + ":" + sa;
  Json ids = Json::array();
  const Json& cur = d["Statement"][0].at_path({"Condition", "StringEquals"})[key];
  std::vector<Json> existing;
  if (cur.is_array()) existing.assign(cur.as_array().begin(), cur.as_array().end());
  else if (cur.is_string()) existing.push_back(cur);
  for (const auto& i : existing)
    if (i.as_string() != trust) ids.push_back(i);
  Json se{{issuer + ":aud", Json::array({"sts.amazonaws.com"})}};
  if (!ids.empty()) se[key] = ids;  // never emit a null list (would break the policy)
  out = make_assume_role_doc(provider, Json{{"StringEquals", se}}).dump();
  return true;
}

std::string gcp_project_id(const std::string& gsa) {
  // <name>@<project>.iam.gserviceaccount.com -> <project>
  const size_t at = gsa.find('@');
  std::string project = at == std::string::npos ? "" : gsa.substr(at + 1);
  const size_t dot = project.find('.');
  return dot == std::string::npos ? project : project.substr(0, dot);
}

void gcp_add_binding(Json& policy, const std::string& member) {
  policy["bindings"].push_back(Json{{"role", WORKLOAD_IDENTITY_ROLE}, {"members", Json::array({member})}});
}
void gcp_revoke_binding(Json& policy, const std::string& member) {
  for (auto& b : policy["bindings"].mut_array()) {
    if (b["role"].as_string() != WORKLOAD_IDENTITY_ROLE) continue;
    Json m = Json::array();
    for (const auto& x : b["members"].as_array())
      if (x.as_string() != member) m.push_back(x);
    b["members"] = m;
  }
}

namespace {
class ConfigMapCloudIam : public CloudIam {
 public:
  ConfigMapCloudIam(std::shared_ptr<Client> c, std::string ns) : c_(std::move(c)), ns_(std::move(ns)) {}
  ApiError get_role_trust_policy(const std::string& role, std::string& doc) override { return get("aws-role-" + role, doc); }
  ApiError set_role_trust_policy(const std::string& role, const std::string& doc) override { return set("aws-role-" + role, doc); }
  ApiError get_sa_iam_policy(const std::string& sa, Json& policy) override {
    std::string s;
    ApiError e = get("gcp-sa-" + sanitize(sa), s);
    if (e.code == 404) {
      policy = Json{{"bindings", Json::array()}};
      return {};
    }
    if (!e) Json::try_parse(s, policy);
    return e;
  }
  ApiError set_sa_iam_policy(const std::string& sa, const Json& policy) override { return set("gcp-sa-" + sanitize(sa), policy.dump()); }

 private:
  static std::string sanitize(std::string s) {
    for (auto& ch : s)
      if (!std::isalnum(static_cast<unsigned char>(ch)) && ch != '-' && ch != '.') ch = '-';
    return to_lower(s);
  }
  ApiError get(const std::string& key, std::string& out) {
    Json cm;
    ApiError e = c_->get("v1", "ConfigMap", ns_, "kfamd-cloud-iam", cm);
    if (e) return e;
    const Json& v = cm["data"][key];
    if (!v.is_string()) return ApiError::NotFound("iam policy", key);
    out = v.as_string();
    return {};
  }
  ApiError set(const std::string& key, const std::string& val) {
    Json cm;
    ApiError e = c_->get("v1", "ConfigMap", ns_, "kfamd-cloud-iam", cm);
    if (e.code == 404) {
      cm = Json{{"apiVersion", "v1"}, {"kind", "ConfigMap"}, {"metadata", Json{{"name", "kfamd-cloud-iam"}, {"namespace", ns_}}},
                {"data", Json{{key, val}}}};
      return c_->create(cm);
    }
    if (e) return e;
    return c_->update_with_retry("v1", "ConfigMap", ns_, "kfamd-cloud-iam", [&](Json& o) {
      o["data"][key] = val;
      return true;
    });
  }
  std::shared_ptr<Client> c_;
  std::string ns_;
};
}  // namespace

std::shared_ptr<CloudIam> make_configmap_cloud_iam(std::shared_ptr<Client> c, std::string ns) {
  return std::make_shared<ConfigMapCloudIam>(std::move(c), std::move(ns));
}

// ---- AuthorizationPolicy -----------------------------------------------------------------------
Json authorization_policy_spec(const Json& profile, const ProfileOptions& o) {
  const std::string nb_principal = getenv_or("NOTEBOOK_CONTROLLER_PRINCIPAL", "cluster.local/ns/kubeflow/sa/notebook-controller-service-account");
  const std::string igw = getenv_or("ISTIO_INGRESS_GATEWAY_PRINCIPAL", "cluster.local/ns/istio-system/sa/istio-ingressgateway-service-account");
  const std::string kfp = getenv_or("KFP_UI_PRINCIPAL", "cluster.local/ns/kubeflow/sa/ml-pipeline-ui");
  const std::string owner = profile.at_path({"spec", "owner", "name"}).as_string();
  return Json{
      {"action", "ALLOW"},
      {"rules",
       Json::array({
           Json{{"when", Json::array({Json{{"key", "request.headers[" + o.userid_header + "]"},
                                           {"values", Json::array({o.userid_prefix + owner})}}})},
                {"from", Json::array({Json{{"source", Json{{"principals", Json::array({igw, kfp})}}}}})}},
           Json{{"when", Json::array({Json{{"key", "source.namespace"}, {"values", Json::array({profile.str_at({"metadata", "name"})})}}})}},
           Json{{"to", Json::array({Json{{"operation", Json{{"paths", Json::array({"/healthz", "/metrics", "/wait-for-drain"})}}}}})}},
           Json{{"from", Json::array({Json{{"source", Json{{"principals", Json::array({nb_principal})}}}}})},
                {"to", Json::array({Json{{"operation", Json{{"methods", Json::array({"GET"})}, {"paths", Json::array({"*/api/kernels"})}}}}})}},
       })}};
}

// ---- reconciler -------------------------------------------------------------------------------------
ProfileReconciler::ProfileReconciler(std::shared_ptr<Client> c, ProfileOptions o, std::shared_ptr<CloudIam> iam)
    : c_(std::move(c)), o_(std::move(o)), iam_(std::move(iam)) {}

ProfileReconciler::~ProfileReconciler() {
  watching_ = false;
  if (watch_th_.joinable()) watch_th_.join();
}

std::map<std::string, std::string> ProfileReconciler::read_labels() {
  if (o_.namespace_labels_path.empty()) return o_.default_labels;
  std::string text;
  if (!read_file(o_.namespace_labels_path, text)) {
    // Q5 deviation: the reference os.Exit(1)s the controller; we keep running on the defaults.
    KF_ERROR("profile-controller", "namespace labels properties file doesn't exist; using defaults",
             Json{{"path", o_.namespace_labels_path}});
    return o_.default_labels;
  }
  bool ok = true;
  auto m = parse_flat_yaml_map(text, &ok);
  if (!ok) KF_ERROR("profile-controller", "Unable to parse default namespace labels (partially applied)");
  return m;
}

Result ProfileReconciler::fail_condition(Json& profile, const std::string& msg, std::string* err) {
  Json& conds = profile["status"]["conditions"];
  for (const auto& c : conds.as_array())
    if (c["type"].as_string() == "Failed" && c["message"].as_string() == msg) return {};
  conds.push_back(Json{{"type", "Failed"}, {"message", msg}});
  ApiError e = c_->update_status(profile);
  if (e) *err = e.message;
  return {};
}

ApiError ProfileReconciler::apply_plugins(const Json& profile, bool revoke) {
  const std::string ns = profile.str_at({"metadata", "name"});
  for (const auto& p : profile.at_path({"spec", "plugins"}).as_array()) {
    const std::string kind = p["kind"].as_string();
    const Json& spec = p["spec"];
    if (kind == KIND_WORKLOAD_IDENTITY) {
      const std::string gsa = spec["gcpServiceAccount"].as_string();
      ApiError e = c_->update_with_retry("v1", "ServiceAccount", ns, DEFAULT_EDITOR, [&](Json& sa) {
        if (revoke) return sa["metadata"]["annotations"].erase(GCP_ANNOTATION_KEY);
        if (annotation(sa, GCP_ANNOTATION_KEY) == gsa) return false;
        set_annotation(sa, GCP_ANNOTATION_KEY, gsa);
        return true;
      });
      if (e && e.code != 404) return e;
      // IAM binding on the GCP service account: <project>.svc.id.goog[ns/default-editor]
      const std::string project = gcp_project_id(gsa);
      const std::string member = "serviceAccount:" + project + ".svc.id.goog[" + ns + "/" + DEFAULT_EDITOR + "]";
      Json policy;
      e = iam_->get_sa_iam_policy(gsa, policy);
      if (e) return e;
      if (revoke) {
        gcp_revoke_binding(policy, member);
      } else {
        bool have = false;
        for (const auto& b : policy["bindings"].as_array())
          for (const auto& m : b["members"].as_array()) have = have || (b["role"].as_string() == WORKLOAD_IDENTITY_ROLE && m.as_string() == member);
        if (!have) gcp_add_binding(policy, member);
      }
      e = iam_->set_sa_iam_policy(gsa, policy);
      if (e) return e;
    } else if (kind == KIND_AWS_IAM_FOR_SERVICE_ACCOUNT) {
      const std::string role = spec["awsIamRole"].as_string();
      ApiError e = c_->update_with_retry("v1", "ServiceAccount", ns, DEFAULT_EDITOR, [&](Json& sa) {
        if (revoke) return sa["metadata"]["annotations"].erase(AWS_ANNOTATION_KEY);
        if (annotation(sa, AWS_ANNOTATION_KEY) == role) return false;
        set_annotation(sa, AWS_ANNOTATION_KEY, role);
        return true;
      });
      if (e && e.code != 404) return e;
      if (spec["annotateOnly"].as_bool()) continue;
      std::string doc;
      const std::string role_name = get_iam_role_name_from_iam_role_arn(role);
      e = iam_->get_role_trust_policy(role_name, doc);
      if (e.code == 404) continue;  // role unknown to the (offline) IAM backend
      if (e) return e;
      std::string out;
      bool exists = false;
      bool changed = revoke ? remove_service_account_in_assume_role_policy(doc, ns, DEFAULT_EDITOR, out)
                            : add_service_account_in_assume_role_policy(doc, ns, DEFAULT_EDITOR, out, &exists);
      if (changed && out != doc) {
        e = iam_->set_role_trust_policy(role_name, out);
        if (e) return e;
      }
    } else {
      KF_INFO("profile-controller", "Plugin not recgonized: " + kind);
    }
  }
  return {};
}

namespace {
bool has_finalizer(const Json& o, const char* fin) {
  for (const auto& f : o.at_path({"metadata", "finalizers"}).as_array())
    if (f.as_string() == fin) return true;
  return false;
}
}  // namespace

ProfileReconciler::Failure ProfileReconciler::ensure_namespace(Json& profile, const std::map<std::string, std::string>& labels,
                                                               bool* stop, Result* stop_result, std::string* err) {
  const std::string name = profile.str_at({"metadata", "name"});
  const std::string owner = profile.at_path({"spec", "owner", "name"}).as_string();
  Json ns{{"apiVersion", "v1"}, {"kind", "Namespace"},
          {"metadata", Json{{"name", name}, {"annotations", Json{{"owner", owner}}}, {"labels", Json{{"istio-injection", "enabled"}}}}}};
  set_namespace_labels(ns, labels);
  set_controller_reference(profile, ns);
  Json found;
  ApiError e = c_->get("v1", "Namespace", "", name, found);
  if (e.code == 404) {
    KF_INFO("profile-controller", "Creating Namespace: " + name);
    Json n = ns;
    e = c_->create(n);
    if (e) return {e, "error creating namespace"};
    // wait for completion (constant backoff, 5 x 3 s in the reference)
    const double deadline = now_seconds() + o_.namespace_wait_s;
    while (c_->get("v1", "Namespace", "", name, found)) {
      if (now_seconds() > deadline) {
        inc_request_error_counter("error namespace create completion", "major");
        *stop = true;
        *stop_result = fail_condition(profile, "Owning namespace failed to create within 15 seconds", err);
        return {};
      }
      ::usleep(50000);
    }
    return {};
  }
  if (e) return {e, nullptr};
  if (!(annotation(found, "owner") == owner && has_annotation(found, "owner"))) {
    inc_request_counter("reject profile taking over existing namespace");
    *stop = true;
    *stop_result = fail_condition(profile, "namespace already exist, but not owned by profile creator " + owner, err);
    return {};
  }
  Json updated = found;
  set_namespace_labels(updated, labels);
  if (updated.at_path({"metadata", "labels"}) != found.at_path({"metadata", "labels"})) return {c_->update(updated), nullptr};
  return {};
}

ApiError ProfileReconciler::ensure_rolebinding(const Json& profile, const std::string& rb_name, const std::string& cluster_role,
                                               const Json& subject, const Json& ann) {
  const std::string ns = profile.str_at({"metadata", "name"});
  Json rb{{"apiVersion", "rbac.authorization.k8s.io/v1"}, {"kind", "RoleBinding"},
          {"metadata", Json{{"name", rb_name}, {"namespace", ns}}},
          {"roleRef", Json{{"apiGroup", "rbac.authorization.k8s.io"}, {"kind", "ClusterRole"}, {"name", cluster_role}}},
          {"subjects", Json::array({subject})}};
  if (ann.is_object()) rb["metadata"]["annotations"] = ann;
  set_controller_reference(profile, rb);
  Json cur;
  ApiError ge = c_->get("rbac.authorization.k8s.io/v1", "RoleBinding", ns, rb_name, cur);
  if (ge.code == 404) return c_->create(rb);
  if (ge) return ge;
  if (cur["roleRef"] == rb["roleRef"] && cur["subjects"] == rb["subjects"]) return ApiError{};
  cur["roleRef"] = rb["roleRef"];
  cur["subjects"] = rb["subjects"];
  return c_->update(cur);
}

// default-editor / default-viewer ServiceAccounts, each bound to its kubeflow-edit / -view role
ProfileReconciler::Failure ProfileReconciler::ensure_service_accounts(const Json& profile) {
  const std::string ns = profile.str_at({"metadata", "name"});
  for (auto sa_role : {std::make_pair(DEFAULT_EDITOR, "kubeflow-edit"), std::make_pair(DEFAULT_VIEWER, "kubeflow-view")}) {
    Json sa{{"apiVersion", "v1"}, {"kind", "ServiceAccount"}, {"metadata", Json{{"name", sa_role.first}, {"namespace", ns}}}};
    set_controller_reference(profile, sa);
    Json cur;
    ApiError ge = c_->get("v1", "ServiceAccount", ns, sa_role.first, cur);
    if (ge.code == 404) ge = c_->create(sa);
    if (ge) return {ge, "error updating ServiceAccount"};
    ge = ensure_rolebinding(profile, sa_role.first, sa_role.second,
                            Json{{"kind", "ServiceAccount"}, {"name", sa_role.first}, {"namespace", ns}}, Json());
    if (ge) return {ge, nullptr};
  }
  return {};
}

// spec.resourceQuotaSpec as the namespace's kf-resource-quota (removed when the spec has none)
ProfileReconciler::Failure ProfileReconciler::ensure_quota(const Json& profile) {
  const std::string ns = profile.str_at({"metadata", "name"});
  const Json& rq = profile.at_path({"spec", "resourceQuotaSpec"});
  if (!(rq["hard"].is_object() && !rq["hard"].empty())) {
    ApiError de = c_->remove("v1", "ResourceQuota", ns, KF_QUOTA);
    if (de && de.code != 404) return {de, nullptr};
    return {};
  }
  Json q{{"apiVersion", "v1"}, {"kind", "ResourceQuota"}, {"metadata", Json{{"name", KF_QUOTA}, {"namespace", ns}}}, {"spec", rq}};
  set_controller_reference(profile, q);
  Json cur;
  ApiError ge = c_->get("v1", "ResourceQuota", ns, KF_QUOTA, cur);
  if (ge.code == 404) {
    ge = c_->create(q);
  } else if (!ge && cur["spec"] != rq) {
    cur["spec"] = rq;
    ge = c_->update(cur);
  }
  if (ge) return {ge, "error updating resource quota"};
  return {};
}

// the default WorkloadIdentity plugin (Q5 fix: the Profile is written only when one is added)
ProfileReconciler::Failure ProfileReconciler::ensure_default_plugins(Json& profile) {
  if (o_.workload_identity.empty()) return {};
  for (const auto& p : profile.at_path({"spec", "plugins"}).as_array())
    if (p["kind"].as_string() == KIND_WORKLOAD_IDENTITY) return {};
  profile["spec"]["plugins"].push_back(Json{{"kind", KIND_WORKLOAD_IDENTITY}, {"spec", Json{{"gcpServiceAccount", o_.workload_identity}}}});
  ApiError e = c_->update(profile);
  if (e) return {e, "error patching DefaultPluginSpec"};
  return {};
}

ProfileReconciler::Failure ProfileReconciler::ensure_finalizer(const Json& profile) {
  if (has_finalizer(profile, PROFILE_FINALIZER)) return {};
  ApiError e = c_->update_with_retry("kubeflow.org/v1", "Profile", "", profile.str_at({"metadata", "name"}), [](Json& o) {
    if (has_finalizer(o, PROFILE_FINALIZER)) return false;
    o["metadata"]["finalizers"].push_back(PROFILE_FINALIZER);
    return true;
  });
  if (e) return {e, "error updating finalizer"};
  return {};
}

// deletion: revoke the plugins, then drop the finalizer (the namespace goes with its owner reference)
ProfileReconciler::Failure ProfileReconciler::finalize(const Json& profile) {
  if (!has_finalizer(profile, PROFILE_FINALIZER)) return {};
  ApiError e = apply_plugins(profile, true);
  if (e) return {e, "error revoking plugin"};
  e = c_->update_with_retry("kubeflow.org/v1", "Profile", "", profile.str_at({"metadata", "name"}), [](Json& o) {
    Json fins = Json::array();
    for (const auto& f : o.at_path({"metadata", "finalizers"}).as_array())
      if (f.as_string() != PROFILE_FINALIZER) fins.push_back(f);
    o["metadata"]["finalizers"] = fins;
    return true;
  });
  if (e) return {e, "error removing finalizer"};
  return {};
}

Result ProfileReconciler::reconcile(const Request& r, std::string* err) {
  auto labels = read_labels();
  Json profile;
  ApiError e = c_->get("kubeflow.org/v1", "Profile", "", r.name, profile);
  if (e.code == 404) {
    inc_request_counter("profile deletion");
    return {};
  }
  if (e) {
    inc_request_error_counter("error reading the profile object", "major");
    *err = e.message;
    return {};
  }
  auto failed = [&](const Failure& f) {
    if (f.counter) inc_request_error_counter(f.counter, "major");
    *err = f.error.message;
    return Result{};
  };
  if (profile.at_path({"metadata", "deletionTimestamp"}).is_string()) {
    if (Failure f = finalize(profile)) return failed(f);
    inc_request_counter("reconcile");
    return {};
  }
  // 1. namespace
  bool stop = false;
  Result stop_result;
  if (Failure f = ensure_namespace(profile, labels, &stop, &stop_result, err)) return failed(f);
  if (stop) return stop_result;
  // 2. the owner's Istio AuthorizationPolicy
  const std::string name = profile.str_at({"metadata", "name"});
  const std::string owner = profile.at_path({"spec", "owner", "name"}).as_string();
  Json ap{{"apiVersion", "security.istio.io/v1beta1"}, {"kind", "AuthorizationPolicy"},
          {"metadata", Json{{"name", AUTHZ_POLICY_ISTIO}, {"namespace", name}, {"annotations", Json{{"user", owner}, {"role", "admin"}}}}},
          {"spec", authorization_policy_spec(profile, o_)}};
  set_controller_reference(profile, ap);
  if ((e = reconcile_owned(*c_, ap, CopyKind::Generic))) return failed({e, "error updating Istio AuthorizationPolicy permission"});
  // 3. ServiceAccounts + their RoleBindings, 4. the owner's RoleBinding "namespaceAdmin"
  if (Failure f = ensure_service_accounts(profile)) return failed(f);
  if ((e = ensure_rolebinding(profile, "namespaceAdmin", "kubeflow-admin", profile.at_path({"spec", "owner"}),
                              Json{{"user", owner}, {"role", "admin"}})))
    return failed({e, "error updating Owner Rolebinding"});
  // 5. ResourceQuota, 6. default plugins, 7. plugins, 8. finalizer
  if (Failure f = ensure_quota(profile)) return failed(f);
  if (Failure f = ensure_default_plugins(profile)) return failed(f);
  if ((e = apply_plugins(profile, false))) return failed({e, "error applying plugin"});
  if (Failure f = ensure_finalizer(profile)) return failed(f);
  inc_request_counter("reconcile");
  return {};
}

void ProfileReconciler::setup(Manager& mgr) {
  hb_ = std::make_unique<Heartbeat>("profile-controller");
  ctl_ = std::make_shared<Controller>("profile-controller", [this](const Request& r, std::string* e) { return reconcile(r, e); });
  Informer& profiles = mgr.informer("kubeflow.org/v1", "Profile");
  ctl_->For(profiles);
  ctl_->Owns(mgr.informer("v1", "Namespace"), "Profile");
  ctl_->Owns(mgr.informer("security.istio.io/v1beta1", "AuthorizationPolicy"), "Profile");
  ctl_->Owns(mgr.informer("v1", "ServiceAccount"), "Profile");
  ctl_->Owns(mgr.informer("rbac.authorization.k8s.io/v1", "RoleBinding"), "Profile");
  mgr.add(ctl_);
  // fsnotify equivalent: inotify on the labels file -> re-enqueue every Profile
  if (!o_.namespace_labels_path.empty()) {
    watching_ = true;
    Informer* pinf = &profiles;
    watch_th_ = std::thread([this, pinf] {
      int fd = ::inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
      int wd = -1;
      int64_t last_mtime = file_mtime_ns(o_.namespace_labels_path);
      while (watching_) {
        if (fd >= 0 && wd < 0) wd = ::inotify_add_watch(fd, o_.namespace_labels_path.c_str(), IN_MODIFY | IN_CLOSE_WRITE | IN_DELETE_SELF | IN_MOVE_SELF);
        bool fire = false;
        if (fd >= 0) {
          pollfd p{fd, POLLIN, 0};
          if (::poll(&p, 1, 200) > 0) {
            char buf[4096];
            ssize_t n = ::read(fd, buf, sizeof buf);
            for (ssize_t i = 0; i < n;) {
              auto* ev = reinterpret_cast<inotify_event*>(buf + i);
              if (ev->mask & (IN_DELETE_SELF | IN_MOVE_SELF | IN_IGNORED)) {
                ::inotify_rm_watch(fd, wd);
                wd = -1;  // re-add (editors replace files)
              }
              fire = true;
              i += static_cast<ssize_t>(sizeof(inotify_event) + ev->len);
            }
          }
        } else {
          ::usleep(500000);
        }
        int64_t m = file_mtime_ns(o_.namespace_labels_path);
        if (m != last_mtime) {
          last_mtime = m;
          fire = true;
        }
        if (fire)
          for (const auto& p : pinf->list()) ctl_->enqueue({"", p.str_at({"metadata", "name"})});
      }
      if (fd >= 0) ::close(fd);
    });
  }
}

}  // namespace kf
