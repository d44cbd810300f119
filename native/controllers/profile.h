// profile.h — N11-N15: Profile (multi-tenancy) reconciler, plugins and monitoring
// (reference components/profile-controller/controllers/{profile_controller.go,plugin_*.go,monitoring.go}).
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <string>
#include <thread>

#include "controllers/common.h"
#include "runtime/runtime.h"

namespace kf {

constexpr const char* AUTHZ_POLICY_ISTIO = "ns-owner-access-istio";
constexpr const char* KF_QUOTA = "kf-resource-quota";
constexpr const char* PROFILE_FINALIZER = "profile-finalizer";
constexpr const char* DEFAULT_EDITOR = "default-editor";
constexpr const char* DEFAULT_VIEWER = "default-viewer";
constexpr const char* KIND_WORKLOAD_IDENTITY = "WorkloadIdentity";
constexpr const char* KIND_AWS_IAM_FOR_SERVICE_ACCOUNT = "AwsIamForServiceAccount";
constexpr const char* GCP_ANNOTATION_KEY = "iam.gke.io/gcp-service-account";
constexpr const char* AWS_ANNOTATION_KEY = "eks.amazonaws.com/role-arn";
constexpr const char* WORKLOAD_IDENTITY_ROLE = "roles/iam.workloadIdentityUser";

// ---- monitoring (N14) ---------------------------------------------------------------------------
void inc_request_counter(const std::string& kind, const std::string& component = "profile-controller");
void inc_request_error_counter(const std::string& kind, const std::string& severity,
                               const std::string& component = "profile-controller");
// KFAM flavour (kfam/monitoring.go): also labels the requesting user, action and path.
void inc_request_counter_full(const std::string& component, const std::string& kind, const std::string& user,
                              const std::string& action, const std::string& path);
void inc_request_error_counter_full(const std::string& component, const std::string& kind, const std::string& user,
                                    const std::string& action, const std::string& path, const std::string& severity);
class Heartbeat {
 public:
  explicit Heartbeat(std::string component, double period_s = 10.0, std::string severity = "minor");
  ~Heartbeat();

 private:
  std::string component_, severity_;
  std::atomic<bool> run_{true};
  std::thread th_;
};

// ---- cloud IAM backend (offline: policies persisted in a ConfigMap so behaviour is observable) ---
class CloudIam {
 public:
  virtual ~CloudIam() = default;
  virtual ApiError get_role_trust_policy(const std::string& role_name, std::string& doc) = 0;
  virtual ApiError set_role_trust_policy(const std::string& role_name, const std::string& doc) = 0;
  virtual ApiError get_sa_iam_policy(const std::string& gcp_sa, Json& policy) = 0;
  virtual ApiError set_sa_iam_policy(const std::string& gcp_sa, const Json& policy) = 0;
};
std::shared_ptr<CloudIam> make_configmap_cloud_iam(std::shared_ptr<Client> c, std::string ns = "kube-system");

// AWS trust-policy document manipulation (plugin_iam.go:141-284), unit-tested
std::string get_issuer_url_from_provider_arn(const std::string& arn);
std::string get_iam_role_name_from_iam_role_arn(const std::string& arn);
// returns false with exists=true when the identity is already present (ConditionExistError)
bool add_service_account_in_assume_role_policy(const std::string& doc, const std::string& ns, const std::string& sa,
                                               std::string& out, bool* exists);
bool remove_service_account_in_assume_role_policy(const std::string& doc, const std::string& ns, const std::string& sa,
                                                  std::string& out);
std::string gcp_project_id(const std::string& gcp_service_account);
void gcp_add_binding(Json& policy, const std::string& member);
void gcp_revoke_binding(Json& policy, const std::string& member);

// Namespace label merge (profile_controller.go:754-773): empty value removes, existing keys kept.
void set_namespace_labels(Json& ns, const std::map<std::string, std::string>& labels);
std::map<std::string, std::string> parse_flat_yaml_map(const std::string& text, bool* ok = nullptr);

struct ProfileOptions {
  std::string userid_header = "kubeflow-userid";
  std::string userid_prefix = "";
  std::string workload_identity;            // default GCP SA for the WorkloadIdentity plugin
  std::string namespace_labels_path;        // hot-reloaded (inotify) like the fsnotify watch
  std::map<std::string, std::string> default_labels = {
      {"katib.kubeflow.org/metrics-collector-injection", "enabled"},
      {"serving.kubeflow.org/inferenceservice", "enabled"},
      {"pipelines.kubeflow.org/enabled", "true"},
      {"app.kubernetes.io/part-of", "kubeflow-profile"}};
  double namespace_wait_s = 15.0;  // backoff.NewConstantBackOff(3s) x 5
};

Json authorization_policy_spec(const Json& profile, const ProfileOptions& o);

class ProfileReconciler {
 public:
  ProfileReconciler(std::shared_ptr<Client> c, ProfileOptions o, std::shared_ptr<CloudIam> iam);
  ~ProfileReconciler();
  Result reconcile(const Request& r, std::string* err);
  void setup(Manager& mgr);

 private:
  std::map<std::string, std::string> read_labels();
  ApiError apply_plugins(const Json& profile, bool revoke);
  Result fail_condition(Json& profile, const std::string& msg, std::string* err);
  // reconcile's steps (profile_controller.go Reconcile, in its order). A step that fails returns the
  // error and names the request-error counter it bumps (nullptr: none)
  struct Failure {
    ApiError error;
    const char* counter = nullptr;
    explicit operator bool() const { return static_cast<bool>(error); }
  };
  // the owned namespace: created (and waited for) or relabelled; `stop` set when reconcile must
  // return `stop_result` (a failed condition) instead of going on
  Failure ensure_namespace(Json& profile, const std::map<std::string, std::string>& labels, bool* stop,
                           Result* stop_result, std::string* err);
  ApiError ensure_rolebinding(const Json& profile, const std::string& rb_name, const std::string& cluster_role,
                              const Json& subject, const Json& ann);
  Failure ensure_service_accounts(const Json& profile);
  Failure ensure_quota(const Json& profile);
  Failure ensure_default_plugins(Json& profile);
  Failure ensure_finalizer(const Json& profile);
  Failure finalize(const Json& profile);
  std::shared_ptr<Client> c_;
  ProfileOptions o_;
  std::shared_ptr<CloudIam> iam_;
  std::shared_ptr<Controller> ctl_;
  std::unique_ptr<Heartbeat> hb_;
  std::atomic<bool> watching_{false};
  std::thread watch_th_;
};

}  // namespace kf
