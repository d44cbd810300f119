// odh.h — N8 OpenshiftNotebookReconciler + N9 ODH NotebookWebhook (platform extension on the
// same Notebook CR), reference components/odh-notebook-controller/controllers/*.go.
//
// Webhook (mutating, Notebook CREATE/UPDATE):
//   CREATE: reconciliation lock kubeflow-resource-stopped=odh-notebook-controller-lock;
//   CREATE/UPDATE: image from an ImageStream in the controller namespace when
//     notebooks.opendatahub.io/last-image-selection=<stream>:<tag> (newest item's
//     dockerImageReference, JUPYTER_IMAGE env updated), trusted CA bundle mount when
//     odh-trusted-ca-bundle exists (creates workbench-trusted-ca-bundle, volume trusted-ca,
//     subPath mount at /etc/pki/tls/custom-certs/ca-bundle.crt + 5 env vars);
//   inject-oauth: oauth-proxy sidecar (:8443, probes /oauth/healthz, 100m/64Mi, volumes
//     oauth-config + tls-certificates, serviceAccountName=<nb>); denied together with service mesh;
//   UPDATE of a running notebook whose pod template the webhook itself would change: keep the old
//     template, set notebooks.opendatahub.io/update-pending=<first difference>.
// Reconciler: CA bundle configmap (PEM + DER structure validated), unmount on deletion,
//   NetworkPolicies <nb>-ctrl-np (:8888 from the controller namespace) / <nb>-oauth-np (:8443),
//   SET_PIPELINE_RBAC RoleBinding elyra-pipelines-<nb>, OAuth SA / Service <nb>-tls / Secret
//   <nb>-oauth-config / reencrypt Route, or an edge Route, then removes the reconciliation lock.
// Conscious deviations (documented): the lock is removed without the 1s/5s blocking wait when no
//   OAuth service account can ever receive a pull secret (non-OAuth notebooks); the OAuth case waits
//   by requeueing instead of sleeping in the worker; RoleBinding subject drift updates the live
//   object (the reference Updates a fresh object without resourceVersion, which always fails).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "admission/admission.h"
#include "core/json.h"
#include "runtime/runtime.h"

namespace kf {

constexpr const char* ODH_ANNOTATION_INJECT_OAUTH = "notebooks.opendatahub.io/inject-oauth";
constexpr const char* ODH_ANNOTATION_SERVICE_MESH = "opendatahub.io/service-mesh";
constexpr const char* ODH_LOCK_VALUE = "odh-notebook-controller-lock";
constexpr const char* ODH_ANNOTATION_LOGOUT_URL = "notebooks.opendatahub.io/oauth-logout-url";
constexpr const char* ODH_ANNOTATION_UPDATE_PENDING = "notebooks.opendatahub.io/update-pending";
constexpr const char* ODH_ANNOTATION_IMAGE_SELECTION = "notebooks.opendatahub.io/last-image-selection";

bool odh_bool_annotation(const Json& obj, const std::string& key);  // strconv.ParseBool semantics
bool odh_oauth_enabled(const Json& nb);
bool odh_service_mesh_enabled(const Json& nb);
bool odh_lock_enabled(const Json& nb);

// webhook pieces
void odh_inject_lock(Json& nb);
void odh_inject_oauth_proxy(Json& nb, const std::string& proxy_image);
void odh_inject_cert_config(Json& nb, const std::string& configmap);
// returns "" or an error ("invalid image selection format")
std::string odh_set_image_from_imagestreams(Json& nb, const std::vector<Json>& imagestreams);
// "{v1.PodSpec}.Containers[0].Image: a != b" (Go field names), "" when equal
std::string json_first_difference(const Json& a, const Json& b, const std::string& root_type);

// reconciler pieces
bool pem_certificate_valid(const std::string& pem);
Json odh_network_policy(const Json& nb, const std::string& controller_ns);
Json odh_oauth_network_policy(const Json& nb);
Json odh_route(const Json& nb);
Json odh_oauth_route(const Json& nb);
Json odh_service_account(const Json& nb);
Json odh_oauth_service(const Json& nb);
Json odh_oauth_secret(const Json& nb);
Json odh_role_binding(const Json& nb, const std::string& name, const std::string& kind, const std::string& role);
// UnsetNotebookCertConfig on a copy: returns true when something was removed
bool odh_unset_cert_config(Json& nb);

struct OdhOptions {
  std::string oauth_proxy_image = "registry.redhat.io/openshift4/ose-oauth-proxy:latest";
  std::string controller_namespace = "opendatahub";
  bool set_pipeline_rbac = false;  // SET_PIPELINE_RBAC
};

AdmissionFn make_odh_notebook_webhook(std::shared_ptr<Client> c, OdhOptions o);

class OdhNotebookReconciler {
 public:
  OdhNotebookReconciler(std::shared_ptr<Client> c, OdhOptions o) : c_(std::move(c)), o_(std::move(o)) {}
  Result reconcile(const Request& r, std::string* err);
  void setup(Manager& mgr, int workers = 1);

 private:
  ApiError reconcile_cert_configmap(const Json& nb, bool* skipped);
  ApiError reconcile_simple(const Json& desired, bool compare_spec);  // create-or-update by labels/spec
  Result remove_lock(const Json& nb, std::string* err);
  std::shared_ptr<Client> c_;
  OdhOptions o_;
  std::shared_ptr<Controller> ctl_;
  std::mutex lock_mu_;
  std::map<std::string, int> lock_attempts_;
};

}  // namespace kf
