// tensorboard.h — N16 Tensorboard reconciler + N17 PVCViewer reconciler and admission (defaulting +
// validation) webhooks.
//
// Tensorboard (reference components/tensorboard-controller/controllers/tensorboard_controller.go):
//   Deployment <name> running TENSORBOARD_IMAGE `tensorboard --logdir=<path> --bind_all` on :6006,
//   Service :80 -> 6006, VirtualService /tensorboard/<ns>/<name>/ (rewrite "/", timeout 300s),
//   logspath forms pvc://<pvc>/<sub> | gs:// (user-gcp-sa secret) | s3:// | /cns/ | legacy tb-volume,
//   RWO_PVC_SCHEDULING preferred node affinity to the node of a *running* pod that mounts the PVC
//   (pod field index spec.volumes.persistentvolumeclaim.claimname), status appends a condition when
//   the deployment's first condition type changes and mirrors readyReplicas.
//   Deployment update copies only labels / replicas / affinity (tensorboard CopyDeploymentSetFields).
//
// PVCViewer (reference components/pvcviewer-controller/{controllers,api/v1alpha1}):
//   defaulting: empty podSpec -> DEFAULT_POD_SPEC_PATH file or a filebrowser container on :8080 with
//   FB_BASEURL=<basePrefix>/<ns>/<name>/; then the `viewer-volume` PVC volume is appended.
//   validation: pvc set, podSpec set, podSpec mounts the pvc.
//   reconcile: Deployment pvcviewer-<name> (Recreate, app.kubernetes.io/{name,instance,part-of}),
//   Service + VirtualService only when spec.networking is set, status {ready, url, conditions}.
//   RWO affinity computed only at Deployment creation. Conscious fix vs reference: several pods on
//   the *same* node no longer suppress the affinity (the reference gives up as if they were on
//   different nodes).
#pragma once

#include <memory>
#include <string>

#include "admission/admission.h"
#include "core/json.h"
#include "runtime/runtime.h"

namespace kf {

// ---- Tensorboard pure helpers (unit-tested) ----------------------------------------------------
bool tb_is_cloud_path(const std::string& p);
bool tb_is_gcs_path(const std::string& p);
bool tb_is_pvc_path(const std::string& p);
std::string tb_extract_pvc_name(const std::string& p);
std::string tb_extract_pvc_subpath(const std::string& p);
// affinity: {} or a preferred node affinity to `node`
Json preferred_node_affinity(const std::string& node);
Json tb_generate_deployment(const Json& tb, const std::string& image, const Json& affinity);
Json tb_generate_service(const Json& tb);
Json tb_generate_virtual_service(const Json& tb, const std::string& gateway, const std::string& host);
bool tb_copy_deployment_fields(const Json& from, Json& to);
// status transition: appends a condition when the deployment's first condition type changed
Json tb_status(const Json& tb, const Json& deployment);

struct TensorboardOptions {
  std::string image = "tensorflow/tensorflow:2.5.1";  // TENSORBOARD_IMAGE
  std::string istio_gateway = "kubeflow/kubeflow-gateway";
  std::string istio_host = "*";
  bool rwo_pvc_scheduling = false;  // RWO_PVC_SCHEDULING
  static TensorboardOptions from_env(std::string* err = nullptr);
};

class TensorboardReconciler {
 public:
  TensorboardReconciler(std::shared_ptr<Client> c, TensorboardOptions o) : c_(std::move(c)), o_(std::move(o)) {}
  Result reconcile(const Request& r, std::string* err);
  void setup(Manager& mgr, int workers = 1);

 private:
  Json node_affinity_for_pvc(const std::string& ns, const std::string& pvc, std::string* err);
  std::shared_ptr<Client> c_;
  TensorboardOptions o_;
  Informer* pods_ = nullptr;
  std::shared_ptr<Controller> ctl_;
};

// ---- PVCViewer --------------------------------------------------------------------------------
constexpr const char* PVCVIEWER_PREFIX = "pvcviewer-";
Json pvcviewer_default(const Json& viewer, const Json& default_pod_spec);  // defaulting webhook
std::string pvcviewer_validate(const Json& viewer);                       // "" when valid
Json pvcviewer_common_labels(const Json& viewer);
Json pvcviewer_generate_deployment(const Json& viewer, const Json& affinity);
Json pvcviewer_generate_service(const Json& viewer);
Json pvcviewer_generate_virtual_service(const Json& viewer, const std::string& gateway);
// node of the (single) non-viewer pod mounting the RWO pvc, or "" (omit affinity)
std::string pvcviewer_rwo_node(const Json& pvc, const std::vector<Json>& pods);

// DEFAULT_POD_SPEC_PATH (YAML/JSON podSpec) is read per request like the reference.
AdmissionFn make_pvcviewer_defaulter();
AdmissionFn make_pvcviewer_validator();

class PVCViewerReconciler {
 public:
  explicit PVCViewerReconciler(std::shared_ptr<Client> c) : c_(std::move(c)) {}
  Result reconcile(const Request& r, std::string* err);
  void setup(Manager& mgr, int workers = 1);

 private:
  ApiError reconcile_status(const std::string& ns, const std::string& name);
  std::shared_ptr<Client> c_;
  std::shared_ptr<Controller> ctl_;
};

}  // namespace kf
