// builtin.h — the workload controllers the reference takes from kube-controller-manager (L0):
// StatefulSet (ordinal pods <name>-<i>, OrderedReady, rolling update by controller-revision-hash,
// volumeClaimTemplates), Deployment -> ReplicaSet -> Pods (RollingUpdate / Recreate), and the
// PersistentVolumeClaim binder (hostpath provisioner; Immediate and WaitForFirstConsumer).
#pragma once

#include <memory>

#include "runtime/runtime.h"

namespace kf {

std::string pod_template_hash(const Json& template_);
bool pod_is_ready(const Json& pod);
bool pod_is_terminal(const Json& pod);

class BuiltinControllers {
 public:
  explicit BuiltinControllers(std::shared_ptr<Client> c) : c_(std::move(c)) {}
  void setup(Manager& mgr, int workers = 1);

  Result reconcile_statefulset(const Request& r, std::string* err);
  Result reconcile_deployment(const Request& r, std::string* err);
  Result reconcile_replicaset(const Request& r, std::string* err);
  Result reconcile_pvc(const Request& r, std::string* err);
  Result reconcile_service_account(const Request& r, std::string* err);

 private:
  Json make_pod(const Json& owner, const Json& tmpl, const std::string& name, const Json& extra_labels);
  std::shared_ptr<Client> c_;
  // FailedCreate / SuccessfulCreate events on the owner, as kube-controller-manager records them
  // (the notebook controller re-emits StatefulSet events onto the Notebook)
  std::unique_ptr<EventRecorder> sts_rec_, rs_rec_;
  Informer* pods_ = nullptr;
  std::shared_ptr<Controller> sts_, dep_, rs_, pvc_, sa_;
};

}  // namespace kf
