// notebook.h — N2 NotebookReconciler, N3 CullingReconciler (reference
// components/notebook-controller/controllers/{notebook_controller.go,culling_controller.go}).
#pragma once

#include <functional>
#include <map>
#include <mutex>

#include <memory>
#include <string>

#include "controllers/common.h"
#include "runtime/runtime.h"

namespace kf {

struct NotebookOptions {
  bool use_istio = false;             // USE_ISTIO
  std::string istio_gateway = "kubeflow/kubeflow-gateway";  // ISTIO_GATEWAY
  std::string istio_host = "*";       // ISTIO_HOST
  std::string cluster_domain = "cluster.local";  // CLUSTER_DOMAIN
  bool add_fsgroup = true;            // ADD_FSGROUP (unset or "true")
  static NotebookOptions from_env();
};

// Pure functions (unit-tested like notebook_controller_test.go).
Json generate_statefulset(const Json& nb, const NotebookOptions& o);
Json generate_service(const Json& nb);
Json generate_virtual_service(const Json& nb, const NotebookOptions& o);
std::string virtual_service_name(const std::string& name, const std::string& ns);
Json pod_cond_to_notebook_cond(const Json& pod_cond);
// createNotebookStatus: readyReplicas from the STS, containerState of the container named like
// the notebook, mirrored pod conditions. Q9 note: the reference only adopts a containerState that
// differs from the previous one; this keeps the previous state instead of dropping it.
Json create_notebook_status(const Json& nb, const Json& sts, const Json& pod);
// nbNameFromInvolvedObject: StatefulSet -> its name; Pod -> its "notebook-name" label.
bool nb_name_from_involved_object(Client& c, const Json& involved, std::string& out);

class NotebookReconciler {
 public:
  NotebookReconciler(std::shared_ptr<Client> c, NotebookOptions o, std::shared_ptr<NotebookMetrics> m);
  Result reconcile(const Request& req, std::string* err);
  void setup(Manager& mgr, int workers = 1);
  std::shared_ptr<Controller> controller() { return ctl_; }

 private:
  Result reemit_event(const Json& event, std::string* err);
  void track_cold_start(const Json& nb, const Json& pod, const Json& status);
  std::shared_ptr<Client> c_;
  NotebookOptions o_;
  std::shared_ptr<NotebookMetrics> m_;
  std::unique_ptr<EventRecorder> rec_;
  std::shared_ptr<Controller> ctl_;
  // first-start tracking, by Notebook uid: when the controller first saw it, when it created the
  // StatefulSet (process-local clock; a restarted controller simply skips in-flight notebooks)
  struct ColdStart {
    double seen = 0, sts = 0;
  };
  std::mutex cs_mu_;
  std::map<std::string, ColdStart> cold_;
};

struct CullingOptions {
  int64_t cull_idle_minutes = 1440;  // CULL_IDLE_TIME
  int64_t check_period_minutes = 1;  // IDLENESS_CHECK_PERIOD
  bool dev = false;                  // DEV: go through the apiserver service proxy (kubectl proxy style)
  std::string proxy_url = "http://localhost:8001";  // KUBE_PROXY_URL (DEV mode)
  std::string cluster_domain = "cluster.local";
  double period_seconds_override = -1;  // tests: sub-minute periods
  // Through the mesh (the gateway's in-cluster listener, node/node.h): the kernels GET goes to
  // mesh_url with Host <nb>.<ns>.svc.<domain> and the culler's ServiceAccount token, so the
  // profile's ns-owner-access-istio policy admits it as the notebook-controller principal
  // (profile_controller.go:419-556, the "*/api/kernels" rule). MESH_URL / MESH_TOKEN_FILE in split
  // mode; kflite wires both in-process. Only for mesh members (istio-injection=enabled): elsewhere
  // the GET goes straight to the Service, from the controller's own namespace.
  std::string mesh_url;
  std::string mesh_token_file;
  std::function<std::string()> mesh_url_fn, peer_token_fn;
  static CullingOptions from_env();
  double period_seconds() const { return period_seconds_override > 0 ? period_seconds_override : check_period_minutes * 60.0; }
};

// Culler helpers (unit-tested like culling_controller_test.go).
bool all_kernels_are_idle(const Json& kernels);
std::string notebook_recent_time(const std::vector<std::string>& times);  // "" on parse error
bool update_timestamp_from_kernels_activity(Json& meta_annotations, const Json& kernels);
bool update_timestamp_from_terminals_activity(Json& meta_annotations, const Json& terminals);
bool notebook_is_idle(const Json& nb, int64_t cull_idle_minutes, int64_t now_ms);
bool culling_check_period_has_passed(const Json& nb, double period_s, int64_t now_ms);
void set_stop_annotation(Json& nb, NotebookMetrics* m);

class CullingReconciler {
 public:
  CullingReconciler(std::shared_ptr<Client> c, CullingOptions o, std::shared_ptr<NotebookMetrics> m);
  Result reconcile(const Request& req, std::string* err);
  void setup(Manager& mgr);
  std::shared_ptr<Controller> controller() { return ctl_; }

 private:
  bool fetch(const std::string& nm, const std::string& ns, const std::string& what, Json& out);
  std::shared_ptr<Client> c_;
  CullingOptions o_;
  std::shared_ptr<NotebookMetrics> m_;
  std::shared_ptr<Controller> ctl_;
};

}  // namespace kf
