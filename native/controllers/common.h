// common.h — shared pieces of the reconcilers:
//   * reconcilehelper (N7, reference common/reconcilehelper/util.go): create-or-update helpers and the
//     "copy owned fields -> needs update?" diff functions, on JSON objects;
//   * culler constants (N4, reference notebook-controller/pkg/culler/culler.go:40-47);
//   * notebook metrics (N5, reference notebook-controller/pkg/metrics/metrics.go).
#pragma once

#include <memory>
#include <string>

#include "core/json.h"
#include "core/metrics.h"
#include "runtime/runtime.h"

namespace kf {

// ---- annotation / label protocol ------------------------------------------
constexpr const char* STOP_ANNOTATION = "kubeflow-resource-stopped";
constexpr const char* LAST_ACTIVITY_ANNOTATION = "notebooks.kubeflow.org/last-activity";
constexpr const char* LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION = "notebooks.kubeflow.org/last_activity_check_timestamp";
constexpr const char* ANNOTATION_REWRITE_URI = "notebooks.kubeflow.org/http-rewrite-uri";
constexpr const char* ANNOTATION_HEADERS_REQUEST_SET = "notebooks.kubeflow.org/http-headers-request-set";
constexpr const char* ANNOTATION_NOTEBOOK_RESTART = "notebooks.opendatahub.io/notebook-restart";
constexpr const char* WORKBENCH_LABEL = "opendatahub.io/workbenches";
constexpr const char* PREFIX_ENV_VAR = "NB_PREFIX";
constexpr int DEFAULT_CONTAINER_PORT = 8888;
constexpr int DEFAULT_SERVING_PORT = 80;
constexpr int64_t DEFAULT_FS_GROUP = 100;
// MI355X additions: GPU placement + readiness-op + cold-start phases.
constexpr const char* GPU_RESOURCE = "amd.com/gpu";
constexpr const char* GPU_MEMORY_RESOURCE = "amd.com/gpu-memory";
constexpr const char* ANNOTATION_GPU_IDS = "amd.com/gpu-ids";
constexpr const char* ANNOTATION_XGMI_RING = "amd.com/xgmi-ring";
constexpr const char* ANNOTATION_GPU_READINESS = "notebooks.kubeflow.org/gpu-readiness";
// first-start phase breakdown (ms) written once on the Notebook when it is Ready (notebook.cc)
constexpr const char* ANNOTATION_COLD_START = "notebooks.kubeflow.org/cold-start-phases";

bool stop_annotation_is_set(const Json& obj);

// ---- reconcilehelper ---------------------------------------------------------------------------
// Each returns true when `to` had to be changed to match the owned fields of `from`.
bool copy_statefulset_fields(const Json& from, Json& to);
// NOTE: the reference compares the replica *pointers* and therefore always reports an
// update; this implementation compares values (conscious fix).
bool copy_deployment_fields(const Json& from, Json& to);
bool copy_service_fields(const Json& from, Json& to);  // selector + ports only, never clusterIP
bool copy_virtual_service(const Json& from, Json& to);  // whole spec

enum class CopyKind { StatefulSet, Deployment, Service, VirtualService, Generic };
// Get `desired` (by apiVersion/kind/ns/name); create it if missing, else copy the owned fields
// and update when they differ. Returns the live object in `live` (optional).
ApiError reconcile_owned(Client& c, const Json& desired, CopyKind kind, Json* live = nullptr, bool* created = nullptr);

// ---- notebook metrics ------------------------------------------------------------------------
struct NotebookMetrics {
  std::shared_ptr<CounterVec> create_total, create_failed_total, culling_total;
  std::shared_ptr<GaugeVec> last_culling_timestamp;
  // MI355X extension: first-start latency of each Notebook by phase (seconds)
  std::shared_ptr<HistogramVec> cold_start_seconds;
  // notebook_running is computed at scrape time from the StatefulSet list (metrics.go:82-99)
  static std::shared_ptr<NotebookMetrics> install(std::shared_ptr<Client> c);
};

}  // namespace kf
