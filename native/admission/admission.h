// admission.h — admission plugins of the control plane.
//
//   PodDefault (N18, reference components/admission-webhook/main.go): Pod CREATE; selects the
//     namespace's PodDefaults by label selector, rejects on any merge conflict (volumes,
//     tolerations, imagePullSecrets, env, volumeMounts (by name and by path), annotations,
//     labels, init containers, sidecars), merges everything, sets command/args when absent
//     (never on istio-proxy), and records poddefault.admission.kubeflow.org/poddefault-<name>.
//     Registered only for namespaces labelled app.kubernetes.io/part-of=kubeflow-profile
//     (manifests/base/mutating-webhook-configuration.yaml) — same gate here.
//   GPU readiness (CS6, new): Pod CREATE of a notebook pod requesting amd.com/gpu gets the
//     `gpu-readiness` init container running kfamd-readiness on the same GPUs.
//   Quota (K7, new + ResourceQuota semantics): Pod CREATE charged against the namespace's
//     ResourceQuotas, including requests./limits. amd.com/gpu and amd.com/gpu-memory (HBM GiB;
//     a pod requesting N GPUs is charged N x 288 GiB unless it states gpu-memory itself);
//     status.used is maintained by the quota controller.
//
// Each plugin is an ApiServer AdmissionFn (in-process, kflite) and can also be served as an
// HTTP AdmissionReview webhook (split binaries) through AdmissionWebhookServer.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "apiserver/apiserver.h"
#include "core/http.h"
#include "runtime/runtime.h"

namespace kf {

// ---- PodDefault (pure functions, unit-tested like admission-webhook/main_test.go) -------------
std::vector<Json> filter_pod_defaults(const std::vector<Json>& list, const Json& pod);
// Returns "" when safe, else the aggregated conflict message.
std::string safe_to_apply_pod_defaults(const Json& pod, const std::vector<Json>& pds);
void apply_pod_defaults(Json& pod, const std::vector<Json>& pds);
// mergeMap: existing + defaults; conflict -> error string
bool merge_map(const Json& existing, const std::vector<Json>& defaults, Json& out, std::string* err);
void set_command_and_args(Json& container, const std::vector<Json>& pds);

struct PodDefaultOptions {
  // namespaces selected for injection (webhook namespaceSelector); empty = all namespaces
  std::string namespace_selector = "app.kubernetes.io/part-of=kubeflow-profile";
};
AdmissionFn make_poddefault_plugin(std::shared_ptr<Client> c, PodDefaultOptions o = {});

struct GpuReadinessOptions {
  std::string image = "kfamd/readiness:gfx950";
  std::vector<std::string> args = {"--m", "4096", "--n", "4096", "--k", "4096", "--iters", "10"};
  bool only_notebooks = true;  // pods carrying the notebook-name label
  // "sidecar" (default): a native sidecar (init container, restartPolicy: Always) that shares the
  // pod's GPUs (KFAMD_SHARE_POD_GPUS; on upstream Kubernetes the equivalent is one DRA ResourceClaim
  // referenced by both containers) and gates Ready through /readyz — the op overlaps the notebook
  // server's start. "init": the r1/r2 blocking init container (device-plugin-only clusters).
  // Per pod: annotation kfamd.io/gpu-readiness-mode. Process-wide: env KFAMD_GPU_READINESS_MODE.
  std::string mode = "sidecar";
  int port = 8689;  // the sidecar's /readyz port
};
AdmissionFn make_gpu_readiness_plugin(GpuReadinessOptions o = {});

// ---- quota ----------------------------------------------------------------------------------
// usage of one pod in quota terms ("requests.cpu", "limits.memory", "requests.amd.com/gpu",
// "amd.com/gpu-memory", "pods", ...)
std::map<std::string, double> pod_quota_usage(const Json& pod, int64_t hbm_gib_per_gpu = 288);
AdmissionFn make_quota_plugin(std::shared_ptr<Client> c, int64_t hbm_gib_per_gpu = 288);
// status.used recompute for every ResourceQuota (controller)
class QuotaController {
 public:
  explicit QuotaController(std::shared_ptr<Client> c, int64_t hbm_gib_per_gpu = 288) : c_(std::move(c)), hbm_(hbm_gib_per_gpu) {}
  void setup(Manager& mgr);
  Result reconcile(const Request& r, std::string* err);

 private:
  std::shared_ptr<Client> c_;
  int64_t hbm_;
  Informer* pods_ = nullptr;
  std::shared_ptr<Controller> ctl_;
};

// ---- HTTP webhook server (split mode) --------------------------------------------------------
class AdmissionWebhookServer {
 public:
  // path -> (plugin, mutating)
  void add(const std::string& path, AdmissionFn fn, bool mutating, std::shared_ptr<const ResourceInfo> res);
  // tls != nullptr: serve HTTPS (the pair is re-read when it changes on disk)
  bool start(const std::string& addr, int port, std::string* err, const TlsServerConfig* tls = nullptr);
  void stop();
  int port() const { return srv_ ? srv_->port() : 0; }
  // Mutating + ValidatingWebhookConfiguration objects pointing at base_url (self-registration of
  // the split binaries; the reference ships them as manifests).
  // ca_pem non-empty: set as every webhook's clientConfig.caBundle (base64).
  std::vector<Json> webhook_configurations(const std::string& base_url, const std::string& name,
                                           const std::string& ca_pem = "") const;
  // Processes one AdmissionReview (exposed for tests).
  Json review(const std::string& path, const Json& admission_review);

 private:
  struct Entry {
    AdmissionFn fn;
    bool mutating;
    std::shared_ptr<const ResourceInfo> res;
  };
  std::map<std::string, Entry> routes_;
  std::unique_ptr<HttpServer> srv_;
};

}  // namespace kf
