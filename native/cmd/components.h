// components.h — wiring of every control-plane component onto a Manager (shared by kflite and
// the split per-component binaries).
#pragma once

#include <memory>
#include <set>
#include <string>
#include <vector>

#include "apiserver/apiserver.h"
#include "core/util.h"
#include "runtime/runtime.h"

namespace kf {

struct ComponentFlags {
  // kubelet / node
  std::string node_name = "mi355x-node-0";
  int64_t gpus = -1;  // -1 = discover from KFD sysfs (or KFAMD_FAKE_GPUS)
  int64_t node_cpus = 0;  // advertised node CPU capacity (0 = online host CPUs)
  int64_t node_memory_gib = 0;  // advertised node memory (0 = host RAM)
  std::string repo_root;  // where kubeflow_rm_amd lives (pod "image" recipes run from here)
  std::string python = "python3";
  double restart_backoff = 10.0;
  std::string pod_cidr_prefix = "127.20";
  std::string sysfs_root;  // GPU discovery root ("" = /sys)
  bool numa_pinning = true;
  bool pod_zygote = true;
  bool pod_warm_gpus = true;
  std::string pod_netns = "auto";  // per-pod network namespaces (node/netns.h)
  std::string image_recipes;
  // gateway (Istio ingress equivalent)
  std::string gateway_addr = "127.0.0.1";
  int64_t gateway_port = 0;
  std::string gateway_name = "kubeflow/kubeflow-gateway";
  bool gateway_authz = true;                  // enforce AuthorizationPolicies at the gateway
  std::string gateway_trusted_proxy_secret_file;  // authn proxy in front of the ingress (see GatewayOptions)
  int64_t mesh_port = 0;                      // in-cluster (mesh) listener: -1 off, 0 ephemeral
  // KFAM
  int64_t kfam_port = -1;  // -1 = disabled unless "kfam" is enabled (then ephemeral)
  std::string userid_header = "kubeflow-userid";
  std::string userid_prefix = "";
  std::string cluster_admin = "";
  // profile controller
  std::string namespace_labels_path;
  std::string workload_identity;  // default GCP service account for the WorkloadIdentity plugin
  // odh
  std::string oauth_proxy_image = "registry.redhat.io/openshift4/ose-oauth-proxy:latest";
  std::string controller_namespace = "opendatahub";
  // admission webhooks as HTTP(S) services (split mode); in kflite they run in-process
  int64_t webhook_port = -1;
  std::string webhook_host = "127.0.0.1";
  // controller-runtime layout: <dir>/tls.crt + tls.key (+ ca.crt for the registered caBundle);
  // explicit files override it (admission-webhook's --tlsCertFile / --tlsKeyFile)
  std::string webhook_cert_dir = "/tmp/k8s-webhook-server/serving-certs";
  std::string webhook_cert_file, webhook_key_file, webhook_ca_file;
  std::string webhook_tls = "auto";  // auto (TLS when the pair exists) | on | off

  void register_flags(Flags& f);
};

class Components {
 public:
  Components(ComponentFlags f, std::shared_ptr<Client> c, ApiServer* local_api, std::string api_url, std::string data_dir);
  ~Components();
  bool setup(Manager& mgr, const std::set<std::string>& enabled, int workers, std::string* err);
  void start();
  void stop();
  int gateway_port() const;
  int mesh_port() const;
  int kfam_port() const;
  int webhook_port() const;

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
};

}  // namespace kf
