// components.cc — see cmd/components.h.
#include "cmd/components.h"

#include <unistd.h>

#include "admission/admission.h"
#include "controllers/builtin.h"
#include "controllers/odh.h"
#include "controllers/profile.h"
#include "controllers/tensorboard.h"
#include "kfam/kfam.h"
#include "controllers/notebook.h"
#include "node/node.h"
#include "core/util.h"

namespace kf {

void ComponentFlags::register_flags(Flags& f) {
  f.add_string("node-name", &node_name, "mi355x-node-0", "kubelet node name");
  f.add_int("gpus", &gpus, -1, "GPUs advertised by the device plugin (-1 = discover from KFD sysfs / KFAMD_FAKE_GPUS)");
  f.add_int("node-cpus", &node_cpus, 0, "node CPU capacity advertised by the kubelet (0 = online host CPUs)");
  f.add_int("node-memory-gib", &node_memory_gib, 0, "node memory capacity advertised by the kubelet (0 = host RAM)");
  f.add_string("repo-root", &repo_root, "", "framework root used by pod image recipes (default: derived from the binary path)");
  f.add_string("python", &python, "python3", "python interpreter for pod image recipes");
  f.add_double("restart-backoff", &restart_backoff, 10.0, "base container restart back-off in seconds");
  f.add_string("pod-cidr-prefix", &pod_cidr_prefix, "127.20", "pod IPs are allocated as <prefix>.x.y (loopback)");
  f.add_string("sysfs-root", &sysfs_root, "", "sysfs root for GPU / PCI / NUMA discovery (default /sys)");
  f.add_bool("numa-pinning", &numa_pinning, true, "pin GPU pods to their GPUs' NUMA-local CPUs");
  f.add_string("image-recipes", &image_recipes, "",
               "JSON list of extra image recipes ({match, argv, passArgs, zygote}) tried before the built-in ones");
  f.add_bool("pod-zygote", &pod_zygote, true,
             "fork Python pod containers from a pre-imported interpreter per image recipe (torch preloaded; "
             "a container whose recipe has none, or that the zygote refuses, starts a fresh interpreter)");
  f.add_bool("pod-warm-gpus", &pod_warm_gpus, true,
             "keep one warm child per GPU in torch zygotes (HIP + device context initialised before a 1-GPU pod "
             "on that GPU starts)");
  f.add_string("pod-netns", &pod_netns, "auto",
               "per-pod network namespaces: auto (when the node can create them), on (required), off");
  f.add_string("gateway-address", &gateway_addr, "127.0.0.1", "ingress gateway bind address");
  f.add_int("gateway-port", &gateway_port, 0, "ingress gateway port (0 = ephemeral)");
  f.add_string("gateway-name", &gateway_name, "kubeflow/kubeflow-gateway", "VirtualService gateway served by the ingress");
  f.add_bool("gateway-authz", &gateway_authz, true,
             "enforce Istio AuthorizationPolicies (ALLOW/DENY) on the ingress and mesh listeners");
  f.add_string("gateway-trusted-proxy-secret-file", &gateway_trusted_proxy_secret_file, "",
               "secret an authenticating proxy in front of the ingress presents (X-Kfamd-Auth-Proxy-Secret) "
               "to assert the userid header");
  f.add_int("mesh-port", &mesh_port, 0, "in-cluster mesh listener port (-1 = off, 0 = ephemeral)");
  f.add_int("kfam-port", &kfam_port, -1, "KFAM port (-1 = ephemeral when kfam is enabled)");
  f.add_string("userid-header", &userid_header, "kubeflow-userid", "user id header (KFAM / profile controller)");
  f.add_string("userid-prefix", &userid_prefix, "", "user id prefix (KFAM / profile controller)");
  f.add_string("cluster-admin", &cluster_admin, "", "KFAM cluster admin user");
  f.add_string("namespace-labels-path", &namespace_labels_path, "", "profile controller namespace labels file");
  f.add_string("workload-identity", &workload_identity, "", "default GCP service account for the WorkloadIdentity plugin");
  f.add_string("oauth-proxy-image", &oauth_proxy_image, "registry.redhat.io/openshift4/ose-oauth-proxy:latest", "ODH oauth proxy image");
  f.add_string("controller-namespace", &controller_namespace, "opendatahub", "ODH controller namespace");
  f.add_int("webhook-port", &webhook_port, -1, "serve admission webhooks on this port (-1 = in-process only)");
  f.add_string("webhook-host", &webhook_host, "127.0.0.1", "webhook server bind address");
  f.add_string("webhook-cert-dir", &webhook_cert_dir, "/tmp/k8s-webhook-server/serving-certs",
               "directory holding tls.crt / tls.key (and ca.crt) for the webhook server");
  f.add_string("webhook-tls-cert-file", &webhook_cert_file, "", "webhook serving certificate (overrides --webhook-cert-dir)");
  f.add_string("webhook-tls-key-file", &webhook_key_file, "", "webhook serving key (overrides --webhook-cert-dir)");
  f.add_string("webhook-ca-file", &webhook_ca_file, "", "CA bundle registered as the webhooks' caBundle (default: <dir>/ca.crt, else the serving certificate)");
  f.add_string("webhook-tls", &webhook_tls, "auto", "auto (HTTPS when the certificate pair exists) | on | off");
}

struct Components::Impl {
  ComponentFlags f;
  std::shared_ptr<Client> c;
  ApiServer* api;
  std::string api_url, data_dir;
  std::shared_ptr<NotebookMetrics> nb_metrics;
  std::unique_ptr<NotebookReconciler> notebook;
  std::unique_ptr<CullingReconciler> culler;
  std::unique_ptr<BuiltinControllers> builtin;
  std::unique_ptr<Scheduler> scheduler;
  std::unique_ptr<Kubelet> kubelet;
  std::unique_ptr<Gateway> gateway;
  std::unique_ptr<ProfileReconciler> profile;
  std::unique_ptr<QuotaController> quota;
  std::unique_ptr<TensorboardReconciler> tensorboard;
  std::unique_ptr<PVCViewerReconciler> pvcviewer;
  std::unique_ptr<KfamService> kfam;
  std::unique_ptr<OdhNotebookReconciler> odh;
  std::unique_ptr<AdmissionWebhookServer> webhooks;
  std::vector<std::function<void()>> starters, stoppers;

  // one unit per component group (Components::setup runs them in this order)
  void setup_notebook(Manager& mgr, const std::set<std::string>& enabled, int workers);
  CullingOptions culler_options(const std::set<std::string>& enabled);
  void setup_admission(Manager& mgr);
  bool setup_apps(Manager& mgr, const std::set<std::string>& enabled, int workers, std::string* err);
  void setup_kubelet(Manager& mgr);
  bool setup_gateway(Manager& mgr, std::string* err);
  bool start_webhook_server(const std::set<std::string>& enabled, std::string* err);
  std::vector<std::string> node_endpoints() const;
};

Components::Components(ComponentFlags f, std::shared_ptr<Client> c, ApiServer* local_api, std::string api_url,
                       std::string data_dir)
    : impl_(std::make_unique<Impl>()) {
  impl_->f = std::move(f);
  impl_->c = std::move(c);
  impl_->api = local_api;
  impl_->api_url = std::move(api_url);
  impl_->data_dir = std::move(data_dir);
}

Components::~Components() { stop(); }

bool Components::setup(Manager& mgr, const std::set<std::string>& enabled, int workers, std::string* err) {
  Impl& I = *impl_;
  I.nb_metrics = NotebookMetrics::install(I.c);
  I.setup_notebook(mgr, enabled, workers);
  if (enabled.count("profile")) {
    ProfileOptions po;
    po.userid_header = I.f.userid_header;
    po.userid_prefix = I.f.userid_prefix;
    po.workload_identity = I.f.workload_identity;
    po.namespace_labels_path = I.f.namespace_labels_path;
    I.profile = std::make_unique<ProfileReconciler>(I.c, po, make_configmap_cloud_iam(I.c));
    I.profile->setup(mgr);
  }
  // HTTP admission server (split binaries); each component below adds its own routes
  if (I.f.webhook_port >= 0 && !I.api) I.webhooks = std::make_unique<AdmissionWebhookServer>();
  if (enabled.count("webhooks")) I.setup_admission(mgr);
  if (!I.setup_apps(mgr, enabled, workers, err)) return false;
  if (enabled.count("builtin")) {
    I.builtin = std::make_unique<BuiltinControllers>(I.c);
    I.builtin->setup(mgr, workers);
  }
  if (enabled.count("scheduler")) {
    I.scheduler = std::make_unique<Scheduler>(I.c);
    I.scheduler->setup(mgr);
  }
  if (enabled.count("kubelet")) I.setup_kubelet(mgr);
  if (enabled.count("gateway") && !I.setup_gateway(mgr, err)) return false;
  return !I.webhooks || I.start_webhook_server(enabled, err);
}

void Components::Impl::setup_notebook(Manager& mgr, const std::set<std::string>& enabled, int workers) {
  if (enabled.count("notebook")) {
    notebook = std::make_unique<NotebookReconciler>(c, NotebookOptions::from_env(), nb_metrics);
    notebook->setup(mgr, workers);
  }
  if (enabled.count("culler") && getenv_or("ENABLE_CULLING", "false") == "true") {
    culler = std::make_unique<CullingReconciler>(c, culler_options(enabled), nb_metrics);
    culler->setup(mgr);
  }
}

CullingOptions Components::Impl::culler_options(const std::set<std::string>& enabled) {
  CullingOptions co = CullingOptions::from_env();
  if (!enabled.count("gateway") || !api || f.mesh_port < 0 || !co.mesh_url.empty()) return co;
  // in-process: the kernels GETs go through this node's mesh listener as the notebook
  // controller's ServiceAccount (NOTEBOOK_CONTROLLER_PRINCIPAL, profile_controller.go:420-422)
  Impl* ip = this;
  co.mesh_url_fn = [ip]() -> std::string {
    return ip->gateway && ip->gateway->mesh_port() ? "http://127.0.0.1:" + std::to_string(ip->gateway->mesh_port()) : "";
  };
  const std::string principal = getenv_or("NOTEBOOK_CONTROLLER_PRINCIPAL",
                                          "cluster.local/ns/kubeflow/sa/notebook-controller-service-account");
  auto parts = split(principal, '/', false);  // <domain>/ns/<ns>/sa/<name>
  const std::string sa_ns = parts.size() == 5 ? parts[2] : "kubeflow";
  const std::string sa = parts.size() == 5 ? parts[4] : "notebook-controller-service-account";
  auto cache = std::make_shared<std::pair<std::string, double>>();
  auto mu = std::make_shared<std::mutex>();
  co.peer_token_fn = [ip, sa_ns, sa, cache, mu]() -> std::string {
    std::lock_guard<std::mutex> g(*mu);
    const double now = static_cast<double>(now_unix_ms()) / 1000.0;
    if (!cache->first.empty() && cache->second - 60 > now) return cache->first;
    WriteOptions sys;
    Json nsobj{{"apiVersion", "v1"}, {"kind", "Namespace"}, {"metadata", Json{{"name", sa_ns}}}};
    ip->api->create(nsobj, sys);  // exists: 409, fine
    Json saobj{{"apiVersion", "v1"}, {"kind", "ServiceAccount"}, {"metadata", Json{{"name", sa}, {"namespace", sa_ns}}}};
    ip->api->create(saobj, sys);
    std::string tok;
    double exp = 0;
    if (ip->api->issue_sa_token(sa_ns, sa, 3600, tok, exp)) return "";
    *cache = {tok, exp};
    return tok;
  };
  return co;
}

void Components::Impl::setup_admission(Manager& mgr) {
  auto pd = make_poddefault_plugin(c);
  auto gpu = make_gpu_readiness_plugin();
  auto quota_plugin = make_quota_plugin(c);
  if (api) {
    // kflite: in-process admission chain (same order as the webhook configurations)
    api->add_mutating_plugin("poddefaults.admission.kubeflow.org", pd);
    api->add_mutating_plugin("gpu-readiness.kfamd.io", gpu);
    api->add_validating_plugin("ResourceQuota", quota_plugin);
  }
  if (webhooks) {
    auto pods = builtin_registry().by_kind("v1", "Pod");
    webhooks->add("/apply-poddefault", pd, true, pods);
    webhooks->add("/gpu-readiness", gpu, true, pods);
    webhooks->add("/quota", quota_plugin, false, pods);
  }
  quota = std::make_unique<QuotaController>(c);
  quota->setup(mgr);
}

// tensorboard, pvcviewer, odh, kfam
bool Components::Impl::setup_apps(Manager& mgr, const std::set<std::string>& enabled, int workers, std::string* err) {
  if (enabled.count("tensorboard")) {
    std::string terr;
    TensorboardOptions to = TensorboardOptions::from_env(&terr);
    if (!terr.empty()) {
      *err = terr;
      return false;
    }
    tensorboard = std::make_unique<TensorboardReconciler>(c, to);
    tensorboard->setup(mgr, workers);
  }
  if (enabled.count("pvcviewer")) {
    pvcviewer = std::make_unique<PVCViewerReconciler>(c);
    pvcviewer->setup(mgr, workers);
    if (api) {
      api->add_mutating_plugin("mpvcviewer.kb.io", make_pvcviewer_defaulter());
      api->add_validating_plugin("vpvcviewer.kb.io", make_pvcviewer_validator());
    }
    if (webhooks) {
      auto viewers = builtin_registry().by_kind("kubeflow.org/v1alpha1", "PVCViewer");
      webhooks->add("/mutate-kubeflow-org-v1alpha1-pvcviewer", make_pvcviewer_defaulter(), true, viewers);
      webhooks->add("/validate-kubeflow-org-v1alpha1-pvcviewer", make_pvcviewer_validator(), false, viewers);
    }
  }
  if (enabled.count("odh")) {
    OdhOptions oo;
    oo.oauth_proxy_image = f.oauth_proxy_image;
    oo.controller_namespace = f.controller_namespace;
    oo.set_pipeline_rbac = to_lower(trim(getenv_or("SET_PIPELINE_RBAC", ""))) == "true";
    odh = std::make_unique<OdhNotebookReconciler>(c, oo);
    odh->setup(mgr, workers);
    auto hook = make_odh_notebook_webhook(c, oo);
    if (api) api->add_mutating_plugin("notebooks.opendatahub.io", hook);
    if (webhooks) webhooks->add("/mutate-notebook-v1", hook, true, builtin_registry().by_kind("kubeflow.org/v1", "Notebook"));
  }
  if (enabled.count("kfam") || f.kfam_port >= 0) {
    KfamOptions ko;
    ko.userid_header = f.userid_header;
    ko.userid_prefix = f.userid_prefix;
    if (!f.cluster_admin.empty()) ko.cluster_admins.push_back(f.cluster_admin);
    kfam = std::make_unique<KfamService>(c, ko, &mgr.informer("rbac.authorization.k8s.io/v1", "RoleBinding"));
    if (!kfam->start("127.0.0.1", static_cast<int>(f.kfam_port < 0 ? 0 : f.kfam_port), err)) return false;
    stoppers.push_back([this] { kfam->stop(); });
  }
  return true;
}

// what pods in their own network namespace can reach on the node (relayed into each namespace)
std::vector<std::string> Components::Impl::node_endpoints() const {
  std::vector<std::string> out;
  Url u;
  if (Url::parse(api_url, u) && (u.host == "127.0.0.1" || u.host == "localhost")) out.push_back("127.0.0.1:" + std::to_string(u.port));
  const std::string gw = f.gateway_addr == "0.0.0.0" ? "127.0.0.1" : f.gateway_addr;
  if (gateway && gateway->port()) out.push_back(gw + ":" + std::to_string(gateway->port()));
  if (gateway && gateway->mesh_port()) out.push_back(gw + ":" + std::to_string(gateway->mesh_port()));
  if (kfam && kfam->port()) out.push_back("127.0.0.1:" + std::to_string(kfam->port()));
  return out;
}

void Components::Impl::setup_kubelet(Manager& mgr) {
  KubeletConfig kc;
  kc.node_name = f.node_name;
  kc.node_cpus = static_cast<int>(f.node_cpus);
  kc.node_memory_gib = f.node_memory_gib;
  kc.root_dir = data_dir.empty() ? "/tmp/kflite-" + random_hex(4) : data_dir + "/kubelet";
  char buf[4096];
  const ssize_t n = ::readlink("/proc/self/exe", buf, sizeof buf - 1);
  const std::string exe = n > 0 ? std::string(buf, static_cast<size_t>(n)) : "";
  kc.repo_root = f.repo_root;
  if (kc.repo_root.empty()) {
    // <root>/kubeflow_rm_amd/bin/kflite -> <root>
    std::string r = exe;
    for (int i = 0; i < 3 && !r.empty(); ++i) r = r.substr(0, r.rfind('/'));
    kc.repo_root = r;
  }
  kc.bin_dir = exe.substr(0, exe.rfind('/'));
  // the in-pod readiness op is a HIP binary that only the regular build produces: a kflite from a
  // sanitizer build dir uses the package's bin/ for it
  const std::string pkg_bin = kc.repo_root + "/kubeflow_rm_amd/bin";
  if (::access((kc.bin_dir + "/kfamd-readiness").c_str(), X_OK) != 0 && ::access((pkg_bin + "/kfamd-readiness").c_str(), X_OK) == 0)
    kc.bin_dir = pkg_bin;
  kc.python = f.python;
  kc.api_url = api_url;
  kc.pod_ip_prefix = f.pod_cidr_prefix;
  kc.restart_backoff = f.restart_backoff;
  kc.gpus = static_cast<int>(f.gpus);
  kc.sysfs_root = f.sysfs_root;
  kc.numa_pinning = f.numa_pinning;
  kc.pod_zygote = f.pod_zygote;
  kc.pod_warm_gpus = f.pod_warm_gpus;
  kc.pod_netns = f.pod_netns;
  kc.recipes_file = f.image_recipes;
  const Impl* self = this;
  kc.egress_endpoints = [self] { return self->node_endpoints(); };
  kubelet = std::make_unique<Kubelet>(c, kc);
  kubelet->setup(mgr);
  if (api) {
    Kubelet* k = kubelet.get();
    api->set_log_provider([k](const std::string& ns, const std::string& pod, const std::string& cont, int64_t tail,
                              std::string& out) { return k->read_logs(ns, pod, cont, tail, out); });
    api->set_exec_provider([k](const std::string& ns, const std::string& pod, const std::string& cont,
                               const std::vector<std::string>& argv, double timeout, int& code, std::string& out,
                               std::string& err) { return k->exec(ns, pod, cont, argv, timeout, code, out, err); });
  }
  starters.push_back([this] { kubelet->start(); });
  stoppers.push_back([this] { kubelet->stop(); });
}

bool Components::Impl::setup_gateway(Manager& mgr, std::string* err) {
  GatewayOptions go;
  go.gateway_name = f.gateway_name;
  go.userid_header = f.userid_header;
  go.userid_prefix = f.userid_prefix;
  go.ingress_principal = getenv_or("ISTIO_INGRESS_GATEWAY_PRINCIPAL", go.ingress_principal);
  go.cluster_domain = getenv_or("CLUSTER_DOMAIN", go.cluster_domain);
  go.enforce = f.gateway_authz;
  go.mesh_port = static_cast<int>(f.mesh_port);
  go.control_plane_namespace = f.controller_namespace;
  if (!f.gateway_trusted_proxy_secret_file.empty()) {
    if (!read_file(f.gateway_trusted_proxy_secret_file, go.trusted_proxy_secret)) {
      *err = "cannot read " + f.gateway_trusted_proxy_secret_file;
      return false;
    }
    go.trusted_proxy_secret = trim(go.trusted_proxy_secret);
  }
  gateway = std::make_unique<Gateway>(c, go);
  gateway->setup(mgr);
  // this node's kubelet gets per-pod inbound enforcement points backed by the gateway's policy
  // checks (NetworkPolicy; Istio AuthorizationPolicy for mesh-injected pods)
  if (kubelet) {
    Gateway* gw = gateway.get();
    kubelet->set_inbound_handler([gw](const InboundTarget& t, HttpRequest& req, HttpResponse& resp) { gw->handle_inbound(t, req, resp); });
    // after kubelet->start() decided whether pods get network namespaces
    starters.push_back([this] { gateway->set_pods_have_listeners(kubelet->pod_netns()); });
  }
  if (!gateway->start(f.gateway_addr, static_cast<int>(f.gateway_port), err)) return false;
  stoppers.push_back([this] { gateway->stop(); });
  return true;
}

// started last: every plugin route is registered before the first request. HTTPS like the
// reference's webhook servers (admission-webhook :4443 ListenAndServeTLS, controller-runtime :8443 /
// :9443 from the serving-certs dir); plain HTTP only for kube-lite development (--webhook-tls=off,
// or auto with no certificate pair present)
bool Components::Impl::start_webhook_server(const std::set<std::string>& enabled, std::string* err) {
  TlsServerConfig tls;
  tls.cert_file = f.webhook_cert_file.empty() ? f.webhook_cert_dir + "/tls.crt" : f.webhook_cert_file;
  tls.key_file = f.webhook_key_file.empty() ? f.webhook_cert_dir + "/tls.key" : f.webhook_key_file;
  const bool have_pair = file_exists(tls.cert_file) && file_exists(tls.key_file);
  const bool use_tls = f.webhook_tls == "on" || (f.webhook_tls == "auto" && have_pair);
  if (f.webhook_tls == "on" && !have_pair) {
    *err = "webhook TLS: missing " + tls.cert_file + " / " + tls.key_file;
    return false;
  }
  if (!webhooks->start(f.webhook_host, static_cast<int>(f.webhook_port), err, use_tls ? &tls : nullptr)) return false;
  stoppers.push_back([this] { webhooks->stop(); });
  if (!use_tls) KF_WARN("webhooks", "serving admission webhooks over plain HTTP (no certificate pair)", Json{{"cert", tls.cert_file}});
  if (api) return true;
  // split mode: register our hooks with the remote API server (the manifests' job upstream)
  const std::string host = f.webhook_host == "0.0.0.0" ? "127.0.0.1" : f.webhook_host;
  const std::string base = std::string(use_tls ? "https://" : "http://") + host + ":" + std::to_string(webhooks->port());
  std::string ca_pem;
  if (use_tls) {
    std::string ca_file = f.webhook_ca_file;
    if (ca_file.empty()) ca_file = file_exists(f.webhook_cert_dir + "/ca.crt") ? f.webhook_cert_dir + "/ca.crt" : tls.cert_file;
    read_file(ca_file, ca_pem);
  }
  std::string cfg_name = "kfamd";
  for (const auto& comp : enabled) cfg_name += "-" + comp;
  for (auto cfg : webhooks->webhook_configurations(base, cfg_name, ca_pem)) {
    Json live;
    ApiError e = c->get(cfg["apiVersion"].as_string(), cfg["kind"].as_string(), "", cfg_name, live);
    if (e.code == 404) e = c->create(cfg);
    else if (!e) {
      live["webhooks"] = cfg["webhooks"];
      e = c->update(live);
    }
    if (e) {
      *err = "registering webhooks: " + e.message;
      return false;
    }
  }
  return true;
}

void Components::start() {
  for (auto& s : impl_->starters) s();
}

void Components::stop() {
  if (!impl_) return;
  for (auto it = impl_->stoppers.rbegin(); it != impl_->stoppers.rend(); ++it) (*it)();
  impl_->stoppers.clear();
}

int Components::gateway_port() const { return impl_->gateway ? impl_->gateway->port() : 0; }
int Components::mesh_port() const { return impl_->gateway ? impl_->gateway->mesh_port() : 0; }
int Components::kfam_port() const { return impl_->kfam ? impl_->kfam->port() : 0; }
int Components::webhook_port() const { return impl_->webhooks ? impl_->webhooks->port() : 0; }

}  // namespace kf
