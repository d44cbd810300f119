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
  f.add_bool("pod-zygote", &pod_zygote, false,
             "fork Python pod containers from a pre-imported interpreter per image recipe (torch preloaded)");
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
  if (enabled.count("notebook")) {
    I.notebook = std::make_unique<NotebookReconciler>(I.c, NotebookOptions::from_env(), I.nb_metrics);
    I.notebook->setup(mgr, workers);
  }
  if (enabled.count("culler") && getenv_or("ENABLE_CULLING", "false") == "true") {
    CullingOptions co = CullingOptions::from_env();
    if (enabled.count("gateway") && I.api && I.f.mesh_port >= 0 && co.mesh_url.empty()) {
      // in-process: the kernels GETs go through this node's mesh listener as the notebook
      // controller's ServiceAccount (NOTEBOOK_CONTROLLER_PRINCIPAL, profile_controller.go:420-422)
      Impl* ip = &I;
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
    }
    I.culler = std::make_unique<CullingReconciler>(I.c, co, I.nb_metrics);
    I.culler->setup(mgr);
  }
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
  if (enabled.count("webhooks")) {
    auto pd = make_poddefault_plugin(I.c);
    auto gpu = make_gpu_readiness_plugin();
    auto quota = make_quota_plugin(I.c);
    if (I.api) {
      // kflite: in-process admission chain (same order as the webhook configurations)
      I.api->add_mutating_plugin("poddefaults.admission.kubeflow.org", pd);
      I.api->add_mutating_plugin("gpu-readiness.kfamd.io", gpu);
      I.api->add_validating_plugin("ResourceQuota", quota);
    }
    if (I.webhooks) {
      auto pods = builtin_registry().by_kind("v1", "Pod");
      I.webhooks->add("/apply-poddefault", pd, true, pods);
      I.webhooks->add("/gpu-readiness", gpu, true, pods);
      I.webhooks->add("/quota", quota, false, pods);
    }
    I.quota = std::make_unique<QuotaController>(I.c);
    I.quota->setup(mgr);
  }
  if (enabled.count("tensorboard")) {
    std::string terr;
    TensorboardOptions to = TensorboardOptions::from_env(&terr);
    if (!terr.empty()) {
      *err = terr;
      return false;
    }
    I.tensorboard = std::make_unique<TensorboardReconciler>(I.c, to);
    I.tensorboard->setup(mgr, workers);
  }
  if (enabled.count("pvcviewer")) {
    I.pvcviewer = std::make_unique<PVCViewerReconciler>(I.c);
    I.pvcviewer->setup(mgr, workers);
    if (I.api) {
      I.api->add_mutating_plugin("mpvcviewer.kb.io", make_pvcviewer_defaulter());
      I.api->add_validating_plugin("vpvcviewer.kb.io", make_pvcviewer_validator());
    }
    if (I.webhooks) {
      auto viewers = builtin_registry().by_kind("kubeflow.org/v1alpha1", "PVCViewer");
      I.webhooks->add("/mutate-kubeflow-org-v1alpha1-pvcviewer", make_pvcviewer_defaulter(), true, viewers);
      I.webhooks->add("/validate-kubeflow-org-v1alpha1-pvcviewer", make_pvcviewer_validator(), false, viewers);
    }
  }
  if (enabled.count("odh")) {
    OdhOptions oo;
    oo.oauth_proxy_image = I.f.oauth_proxy_image;
    oo.controller_namespace = I.f.controller_namespace;
    oo.set_pipeline_rbac = to_lower(trim(getenv_or("SET_PIPELINE_RBAC", ""))) == "true";
    I.odh = std::make_unique<OdhNotebookReconciler>(I.c, oo);
    I.odh->setup(mgr, workers);
    auto hook = make_odh_notebook_webhook(I.c, oo);
    if (I.api) I.api->add_mutating_plugin("notebooks.opendatahub.io", hook);
    if (I.webhooks) I.webhooks->add("/mutate-notebook-v1", hook, true, builtin_registry().by_kind("kubeflow.org/v1", "Notebook"));
  }
  if (enabled.count("kfam") || I.f.kfam_port >= 0) {
    KfamOptions ko;
    ko.userid_header = I.f.userid_header;
    ko.userid_prefix = I.f.userid_prefix;
    if (!I.f.cluster_admin.empty()) ko.cluster_admins.push_back(I.f.cluster_admin);
    I.kfam = std::make_unique<KfamService>(I.c, ko, &mgr.informer("rbac.authorization.k8s.io/v1", "RoleBinding"));
    if (!I.kfam->start("127.0.0.1", static_cast<int>(I.f.kfam_port < 0 ? 0 : I.f.kfam_port), err)) return false;
    I.stoppers.push_back([&I] { I.kfam->stop(); });
  }
  if (enabled.count("builtin")) {
    I.builtin = std::make_unique<BuiltinControllers>(I.c);
    I.builtin->setup(mgr, workers);
  }
  if (enabled.count("scheduler")) {
    I.scheduler = std::make_unique<Scheduler>(I.c);
    I.scheduler->setup(mgr);
  }
  if (enabled.count("kubelet")) {
    KubeletConfig kc;
    kc.node_name = I.f.node_name;
    kc.node_cpus = static_cast<int>(I.f.node_cpus);
    kc.node_memory_gib = I.f.node_memory_gib;
    kc.root_dir = I.data_dir.empty() ? "/tmp/kflite-" + random_hex(4) : I.data_dir + "/kubelet";
    kc.repo_root = I.f.repo_root;
    if (kc.repo_root.empty()) {
      char buf[4096];
      ssize_t n = ::readlink("/proc/self/exe", buf, sizeof buf - 1);
      std::string exe = n > 0 ? std::string(buf, static_cast<size_t>(n)) : "";
      // <root>/kubeflow_rm_amd/bin/kflite -> <root>
      for (int i = 0; i < 3 && !exe.empty(); ++i) exe = exe.substr(0, exe.rfind('/'));
      kc.repo_root = exe;
    }
    {
      char buf[4096];
      ssize_t n = ::readlink("/proc/self/exe", buf, sizeof buf - 1);
      std::string exe = n > 0 ? std::string(buf, static_cast<size_t>(n)) : "";
      kc.bin_dir = exe.substr(0, exe.rfind('/'));
      // the in-pod readiness op is a HIP binary that only the regular build produces: a kflite
      // from a sanitizer build dir uses the package's bin/ for it
      const std::string pkg_bin = kc.repo_root + "/kubeflow_rm_amd/bin";
      if (::access((kc.bin_dir + "/kfamd-readiness").c_str(), X_OK) != 0 &&
          ::access((pkg_bin + "/kfamd-readiness").c_str(), X_OK) == 0)
        kc.bin_dir = pkg_bin;
    }
    kc.python = I.f.python;
    kc.api_url = I.api_url;
    kc.pod_ip_prefix = I.f.pod_cidr_prefix;
    kc.restart_backoff = I.f.restart_backoff;
    kc.gpus = static_cast<int>(I.f.gpus);
    kc.sysfs_root = I.f.sysfs_root;
    kc.numa_pinning = I.f.numa_pinning;
    kc.pod_zygote = I.f.pod_zygote;
    kc.recipes_file = I.f.image_recipes;
    I.kubelet = std::make_unique<Kubelet>(I.c, kc);
    I.kubelet->setup(mgr);
    if (I.api) {
      Kubelet* k = I.kubelet.get();
      I.api->set_log_provider([k](const std::string& ns, const std::string& pod, const std::string& cont, int64_t tail,
                                  std::string& out) { return k->read_logs(ns, pod, cont, tail, out); });
      I.api->set_exec_provider([k](const std::string& ns, const std::string& pod, const std::string& cont,
                                   const std::vector<std::string>& argv, double timeout, int& code, std::string& out,
                                   std::string& err) { return k->exec(ns, pod, cont, argv, timeout, code, out, err); });
    }
    I.starters.push_back([&I] { I.kubelet->start(); });
    I.stoppers.push_back([&I] { I.kubelet->stop(); });
  }
  if (enabled.count("gateway")) {
    GatewayOptions go;
    go.gateway_name = I.f.gateway_name;
    go.userid_header = I.f.userid_header;
    go.userid_prefix = I.f.userid_prefix;
    go.ingress_principal = getenv_or("ISTIO_INGRESS_GATEWAY_PRINCIPAL", go.ingress_principal);
    go.cluster_domain = getenv_or("CLUSTER_DOMAIN", go.cluster_domain);
    go.enforce = I.f.gateway_authz;
    go.mesh_port = static_cast<int>(I.f.mesh_port);
    if (!I.f.gateway_trusted_proxy_secret_file.empty()) {
      if (!read_file(I.f.gateway_trusted_proxy_secret_file, go.trusted_proxy_secret)) {
        *err = "cannot read " + I.f.gateway_trusted_proxy_secret_file;
        return false;
      }
      go.trusted_proxy_secret = trim(go.trusted_proxy_secret);
    }
    I.gateway = std::make_unique<Gateway>(I.c, go);
    I.gateway->setup(mgr);
    // this node's kubelet gets per-pod inbound enforcement points backed by the gateway's policy
    // check (profile namespaces are istio-injection=enabled: direct pod-IP traffic is evaluated too)
    if (I.kubelet && go.enforce) {
      Gateway* gw = I.gateway.get();
      I.kubelet->set_inbound_handler(
          [gw](const InboundTarget& t, HttpRequest& req, HttpResponse& resp) { gw->handle_inbound(t, req, resp); });
    }
    if (!I.gateway->start(I.f.gateway_addr, static_cast<int>(I.f.gateway_port), err)) return false;
    I.stoppers.push_back([&I] { I.gateway->stop(); });
  }
  if (I.webhooks) {
    // started last: every plugin route is registered before the first request
    // HTTPS like the reference's webhook servers (admission-webhook :4443 ListenAndServeTLS,
    // controller-runtime :8443 / :9443 from the serving-certs dir); plain HTTP only for kube-lite
    // development (--webhook-tls=off, or auto with no certificate pair present)
    TlsServerConfig tls;
    tls.cert_file = I.f.webhook_cert_file.empty() ? I.f.webhook_cert_dir + "/tls.crt" : I.f.webhook_cert_file;
    tls.key_file = I.f.webhook_key_file.empty() ? I.f.webhook_cert_dir + "/tls.key" : I.f.webhook_key_file;
    const bool have_pair = file_exists(tls.cert_file) && file_exists(tls.key_file);
    const bool use_tls = I.f.webhook_tls == "on" || (I.f.webhook_tls == "auto" && have_pair);
    if (I.f.webhook_tls == "on" && !have_pair) {
      *err = "webhook TLS: missing " + tls.cert_file + " / " + tls.key_file;
      return false;
    }
    if (!I.webhooks->start(I.f.webhook_host, static_cast<int>(I.f.webhook_port), err, use_tls ? &tls : nullptr)) return false;
    I.stoppers.push_back([&I] { I.webhooks->stop(); });
    if (!use_tls) KF_WARN("webhooks", "serving admission webhooks over plain HTTP (no certificate pair)", Json{{"cert", tls.cert_file}});
    if (!I.api) {
      // split mode: register our hooks with the remote API server (the manifests' job upstream)
      const std::string host = I.f.webhook_host == "0.0.0.0" ? "127.0.0.1" : I.f.webhook_host;
      const std::string base = std::string(use_tls ? "https://" : "http://") + host + ":" + std::to_string(I.webhooks->port());
      std::string ca_pem;
      if (use_tls) {
        std::string ca_file = I.f.webhook_ca_file;
        if (ca_file.empty()) ca_file = file_exists(I.f.webhook_cert_dir + "/ca.crt") ? I.f.webhook_cert_dir + "/ca.crt" : tls.cert_file;
        read_file(ca_file, ca_pem);
      }
      std::string cfg_name = "kfamd";
      for (const auto& c : enabled) cfg_name += "-" + c;
      for (auto cfg : I.webhooks->webhook_configurations(base, cfg_name, ca_pem)) {
        Json live;
        ApiError e = I.c->get(cfg["apiVersion"].as_string(), cfg["kind"].as_string(), "", cfg_name, live);
        if (e.code == 404) e = I.c->create(cfg);
        else if (!e) {
          live["webhooks"] = cfg["webhooks"];
          e = I.c->update(live);
        }
        if (e) {
          *err = "registering webhooks: " + e.message;
          return false;
        }
      }
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
