// node.h — the single-node runtime that the reference takes from Kubernetes L0
// (kube-scheduler, kubelet + AMD device plugin, Istio ingress gateway), re-designed for one
// 8 x MI355X node:
//
//   Scheduler  filters nodes (Ready, taints/tolerations, nodeSelector, required node affinity,
//              cpu / memory / amd.com/gpu / amd.com/gpu-memory fit) and scores them (preferred
//              affinity, least-allocated); binds by setting spec.nodeName; records
//              PodScheduled + Scheduled/FailedScheduling events.
//   Kubelet    registers the Node (capacity from the xGMI topology: amd.com/gpu, amd.com/gpu-memory
//              in GiB), runs pods as supervised process groups ("containers" = processes; images
//              resolve to process recipes), allocates GPUs through the topology-aware allocator at
//              admission (device-plugin Allocate) and injects HIP_VISIBLE_DEVICES + RCCL/torchrun env,
//              gives every pod its own loopback IP (127.20.x.y) so every notebook listens on :8888,
//              materialises volumes (emptyDir / PVC / configMap / secret) under the pod sandbox,
//              runs init containers in order, HTTP/TCP/exec probes, restart policies with back-off,
//              optionally forks Python containers from a per-recipe pre-imported interpreter
//              (--pod-zygote: torch imported once per node, kubeflow_rm_amd/images/zygote.py),
//              graceful termination, termination messages, container logs, and full pod status with
//              millisecond timestamps (the cold-start phase breakdown of SURVEY §5.1).
//   Gateway    HTTP reverse proxy that serves Istio VirtualServices (uri prefix match, rewrite,
//              headers.request.set, timeout) and OpenShift Routes for the embedded cluster, and the
//              policy enforcement point Istio is in the reference: end-user authentication (bearer
//              token / session cookie via TokenReview, or a trusted authn proxy), the userid header set
//              only from that identity, and AuthorizationPolicy ALLOW/DENY evaluation (node/authz.h) on
//              the ingress listener and on an in-cluster mesh listener (ServiceAccount principals).
#pragma once

#include <atomic>
#include <functional>
#include <optional>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <regex>
#include <string>
#include <thread>
#include <vector>

#include "core/http.h"
#include "core/metrics.h"
#include "gpu/topology.h"
#include "node/netns.h"
#include "runtime/runtime.h"

namespace kf {

class Prober;  // node/prober.h

// Resource accounting helpers (shared with the quota admission plugin).
// Effective pod request: max(sum(containers), max(initContainers)) per resource; extended
// resources default their request to the limit.
Json pod_requests(const Json& pod);
double resource_value(const std::string& name, const Json& quantity);  // cpu cores, bytes, counts

class Scheduler {
 public:
  explicit Scheduler(std::shared_ptr<Client> c) : c_(std::move(c)) {}
  void setup(Manager& mgr);
  Result reconcile(const Request& r, std::string* err);
  // pure helpers (unit-tested)
  static bool tolerates(const Json& pod, const Json& node);
  static bool matches_affinity(const Json& pod, const Json& node);
  static int64_t preferred_score(const Json& pod, const Json& node);

 private:
  std::shared_ptr<Client> c_;
  Informer* pods_ = nullptr;
  Informer* nodes_ = nullptr;
  std::unique_ptr<EventRecorder> rec_;
  std::shared_ptr<Controller> ctl_;
  // bound by us, not yet visible in the pod cache (touched only by the single scheduler worker)
  struct Assumed {
    std::string ns, name, node;
    Json requests;
  };
  std::map<std::string, Assumed> assumed_;
};

struct KubeletConfig {
  std::string node_name = "mi355x-node-0";
  std::string root_dir;      // pod sandboxes, PV dirs, logs
  std::string repo_root;     // kubeflow_rm_amd location for image recipes
  std::string bin_dir;       // native binaries (kfamd-readiness)
  std::string python = "python3";
  std::string api_url;       // exported to pods as KUBERNETES_SERVICE_HOST/PORT
  std::string pod_ip_prefix = "127.20";
  std::string app_ip_prefix = "127.21";  // the private address a mesh-injected pod's apps bind
  double restart_backoff = 10.0;
  int gpus = -1;
  int node_cpus = 0;         // advertised CPU capacity (0 = online host CPUs)
  int64_t node_memory_gib = 0;  // advertised memory (0 = host RAM)
  std::string recipes_file;  // optional JSON overriding the image recipes
  std::string sysfs_root;    // "" = /sys (tests: a fake tree with class/kfd, bus/pci, devices/system/node)
  bool numa_pinning = true;  // pin GPU pods' processes to their devices' NUMA-local CPUs
  // start a pre-imported interpreter (kubeflow_rm_amd/images/zygote.py) per image recipe that names
  // one, and fork Python containers from it instead of exec'ing a fresh interpreter
  bool pod_zygote = true;
  // a torch zygote keeps one warm child per node GPU (HIP + device context up) that a 1-GPU
  // container on that GPU takes over (kubeflow_rm_amd/images/zygote.py); real GPUs only
  bool pod_warm_gpus = true;
  // per-pod network namespaces (node/netns.h): "auto" (when the node can create them and a policy
  // enforcer is wired), "on" (required: pods fail admission without one), "off" (private-address
  // convention only)
  std::string pod_netns = "auto";
  // the node endpoints ("127.0.0.1:<port>") relayed into every pod namespace: API server, ingress
  // gateway, mesh listener, KFAM (evaluated when a pod is admitted: ports may be ephemeral)
  std::function<std::vector<std::string>()> egress_endpoints;
};

struct ContainerRt;  // one container's process state (kubelet.cc)

// A pod's inbound enforcement point (the CNI's NetworkPolicy hook + the Istio sidecar's inbound
// listener): the kubelet binds pod_ip:port (host namespace) for every declared TCP containerPort —
// of every pod when pods have their own network namespace (node/netns.h), else of mesh-injected and
// NetworkPolicy-selected pods, whose apps then listen on a private app_ip — and each request is
// handed to the gateway's policy check (Gateway::handle_inbound) before it is proxied to the app.
// Kubelet probes go to the app directly (exempt, as Istio's rewritten probes are).
struct InboundTarget {
  std::string ns, name, app_ip, pod_ip;
  int port = 0;
  std::string port_name;  // the containerPort's name (NetworkPolicy named ports)
  std::map<std::string, std::string> labels;
  bool mesh = false;                      // Istio sidecar semantics (AuthorizationPolicies) too
  std::shared_ptr<const PodNetns> netns;  // the app's namespace (nullptr: app_ip on the host)
};
using InboundHandler = std::function<void(const InboundTarget&, HttpRequest&, HttpResponse&)>;

class Kubelet {
 public:
  Kubelet(std::shared_ptr<Client> c, KubeletConfig cfg);
  ~Kubelet();
  void setup(Manager& mgr);
  void start();  // node registration + heartbeat
  void stop();
  Result reconcile(const Request& r, std::string* err);
  bool read_logs(const std::string& ns, const std::string& pod, const std::string& container, int64_t tail,
                 std::string& out);
  // pods/exec: argv in a running container's env, working directory and CPU mask (a new process in
  // the container's place; output = stdout + stderr); false + err when it cannot run
  bool exec(const std::string& ns, const std::string& pod, const std::string& container,
            const std::vector<std::string>& argv, double timeout_s, int& exit_code, std::string& output, std::string& err);
  GpuAllocator& gpus() { return *alloc_; }
  bool pod_netns() const { return netns_; }
  const std::string& node_name() const { return cfg_.node_name; }
  // pods of mesh-injected namespaces (label istio-injection=enabled, pod annotation
  // sidecar.istio.io/inject not "false") get an inbound listener per containerPort (set before start)
  void set_inbound_handler(InboundHandler h) { inbound_ = std::move(h); }

  struct PodRuntime;
  // image -> argv resolution (unit-tested)
  // zygote (optional): the recipe's preload list when its containers may fork from a zygote
  std::vector<std::string> resolve_argv(const Json& container, std::string* why = nullptr,
                                        std::string* zygote = nullptr) const;

 private:
  Json node_object() const;
  void heartbeat_loop();
  void register_gpu_metrics();
  void register_telemetry_metrics();
  bool metrics_registered_ = false;
  void terminate_pod(PodRuntime& rt, int64_t grace_s);
  // one reconcile pass, in units (kubelet.cc): lookup / deletion / admission, then the containers
  struct PodSync;
  std::shared_ptr<PodRuntime> lookup_runtime(const Request& r, const ApiError& e, const Json& pod);
  void finish_deletion(const Request& r, const Json& pod, const std::shared_ptr<PodRuntime>& rt, std::string* err);
  std::shared_ptr<PodRuntime> admit(const Request& r, const Json& pod);
  void allocate_gpus(PodRuntime& rt, const Json& pod);
  std::map<std::string, std::string> prepare_volumes(PodRuntime& rt, const Json& pod);
  void build_containers(PodRuntime& rt, const Json& pod, const std::map<std::string, std::string>& vol_dirs);
  void fail_admission(const Request& r, const std::string& why);
  void container_env(const PodSync& s, const Json& c, std::vector<std::string>& envv,
                     std::map<std::string, std::string>& envm);
  void start_container(PodSync& s, ContainerRt& cr);
  std::function<bool()> make_probe(const PodSync& s, const Json& probe, const Json& c);
  std::optional<bool> probe_verdict(PodSync& s, ContainerRt& cr, const char* kind, const Json& probe, const Json& c,
                                    bool due);
  void tick_probes(PodSync& s, ContainerRt& cr, const Json& c);
  void tick_long_running(PodSync& s, ContainerRt& cr, bool always_restart);
  void run_init_containers(PodSync& s);
  void publish_readiness(PodSync& s);
  ApiError write_status(PodSync& s);
  bool wants_sidecar(const Json& pod);
  bool selected_by_netpol(const Json& pod);
  void start_inbound(PodRuntime& rt, const Json& pod, bool mesh);
  bool setup_pod_network(PodRuntime& rt, const Json& pod);
  InboundHandler inbound_;
  bool netns_ = false;                  // pods get their own network namespace (decided at start())
  std::unique_ptr<EgressRelay> relay_;  // their egress to the node endpoints
  std::shared_ptr<Client> c_;
  KubeletConfig cfg_;
  std::unique_ptr<GpuAllocator> alloc_;
  Json recipes_;
  std::vector<std::regex> recipe_re_;  // recipes_[i]["match"], compiled once (std::regex construction is not thread-safe)
  std::mutex mu_;
  std::map<std::string, std::shared_ptr<PodRuntime>> pods_;  // uid -> runtime
  std::map<std::string, std::string> key_to_uid_;            // ns/name -> uid
  uint32_t next_ip_ = 2;
  std::set<int> rdzv_ports_;  // MASTER_PORTs handed to running multi-GPU pods
  int alloc_rdzv_port();
  std::unique_ptr<EventRecorder> rec_;
  std::unique_ptr<Prober> prober_;  // probes run on its threads, never on a reconcile worker
  std::shared_ptr<Controller> ctl_;
  std::atomic<bool> running_{false};
  std::atomic<bool> stopping_{false};
  std::thread hb_;
  // container exits wake the pod's reconcile at once (pidfd + epoll; PLEG without the relist
  // latency): the init container's exit gates Initialized, a crash needs a restart
  void watch_exit(pid_t pid, const std::string& ns, const std::string& name);
  void exit_watch_loop();
  int epfd_ = -1;
  int wake_fd_ = -1;
  std::mutex watch_mu_;
  std::map<int, std::pair<std::string, std::string>> watched_;  // pidfd -> pod ns/name
  std::thread exit_watch_;
  void watch_fd(int fd, const std::string& ns, const std::string& name);
  // pre-imported interpreters, keyed by preload list (cfg_.pod_zygote)
  struct Zygote {
    std::string preload, sock, log;
    pid_t pid = -1;
    double started = 0;
    int quick_exits = 0;  // exits within 30 s of a start, in a row: 3 and it is not restarted
  };
  std::map<std::string, Zygote> zygotes_;  // guarded by zy_mu_ (start() runs after the workers)
  std::mutex zy_mu_;
  void start_zygotes();
  void stop_zygotes();
  // warm GPU readiness ops (kfamd-readiness --warm-op), one per node GPU
  struct WarmOp {
    int dev = 0;
    pid_t pid = -1;
    double started = 0, next_start = 0;
    int failures = 0;  // warm-up failures in a row: 3 and the device gets none
  };
  std::vector<WarmOp> warm_ops_;
  std::mutex wo_mu_;
  // the node's trusted comgr seed (seed_comgr_cache): RCCL's device-code builds made once by the
  // kubelet's own readiness op, hard-linked into each namespace's new code-object cache
  std::string comgr_seed_;
  pid_t seed_pid_ = -1;
  std::string warm_dir_;  // set once in start() before any pod is admitted
  void start_warm_ops();
  void seed_comgr_cache();
  void finish_comgr_seed();
  void link_comgr_seed(const std::string& cache_dir);
  void supervise_warm_ops();
  void stop_warm_ops();
  void supervise_zygotes();  // heartbeat thread: restart a zygote that exited
  bool spawn_zygote(Zygote& z);
};

struct GatewayOptions {
  std::string gateway_name = "kubeflow/kubeflow-gateway";  // VirtualService gateway served by the ingress
  // identity: the header the ingress sets from the authenticated user (profile / KFAM policies and
  // the web apps read it), minus nothing, plus userid_prefix
  std::string userid_header = "kubeflow-userid";
  std::string userid_prefix;
  // the principals the profile's ns-owner-access-istio policy names
  std::string ingress_principal = "cluster.local/ns/istio-system/sa/istio-ingressgateway-service-account";
  std::string ingress_namespace = "istio-system";
  std::string root_namespace = "istio-system";  // mesh-wide AuthorizationPolicies live here
  std::string cluster_domain = "cluster.local";
  // an authenticating proxy in front of the ingress (oauth2-proxy / dex) may assert the userid header
  // when it presents this secret in X-Kfamd-Auth-Proxy-Secret (empty = no trusted proxy)
  std::string trusted_proxy_secret;
  std::string auth_cookie = "kfamd-token";  // browser sessions: the bearer token as a cookie
  bool enforce = true;                      // evaluate AuthorizationPolicies (ALLOW/DENY)
  int mesh_port = -1;                       // in-cluster listener (-1 = off, 0 = ephemeral)
  // NetworkPolicy source of a connection made straight to a pod's inbound listener by a node process
  // (the culler, the API server's service proxy): the control plane's namespace
  std::string control_plane_namespace = "kubeflow";
};

class Gateway {
 public:
  Gateway(std::shared_ptr<Client> c, GatewayOptions o);
  ~Gateway();
  void setup(Manager& mgr);
  bool start(const std::string& addr, int port, std::string* err);
  void stop();
  int port() const { return srv_ ? srv_->port() : 0; }
  int mesh_port() const { return mesh_ ? mesh_->port() : 0; }
  // ingress: VirtualService / Route match, end-user authentication, policy check, proxy
  void handle(HttpRequest& req, HttpResponse& resp);
  // mesh (the destination sidecars' job, done node-wide like Istio ambient's ztunnel): Host names a
  // Service, the caller's identity is its ServiceAccount token in X-Kfamd-Peer-Token
  void handle_mesh(HttpRequest& req, HttpResponse& resp);
  // a pod's inbound listener (InboundTarget): NetworkPolicy (ingress rules against the caller's
  // namespace / pod labels / address) for every pod with a listener, then, for mesh-injected pods,
  // the namespace's AuthorizationPolicies on the pod's own labels. Requests the ingress / mesh
  // listener authorized carry a signed proof naming the caller (X-Kfamd-Hop); any other caller is
  // evaluated with its own identity (ServiceAccount token in X-Kfamd-Peer-Token, else none). Then
  // proxied to the app (inside the pod's network namespace when it has one).
  void handle_inbound(const InboundTarget& t, HttpRequest& req, HttpResponse& resp);
  void set_pods_have_listeners(bool v) { pods_have_listeners_ = v; }

  struct Route {
    std::string prefix, rewrite, dest_host;
    int dest_port = 80;
    Json headers;
    double timeout_s = 300;
    bool exact = false;
  };
  // best matching VirtualService route for host + path (unit-tested)
  static bool match(const std::vector<Json>& vss, const std::string& gateway, const std::string& host,
                    const std::string& path, Route& out);

  struct Identity {
    bool authenticated = false;
    std::string username;
    std::vector<std::string> groups;
    bool service_account() const { return starts_with_sa(username); }
    static bool starts_with_sa(const std::string& u) { return u.rfind("system:serviceaccount:", 0) == 0; }
  };
  // TokenReview through the API server, cached (positive 10 s, negative 2 s)
  Identity review_token(const std::string& token);

 private:
  bool authorize(const std::string& dest_host, int dest_port, const HttpRequest& req, const std::string& path,
                 const Headers& fwd, const std::string& principal, const std::string& source_ns, std::string* why);
  bool authorize_workload(const std::string& ns, const std::map<std::string, std::string>& labels, int dest_port,
                          const HttpRequest& req, const std::string& path, const Headers& fwd,
                          const std::string& principal, const std::string& source_ns, std::string* why);
  void peer_identity(const HttpRequest& req, std::string& principal, std::string& source_ns);
  // the caller a signed hop proof names (kHopHeader in gateway.cc)
  struct HopClaims {
    std::string principal, source_ns;
    bool source_pod = false;
    std::map<std::string, std::string> source_labels;
  };
  std::string stamp_hop(const std::string& method, const std::string& path, const std::string& dest_ns,
                        const HopClaims& who) const;
  bool verify_hop(const std::string& value, const std::string& method, const std::string& path,
                  const std::string& dest_ns, HopClaims& out) const;
  HopClaims mesh_caller(const HttpRequest& req);
  std::map<std::string, std::string> namespace_labels(const std::string& ns);
  bool dest_has_listener(const std::string& ns);
  Result reconcile_mesh_policy(const Request& r, std::string* err);
  std::shared_ptr<Controller> mesh_np_;
  std::string hop_secret_;  // HMAC key of the hop proofs
  std::atomic<bool> pods_have_listeners_{false};  // every pod has an inbound listener (kubelet --pod-netns)
  void forward(HttpRequest& req, HttpResponse& resp, const std::string& url, Headers h, int timeout_ms);

  std::shared_ptr<Client> c_;
  GatewayOptions o_;
  Informer* vs_ = nullptr;
  Informer* routes_ = nullptr;
  Informer* policies_ = nullptr;
  Informer* services_ = nullptr;
  Informer* netpols_ = nullptr;
  Informer* namespaces_ = nullptr;
  std::unique_ptr<HttpServer> srv_, mesh_;
  std::shared_ptr<CounterVec> upgrades_, streams_, decisions_;
  // host an OpenShift router gives a Route without spec.host: <name>-<namespace>.<domain>
  // (KFAMD_ROUTE_DOMAIN, default apps.kube-lite)
  std::string route_domain_;
  std::mutex tok_mu_;
  std::map<std::string, std::pair<Identity, double>> tok_cache_;  // token -> (identity, expiry)
};

}  // namespace kf
