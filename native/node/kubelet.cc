// kubelet.cc — process-pod kubelet with the MI355X device plugin (see node.h).
#include <cstdio>
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <signal.h>
#include <sched.h>
#include <spawn.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/epoll.h>
#include <sys/ioctl.h>
#include <sys/eventfd.h>
#include <sys/syscall.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <unistd.h>
#include <linux/fs.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <functional>
#include <optional>
#include <random>
#include <regex>
#include <set>

#include "controllers/common.h"
#include "core/resources.h"
#include "core/util.h"
#include "gpu/smi.h"
#include "node/node.h"
#include "node/netpol.h"
#include "node/prober.h"

extern char** environ;

namespace kf {

namespace {
std::string ms_now() { return rfc3339_ms_now(); }

int64_t probe_i(const Json& probe, const char* key, int64_t def) { return probe[key].as_int(def); }

// env KFAMD_SHARE_POD_GPUS=true: the container sees the pod's allocated GPUs without requesting its
// own (what one DRA ResourceClaim shared by two containers gives on upstream Kubernetes)
bool shares_pod_gpus(const Json& c) {
  for (const auto& e : c["env"].as_array())
    if (e["name"].as_string() == "KFAMD_SHARE_POD_GPUS") return e["value"].as_string() == "true";
  return false;
}

bool tcp_connect(const std::string& ip, int port, int timeout_ms) {
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return false;
  ::fcntl(fd, F_SETFL, O_NONBLOCK);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(static_cast<uint16_t>(port));
  ::inet_pton(AF_INET, ip.c_str(), &sa.sin_addr);
  int rc = ::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa);
  bool ok = rc == 0;
  if (!ok && errno == EINPROGRESS) {
    pollfd p{fd, POLLOUT, 0};
    if (::poll(&p, 1, timeout_ms) > 0) {
      int err = 0;
      socklen_t l = sizeof err;
      ::getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &l);
      ok = err == 0;
    }
  }
  ::close(fd);
  return ok;
}

bool executable(const std::string& path) { return ::access(path.c_str(), X_OK) == 0; }

std::string which(const std::string& cmd) {
  if (cmd.empty()) return "";
  if (cmd.find('/') != std::string::npos) return executable(cmd) ? cmd : "";
  for (const auto& dir : split(getenv_or("PATH", "/usr/bin:/bin"), ':', true)) {
    std::string p = dir + "/" + cmd;
    if (executable(p)) return p;
  }
  return "";
}

// $(VAR) expansion (Kubernetes command/args semantics; $$ escapes)
std::string expand_vars(const std::string& s, const std::map<std::string, std::string>& env) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '$' && i + 1 < s.size() && s[i + 1] == '$') {
      out += '$';
      ++i;
    } else if (s[i] == '$' && i + 1 < s.size() && s[i + 1] == '(') {
      size_t e = s.find(')', i + 2);
      if (e == std::string::npos) {
        out += s.substr(i);
        break;
      }
      std::string name = s.substr(i + 2, e - i - 2);
      auto it = env.find(name);
      out += it != env.end() ? it->second : s.substr(i, e - i + 1);
      i = e;
    } else {
      out += s[i];
    }
  }
  return out;
}

const char* kDefaultRecipes = R"([
  {"match": "cmd:kfamd-readiness|kfamd-readiness|gpu-readiness", "argv": ["{bin}/kfamd-readiness"], "passArgs": true},
  {"match": "odh-notebook-controller", "argv": ["{bin}/odh-notebook-controller"], "passArgs": true},
  {"match": "kfamd/notebook-controller|notebook-controller:", "argv": ["{bin}/notebook-controller"], "passArgs": true},
  {"match": "profile-controller", "argv": ["{bin}/profile-controller"], "passArgs": true},
  {"match": "access-management|/kfam", "argv": ["{bin}/access-management"], "passArgs": true},
  {"match": "tensorboard-controller", "argv": ["{bin}/tensorboard-controller"], "passArgs": true},
  {"match": "pvcviewer-controller", "argv": ["{bin}/pvcviewer-controller"], "passArgs": true},
  {"match": "admission-webhook|poddefaults-webhook", "argv": ["{bin}/admission-webhook"], "passArgs": true},
  {"match": "cmd:tensorboard", "argv": ["{python}", "-m", "kubeflow_rm_amd.images.tensorboard_server"], "passArgs": true},
  {"match": "cmd:jupyter|cmd:start-notebook.sh|cmd:start.sh", "argv": ["{python}", "-m", "kubeflow_rm_amd.images.notebook_server"], "zygote": "torch,kubeflow_rm_amd.images.notebook_server"},
  {"match": "oauth-proxy|oauth_proxy", "argv": ["{python}", "-m", "kubeflow_rm_amd.images.oauth_proxy"], "passArgs": true},
  {"match": "filebrowser", "argv": ["{python}", "-m", "kubeflow_rm_amd.images.filebrowser"], "passArgs": true},
  {"match": "jupyter-web-app|crud-web-apps/jupyter", "argv": ["{python}", "-m", "kubeflow_rm_amd.webapps.jupyter"]},
  {"match": "tensorboards-web-app|crud-web-apps/tensorboards", "argv": ["{python}", "-m", "kubeflow_rm_amd.webapps.tensorboards"]},
  {"match": "volumes-web-app|crud-web-apps/volumes", "argv": ["{python}", "-m", "kubeflow_rm_amd.webapps.volumes"]},
  {"match": "centraldashboard", "argv": ["{python}", "-m", "kubeflow_rm_amd.webapps.dashboard"]},
  {"match": "tensorboard|tensorflow/tensorflow", "argv": ["{python}", "-m", "kubeflow_rm_amd.images.tensorboard_server"], "passArgs": true},
  {"match": "jupyter|notebook|scipy|pytorch|tensorflow|codeserver|code-server|rstudio|workbench|s2i-", "argv": ["{python}", "-m", "kubeflow_rm_amd.images.notebook_server"], "zygote": "torch,kubeflow_rm_amd.images.notebook_server"},
  {"match": ".*", "argv": ["{python}", "-m", "kubeflow_rm_amd.images.generic_server"], "passArgs": true}
])";
}  // namespace

// ---------------------------------------------------------------------------------------------
struct ContainerRt {
  std::string name;
  bool init = false;
  bool sidecar = false;  // native sidecar: an init container with restartPolicy: Always (K8s 1.29)
  pid_t pid = -1;
  std::string state = "waiting";  // waiting | running | terminated
  std::string reason = "ContainerCreating";
  std::string started_at, finished_at, message;
  int exit_code = 0;
  int restarts = 0;
  bool ready = false, started_probe_ok = true;
  int ready_ok = 0, ready_fail = 0, live_fail = 0, startup_ok = 0, startup_fail = 0;
  double next_ready_probe = 0, next_live_probe = 0, next_startup_probe = 0, backoff_until = 0;
  double run_started = 0;
  uint64_t probe_gen = 0;  // Prober generation of this run: verdicts of earlier runs are dropped
  Json last_state = Json::object();
  std::string log_path, term_path;
  // forked by a zygote (not our child): the exit status arrives on this connection; -1 = our own
  // child (waitpid). zorphan: the zygote went away first, exit is noticed by kill(pid, 0)
  int zfd = -1;
  bool zorphan = false;
  // what the running process was started with (pods/exec runs commands in the same environment)
  std::vector<std::string> envv;
  std::string cwd;
  std::vector<int> cpus;
};

struct Kubelet::PodRuntime {
  std::string uid, ns, name, dir, ip;
  std::string app_ip;  // where its apps listen: ip, or the private address behind the inbound listeners
  std::vector<std::unique_ptr<HttpServer>> inbound;  // one per containerPort of a mesh-injected pod
  Placement gpus;
  int rdzv_port = 0;  // torch.distributed rendezvous port of a multi-GPU pod (unique on the node)
  bool gpu_ok = true;
  std::string gpu_error;
  std::shared_ptr<PodNetns> netns;  // kubelet --pod-netns: the pod's own network namespace  // why the device plugin refused the pod (UnexpectedAdmissionError message)
  std::map<std::string, std::string> mounts;  // mountPath -> host dir (per container union)
  std::vector<ContainerRt> init, main;
  size_t init_done = 0;
  bool init_failed = false;
  bool readiness_published = false;  // gpu-readiness sidecar report copied to the pod annotation
  std::string start_time;
  bool terminating = false;
  double kill_deadline = 0;
  bool announced_kill = false;
  // held by a reconcile pass for this pod, and by stop() around terminate_pod: the workqueue keeps
  // one worker per key, stop() comes from outside it
  std::mutex op_mu;
};

namespace {
std::string comgr_seed_dir();
}  // namespace

Kubelet::Kubelet(std::shared_ptr<Client> c, KubeletConfig cfg) : c_(std::move(c)), cfg_(std::move(cfg)) {
  comgr_seed_ = comgr_seed_dir();  // set before any thread: pod workers read it (link_comgr_seed)
  // pod addresses start at a random point of the 16-bit range: on a node without per-pod network
  // namespaces, a process a previous kubelet on this host left behind (a test cluster stopped a
  // moment ago) can still hold <addr>:<port>, and every instance counting from .0.2 would hand
  // that address straight out again
  {
    std::random_device rd;
    next_ip_ = 2 + rd() % 60000;
  }
  GpuTopology topo = cfg_.gpus >= 0            ? GpuTopology::synthetic(cfg_.gpus)
                     : !cfg_.sysfs_root.empty() ? GpuTopology::discover(SysfsRoots::under(cfg_.sysfs_root))
                                                : GpuTopology::discover();
  alloc_ = std::make_unique<GpuAllocator>(topo);
  recipes_ = Json::parse(kDefaultRecipes);
  if (!cfg_.recipes_file.empty()) {
    std::string t;
    Json extra;
    if (read_file(cfg_.recipes_file, t) && Json::try_parse(t, extra) && extra.is_array()) {
      Json merged = extra;
      for (const auto& r : recipes_.as_array()) merged.push_back(r);
      recipes_ = merged;
    }
  }
  for (const auto& r : recipes_.as_array()) recipe_re_.emplace_back(r["match"].as_string(), std::regex::icase);
  epfd_ = ::epoll_create1(EPOLL_CLOEXEC);
  wake_fd_ = ::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  if (epfd_ >= 0 && wake_fd_ >= 0) {
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = wake_fd_;
    ::epoll_ctl(epfd_, EPOLL_CTL_ADD, wake_fd_, &ev);
  }
  if (cfg_.root_dir.empty()) cfg_.root_dir = "/tmp/kflite-" + random_hex(4);
  make_dirs(cfg_.root_dir + "/pods");
  make_dirs(cfg_.root_dir + "/pv");
  rec_ = std::make_unique<EventRecorder>(c_, "kubelet");
  prober_ = std::make_unique<Prober>([this](const std::string& ns, const std::string& name) {
    if (ctl_) ctl_->enqueue(Request{ns, name});
  });
}

// Process pods share the host network namespace, and torch's TCPStore listens on the wildcard
// address: two multi-GPU notebooks with the same MASTER_PORT would collide whatever MASTER_ADDR
// says. Each multi-GPU pod gets its own port (unique among this node's pods and free on the host
// when handed out); MASTER_ADDR is the pod's own 127.x address. (In a real cluster every pod has
// its own network namespace and the fixed port would do.)
int Kubelet::alloc_rdzv_port() {
  std::lock_guard<std::mutex> g(mu_);
  for (int port = 29500; port < 29500 + 4096; ++port) {
    if (rdzv_ports_.count(port)) continue;
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) break;
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port));
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    // torch's TCPStore listens with SO_REUSEADDR, so a released port in TIME_WAIT is reusable
    const int one = 1;
    ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    const bool free_now = ::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) == 0;
    ::close(fd);
    if (!free_now) continue;
    rdzv_ports_.insert(port);
    return port;
  }
  return 29500;  // nothing free in the range: fall back to torch's default and let it report
}

Kubelet::~Kubelet() {
  stop();
  prober_->stop();  // also when start() never ran
  for (auto& kv : watched_) ::close(kv.first);
  if (epfd_ >= 0) ::close(epfd_);
  if (wake_fd_ >= 0) ::close(wake_fd_);
}

std::vector<std::string> Kubelet::resolve_argv(const Json& container, std::string* why, std::string* zygote) const {
  if (zygote) zygote->clear();
  std::vector<std::string> cmd, args;
  for (const auto& x : container["command"].as_array()) cmd.push_back(x.as_string());
  for (const auto& x : container["args"].as_array()) args.push_back(x.as_string());
  if (!cmd.empty() && !which(cmd[0]).empty()) {
    if (why) *why = "command";
    std::vector<std::string> out = cmd;
    out.insert(out.end(), args.begin(), args.end());
    return out;
  }
  std::vector<std::string> keys;
  if (!cmd.empty()) {
    std::string base = cmd[0].substr(cmd[0].rfind('/') == std::string::npos ? 0 : cmd[0].rfind('/') + 1);
    keys.push_back("cmd:" + base);
  }
  keys.push_back(container["image"].as_string());
  for (const auto& key : keys) {
    const auto& recipes = recipes_.as_array();
    for (size_t i = 0; i < recipes.size(); ++i) {
      const Json& r = recipes[i];
      if (!std::regex_search(key, recipe_re_[i])) continue;
      std::vector<std::string> out;
      for (const auto& a : r["argv"].as_array()) {
        std::string s = replace_all(a.as_string(), "{python}", cfg_.python);
        s = replace_all(s, "{bin}", cfg_.bin_dir);
        out.push_back(s);
      }
      if (r["passArgs"].as_bool()) {
        if (cmd.size() > 1) out.insert(out.end(), cmd.begin() + 1, cmd.end());
        out.insert(out.end(), args.begin(), args.end());
      }
      if (why) *why = "recipe:" + r["match"].as_string();
      if (zygote) *zygote = r["zygote"].as_string();
      return out;
    }
  }
  return {"sleep", "infinity"};
}

// ---- node registration ------------------------------------------------------------------------
Json Kubelet::node_object() const {
  const auto& topo = alloc_->topology();
  int64_t hbm_gib = 0;
  for (const auto& g : topo.gpus) hbm_gib += g.hbm_bytes >> 30;
  const long cpus = cfg_.node_cpus > 0 ? cfg_.node_cpus : ::sysconf(_SC_NPROCESSORS_ONLN);
  const long pages = ::sysconf(_SC_PHYS_PAGES), psize = ::sysconf(_SC_PAGE_SIZE);
  Json cap{{"cpu", std::to_string(cpus)},
           {"memory", cfg_.node_memory_gib > 0 ? std::to_string(cfg_.node_memory_gib) + "Gi"
                                                : std::to_string(static_cast<int64_t>(pages) * psize / 1024) + "Ki"},
           {"pods", "110"},
           {"ephemeral-storage", "1Ti"},
           {GPU_RESOURCE, std::to_string(topo.size())},
           {GPU_MEMORY_RESOURCE, std::to_string(hbm_gib)}};
  Json labels{{"kubernetes.io/hostname", cfg_.node_name},
              {"kubernetes.io/os", "linux"},
              {"kubernetes.io/arch", "amd64"},
              {"node.kubernetes.io/instance-type", "mi355x-x" + std::to_string(topo.size())},
              {"amd.com/gpu.present", topo.size() > 0 ? "true" : "false"},
              {"amd.com/gpu.count", std::to_string(topo.size())}};
  if (topo.size() > 0) {
    labels["amd.com/gpu.family"] = "CDNA4";
    labels["amd.com/gpu.arch"] = topo.gpus[0].gfx;
    labels["amd.com/gpu.product-name"] = "AMD_Instinct_MI355X";
    labels["amd.com/gpu.xgmi"] = topo.describe().find("full-mesh") != std::string::npos ? "full-mesh" : "partial";
    // partition modes and the HBM each schedulable device really has (CPX/NPS2 split a package)
    labels["amd.com/gpu.compute-partitioning-mode"] = to_lower(topo.gpus[0].compute_partition);
    labels["amd.com/gpu.memory-partitioning-mode"] = to_lower(topo.gpus[0].memory_partition);
    labels["amd.com/gpu.hbm-gib-per-device"] = std::to_string(topo.gpus[0].hbm_bytes >> 30);
    labels["amd.com/gpu.packages"] = std::to_string(topo.physical_count());
  }
  return Json{{"apiVersion", "v1"},
              {"kind", "Node"},
              {"metadata", Json{{"name", cfg_.node_name}, {"labels", labels},
                                {"annotations", Json{{"amd.com/gpu-topology", topo.to_json().dump()},
                                                     {"kfamd.io/pod-network", netns_ ? "netns" : "host"}}}}},
              {"spec", Json{{"providerID", "kflite://" + cfg_.node_name}}},
              {"status", Json{{"capacity", cap},
                              {"allocatable", cap},
                              {"addresses", Json::array({Json{{"type", "InternalIP"}, {"address", "127.0.0.1"}},
                                                         Json{{"type", "Hostname"}, {"address", cfg_.node_name}}})},
                              {"nodeInfo", Json{{"kubeletVersion", "v1.29.0-kflite"}, {"containerRuntimeVersion", "kflite-process://1"},
                                                {"operatingSystem", "linux"}, {"architecture", "amd64"},
                                                {"osImage", "kflite process runtime"}}},
                              {"conditions", Json::array({Json{{"type", "Ready"}, {"status", "True"}, {"reason", "KubeletReady"},
                                                               {"message", "kubelet is posting ready status"},
                                                               {"lastHeartbeatTime", rfc3339_now()},
                                                               {"lastTransitionTime", rfc3339_now()}}})}}}};
}

void Kubelet::start() {
  // pod network namespaces need the privilege to create them and an enforcement point to reach the
  // apps through (the gateway's inbound handler)
  std::string why;
  const bool capable = cfg_.pod_netns != "off" && pod_netns_supported(&why);
  netns_ = capable && inbound_;
  if (netns_) relay_ = std::make_unique<EgressRelay>();
  if (cfg_.pod_netns == "on" && !netns_)
    KF_ERROR("kubelet", "--pod-netns=on but pods cannot get a network namespace; they fail admission",
             Json{{"reason", capable ? "no policy enforcer (gateway) on this node" : why}});
  else if (cfg_.pod_netns == "auto" && !netns_)
    KF_WARN("kubelet", "pods share the host network namespace (private-address convention only)",
            Json{{"reason", capable ? "no policy enforcer (gateway) on this node" : why}});
  Json node = node_object();
  Json existing;
  if (c_->get("v1", "Node", "", cfg_.node_name, existing).code == 404) {
    Json n = node;
    c_->create(n);
  }
  c_->update_with_retry(
      "v1", "Node", "", cfg_.node_name,
      [&](Json& o) {
        o["status"] = node["status"];
        return true;
      },
      true);
  c_->update_with_retry("v1", "Node", "", cfg_.node_name, [&](Json& o) {
    o["metadata"]["labels"] = node.at_path({"metadata", "labels"});
    o["metadata"]["annotations"] = node.at_path({"metadata", "annotations"});
    return true;
  });
  if (cfg_.pod_zygote) start_zygotes();
  start_warm_ops();
  running_ = true;
  hb_ = std::thread([this] {
    set_thread_name("kubelet-hb");
    heartbeat_loop();
  });
  if (epfd_ >= 0 && wake_fd_ >= 0) {
    exit_watch_ = std::thread([this] {
      set_thread_name("kubelet-exits");
      exit_watch_loop();
    });
  }
}

void Kubelet::watch_exit(pid_t pid, const std::string& ns, const std::string& name) {
  if (epfd_ < 0 || pid <= 0) return;
#ifdef SYS_pidfd_open
  const int pfd = static_cast<int>(::syscall(SYS_pidfd_open, pid, 0));
#else
  const int pfd = -1;
#endif
  if (pfd < 0) return;  // no pidfd (old kernel): the startup re-sync still notices the exit
  ::fcntl(pfd, F_SETFD, FD_CLOEXEC);
  watch_fd(pfd, ns, name);
}

// fd readable = the container exited (a pidfd, or a zygote connection carrying the exit status);
// the watch owns fd and closes it when it fires
void Kubelet::watch_fd(int fd, const std::string& ns, const std::string& name) {
  if (epfd_ < 0 || fd < 0) {
    if (fd >= 0) ::close(fd);
    return;
  }
  std::lock_guard<std::mutex> g(watch_mu_);
  watched_[fd] = {ns, name};
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = fd;
  if (::epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev) != 0) {
    watched_.erase(fd);
    ::close(fd);
  }
}


void Kubelet::exit_watch_loop() {
  epoll_event evs[32];
  while (running_) {
    const int n = ::epoll_wait(epfd_, evs, 32, 1000);
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd == wake_fd_) continue;
      std::pair<std::string, std::string> key;
      {
        std::lock_guard<std::mutex> g(watch_mu_);
        auto it = watched_.find(fd);
        if (it == watched_.end()) continue;
        key = it->second;
        watched_.erase(it);
        ::epoll_ctl(epfd_, EPOLL_CTL_DEL, fd, nullptr);
        ::close(fd);
      }
      // the pidfd is readable once the process has exited (not reaped: reconcile's waitpid does)
      if (ctl_) ctl_->enqueue(Request{key.first, key.second});
    }
  }
}

void Kubelet::heartbeat_loop() {
  while (running_) {
    for (int i = 0; i < 100 && running_; ++i) {
      ::usleep(100000);
      if (cfg_.pod_zygote && i % 10 == 9 && running_) supervise_zygotes();
      if (running_) supervise_warm_ops();
    }
    if (!running_) break;
    c_->update_with_retry(
        "v1", "Node", "", cfg_.node_name,
        [&](Json& o) {
          for (auto& c : o["status"]["conditions"].mut_array())
            if (c["type"].as_string() == "Ready") c["lastHeartbeatTime"] = rfc3339_now();
          return true;
        },
        true);
  }
}

void Kubelet::stop() {
  if (metrics_registered_) {  // the collectors capture `this`
    for (const char* n : {"kfamd_gpu_allocated", "kfamd_gpu_hbm_allocated_bytes", "kfamd_gpu_vram_used_bytes",
                          "kfamd_gpu_vram_total_bytes", "kfamd_gpu_busy_percent", "kfamd_gpu_gfx_activity_percent",
                          "kfamd_gpu_hbm_activity_percent", "kfamd_gpu_power_watts", "kfamd_gpu_temperature_celsius",
                          "kfamd_gpu_gfxclk_mhz", "kfamd_gpu_energy_joules_total", "kfamd_gpu_xgmi_read_bytes_total",
                          "kfamd_gpu_xgmi_write_bytes_total", "kfamd_gpu_throttle_residency_ratio"})
      Registry::global().unregister(n);
    metrics_registered_ = false;
  }
  if (!running_.exchange(false)) return;
  stopping_ = true;
  prober_->stop();  // waits for in-flight probes (each bounded by its timeoutSeconds)
  if (hb_.joinable()) hb_.join();
  if (wake_fd_ >= 0) {
    const uint64_t one = 1;
    (void)!::write(wake_fd_, &one, sizeof one);
  }
  if (exit_watch_.joinable()) exit_watch_.join();
  // the epoll set and eventfd stay open until the destructor: a reconcile still in flight may
  // register one more pidfd
  std::vector<std::shared_ptr<PodRuntime>> all;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : pods_) all.push_back(kv.second);
  }
  for (auto& rt : all) {
    std::lock_guard<std::mutex> pl(rt->op_mu);
    terminate_pod(*rt, 0);
  }
  if (relay_) relay_->stop();
  stop_zygotes();
  stop_warm_ops();
}

// ---- process management ---------------------------------------------------------------------------
namespace {
// The child inherits the spawning thread's CPU mask: pin this thread to `cpus` around the spawn
// (race-free: the child starts with the mask, before any of its threads exist), then restore.
struct ScopedThreadAffinity {
  cpu_set_t saved;
  bool active = false;
  explicit ScopedThreadAffinity(const std::vector<int>& cpus) {
    if (cpus.empty() || ::sched_getaffinity(0, sizeof saved, &saved) != 0) return;
    cpu_set_t want;
    CPU_ZERO(&want);
    for (int c : cpus)
      if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &saved)) CPU_SET(c, &want);  // within our own cgroup/cpuset
    if (CPU_COUNT(&want) == 0) return;
    active = ::sched_setaffinity(0, sizeof want, &want) == 0;
  }
  ~ScopedThreadAffinity() {
    if (active) ::sched_setaffinity(0, sizeof saved, &saved);
  }
};

// `ns`: the pod's network namespace; the child starts in it (posix_spawn from a thread inside it)
pid_t spawn(const std::vector<std::string>& argv, const std::vector<std::string>& env, const std::string& cwd,
            const std::string& log_path, std::string* err, const std::vector<int>& cpus = {},
            const PodNetns* ns = nullptr) {
  ScopedThreadAffinity pin(cpus);
  posix_spawn_file_actions_t fa;
  posix_spawnattr_t at;
  posix_spawn_file_actions_init(&fa);
  posix_spawnattr_init(&at);
  posix_spawnattr_setflags(&at, POSIX_SPAWN_SETSID | POSIX_SPAWN_SETSIGDEF | POSIX_SPAWN_SETSIGMASK);
  sigset_t all, none;
  sigfillset(&all);
  sigemptyset(&none);
  posix_spawnattr_setsigdefault(&at, &all);
  posix_spawnattr_setsigmask(&at, &none);
  posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  posix_spawn_file_actions_addopen(&fa, 1, log_path.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
  posix_spawn_file_actions_adddup2(&fa, 1, 2);
  posix_spawn_file_actions_addchdir_np(&fa, cwd.c_str());
  std::vector<char*> av, ev;
  for (const auto& a : argv) av.push_back(const_cast<char*>(a.c_str()));
  av.push_back(nullptr);
  for (const auto& e : env) ev.push_back(const_cast<char*>(e.c_str()));
  ev.push_back(nullptr);
  std::string exe = which(argv[0]);
  pid_t pid = -1;
  int rc;
  {
    NetnsScope in(ns);
    rc = !in.ok() ? errno : exe.empty() ? ENOENT : posix_spawn(&pid, exe.c_str(), &fa, &at, av.data(), ev.data());
  }
  posix_spawn_file_actions_destroy(&fa);
  posix_spawnattr_destroy(&at);
  if (rc != 0) {
    if (err) *err = std::string("exec ") + argv[0] + ": " + std::strerror(rc);
    return -1;
  }
  return pid;
}

// An exec probe's process (on a Prober thread): wait up to timeout_ms for it (pidfd + poll, no
// spinning), SIGKILL its group past that, reap it. Returns its exit code (non-zero on timeout).
int wait_probe_process(pid_t pid, int timeout_ms) {
  int st = 0;
#ifdef SYS_pidfd_open
  const int pfd = static_cast<int>(::syscall(SYS_pidfd_open, pid, 0));
#else
  const int pfd = -1;
#endif
  bool timed_out = false, waited = false;
  if (pfd >= 0) {
    pollfd p{pfd, POLLIN, 0};
    int rc;
    do rc = ::poll(&p, 1, timeout_ms);
    while (rc < 0 && errno == EINTR);
    ::close(pfd);
    // a poll that fails for any other reason falls back to the deadline loop below: never a
    // blocking waitpid on a probe that may not exit
    if (rc >= 0) {
      timed_out = rc == 0;
      waited = true;
    }
  }
  if (!waited) {
    const double deadline = now_seconds() + timeout_ms / 1000.0;
    pid_t r;
    while ((r = ::waitpid(pid, &st, WNOHANG)) == 0 || (r < 0 && errno == EINTR)) {
      if (now_seconds() > deadline) {
        timed_out = true;
        break;
      }
      ::usleep(5000);
    }
    if (!timed_out) {
      if (r < 0) return 128;  // not our child any more (reaped elsewhere)
      return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
    }
  }
  if (timed_out) ::kill(-pid, SIGKILL);
  while (::waitpid(pid, &st, 0) < 0 && errno == EINTR) {
  }
  if (timed_out) return 124;
  return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
}

// returns true when the process has exited (fills status)
bool reap(pid_t pid, int& exit_code, std::string& reason) {
  int st = 0;
  pid_t r = ::waitpid(pid, &st, WNOHANG);
  if (r == 0) return false;
  if (r < 0) {
    exit_code = 128;
    reason = "Error";
    return true;
  }
  if (WIFEXITED(st)) {
    exit_code = WEXITSTATUS(st);
  } else if (WIFSIGNALED(st)) {
    exit_code = 128 + WTERMSIG(st);
  }
  reason = exit_code == 0 ? "Completed" : (exit_code == 137 ? "OOMKilled" : "Error");
  if (WIFSIGNALED(st) && WTERMSIG(st) == SIGKILL) reason = "Error";
  return true;
}

// Container start through a zygote (kubeflow_rm_amd/images/zygote.py): one connection per container,
// request = the argv after the interpreter + env + cwd + log + CPU mask, reply {"pid": N}; the exit
// status arrives later on the same connection (*zfd keeps it). Returns -1 when the zygote is not
// there or refuses (the caller then spawns a fresh interpreter).
pid_t zygote_spawn(const std::string& sock, const std::vector<std::string>& argv, const std::vector<std::string>& env,
                   const std::string& cwd, const std::string& log_path, const std::vector<int>& cpus, int* zfd,
                   std::string* err, const std::string& netns_path = "", int warm_device = -1, bool* warm = nullptr) {
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  if (sock.size() >= sizeof a.sun_path) {
    ::close(fd);
    return -1;
  }
  std::memcpy(a.sun_path, sock.c_str(), sock.size() + 1);
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
    ::close(fd);
    return -1;
  }
  Json req{{"argv", Json::array()}, {"env", Json::array()}, {"cwd", cwd}, {"log", log_path}, {"cpus", Json::array()}};
  for (size_t i = 1; i < argv.size(); ++i) req["argv"].push_back(argv[i]);
  for (const auto& e : env) req["env"].push_back(e);
  for (int c : cpus) req["cpus"].push_back(static_cast<int64_t>(c));
  if (!netns_path.empty()) req["netns"] = netns_path;  // the child joins the pod's namespace first
  if (warm_device >= 0) req["warm_device"] = warm_device;  // a warm child of that GPU may take it
  const std::string line = req.dump() + "\n";
  size_t off = 0;
  while (off < line.size()) {
    const ssize_t n = ::send(fd, line.data() + off, line.size() - off, MSG_NOSIGNAL);
    if (n <= 0) {
      ::close(fd);
      return -1;
    }
    off += static_cast<size_t>(n);
  }
  // the reply line, byte by byte: a fast-exiting child's exit line may follow it in the same segment
  std::string reply;
  const double deadline = now_seconds() + 10;
  while (reply.empty() || reply.back() != '\n') {
    pollfd p{fd, POLLIN, 0};
    const int left = static_cast<int>((deadline - now_seconds()) * 1000);
    if (left <= 0 || ::poll(&p, 1, left) <= 0) break;
    char ch;
    if (::recv(fd, &ch, 1, 0) != 1) break;
    reply += ch;
  }
  Json r;
  if (!Json::try_parse(reply, r) || !r["pid"].is_number()) {
    if (err) *err = "zygote: " + (r["error"].is_string() ? r["error"].as_string() : std::string("no reply"));
    ::close(fd);
    return -1;
  }
  *zfd = fd;
  if (warm) *warm = r["warm"].as_bool();
  return static_cast<pid_t>(r["pid"].as_int());
}

// reap() for either kind of container process: our child (waitpid) or a zygote's (its status line)
bool reap_container(pid_t pid, int& zfd, bool& zorphan, int& exit_code, std::string& reason) {
  if (zorphan) {  // the zygote died before its child: no status to be had, only whether it is gone
    if (::kill(pid, 0) == 0 || errno == EPERM) return false;
    exit_code = 137;
    reason = "Error";
    zorphan = false;
    return true;
  }
  if (zfd < 0) return reap(pid, exit_code, reason);
  char buf[512];
  const ssize_t n = ::recv(zfd, buf, sizeof buf - 1, MSG_DONTWAIT);
  if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) return false;
  ::close(zfd);
  zfd = -1;
  Json st;
  if (n > 0 && Json::try_parse(std::string(buf, static_cast<size_t>(n)), st) && st["exit"].is_number()) {
    exit_code = static_cast<int>(st["exit"].as_int());
    const int sig = static_cast<int>(st["signal"].as_int());
    reason = exit_code == 0 ? "Completed" : (exit_code == 137 ? "OOMKilled" : "Error");
    if (sig == SIGKILL) reason = "Error";
    return true;
  }
  zorphan = true;  // EOF without a status: the zygote is gone
  return reap_container(pid, zfd, zorphan, exit_code, reason);
}
}  // namespace

// One pre-imported interpreter per distinct recipe preload list. Started with the container base
// env (PATH, LD_LIBRARY_PATH, HSA_*, KFAMD_*, PYTHONPATH = the framework): the forked containers
// replace it with their own. A zygote that is not up yet (the first seconds after node start) or
// that died is simply not used.
bool Kubelet::spawn_zygote(Zygote& z) {
  std::vector<std::string> env;
  for (char** e = environ; *e; ++e) {
    std::string kv = *e;
    const std::string k = kv.substr(0, kv.find('='));
    if (k == "PATH" || k == "LANG" || k == "LD_LIBRARY_PATH" || k == "TMPDIR" || starts_with(k, "HSA_") ||
        starts_with(k, "KFAMD_") || starts_with(k, "ROCM") || k == "OMP_NUM_THREADS" || k == "HOME")
      env.push_back(kv);
  }
  env.push_back("PYTHONPATH=" + cfg_.repo_root);
  env.push_back("PYTHONUNBUFFERED=1");
  std::vector<std::string> argv{cfg_.python, "-m", "kubeflow_rm_amd.images.zygote", "--socket", z.sock, "--preload", z.preload};
  // warm GPU children (zygote.py): one per node GPU, HIP + device context + first op done before a
  // 1-GPU pod on that device is admitted; real GPUs only, torch zygotes only
  if (cfg_.pod_warm_gpus && contains(z.preload, "torch") && alloc_->topology().source != "synthetic" &&
      ::access("/dev/kfd", R_OK | W_OK) == 0 && alloc_->topology().size() > 0) {
    std::vector<std::string> ids;
    for (int i = 0; i < alloc_->topology().size(); ++i) ids.push_back(std::to_string(i));
    argv.push_back("--warm-devices");
    argv.push_back(join(ids, ","));
  }
  std::string err;
  z.pid = spawn(argv, env, cfg_.root_dir, z.log, &err);
  z.started = now_seconds();
  return z.pid > 0;
}

void Kubelet::start_zygotes() {
  int i = 0;
  std::lock_guard<std::mutex> g(zy_mu_);
  for (const auto& r : recipes_.as_array()) {
    const std::string pre = r["zygote"].as_string();
    if (pre.empty() || zygotes_.count(pre)) continue;
    Zygote z;
    z.preload = pre;
    z.sock = cfg_.root_dir + "/zygote-" + std::to_string(i) + ".sock";
    z.log = cfg_.root_dir + "/zygote-" + std::to_string(i) + ".log";
    ++i;
    if (spawn_zygote(z)) zygotes_[pre] = z;
  }
}

// A zygote that exited (killed, OOM, crashed) is started again; containers meanwhile start fresh
// interpreters. One that keeps exiting right after its start (e.g. it refused to serve because its
// preload opened the GPU driver) is given up after three tries.
void Kubelet::supervise_zygotes() {
  std::lock_guard<std::mutex> g(zy_mu_);
  for (auto& kv : zygotes_) {
    Zygote& z = kv.second;
    int code = 0;
    std::string reason;
    if (z.pid <= 0 || !reap(z.pid, code, reason)) continue;
    z.quick_exits = now_seconds() - z.started < 30 ? z.quick_exits + 1 : 0;
    {
      std::ofstream lf(z.log, std::ios::app);
      lf << "# kflite: zygote " << z.pid << " exited (" << code << ")"
         << (z.quick_exits >= 3 ? "; not restarted (exits right after start)" : "; restarting") << "\n";
    }
    z.pid = -1;
    static const auto restarts =
        Registry::global().counter("kubelet_zygote_restarts_total", "pre-imported interpreters restarted after an exit");
    if (z.quick_exits < 3 && spawn_zygote(z)) restarts->inc();
  }
}

// Warm readiness ops (kfamd-readiness --warm-op): per node GPU, an op process with HIP, the device
// context and a hardware queue already up, waiting on <root>/warm-readiness/gpu-<d>.sock for the
// gpu-readiness sidecar of a 1-GPU pod on <d> (readiness.cc claim_warm_op). Each serves one pod and
// exits; the next one starts kWarmOpRespawnS later (after the claiming pod's own GPU bring-up).
namespace {
constexpr double kWarmOpRespawnS = 0.3;

// The node's comgr seed: the first RCCL communicator in a process builds RCCL's device code through
// comgr (~680 MB of cache entries, 3.8 s of the 5.5 s first `ncclCommInitAll` on MI355X; every later
// process with that cache takes 1.7 s, profiles/r6k_rccl_init). Each namespace has its own cache
// (container_env: tenants never share writable code objects), so each namespace's first RCCL pod
// paid it. The kubelet builds the entries once per node with its own readiness op (a trusted binary,
// a clean env, GPU 0, at low priority) into a node directory outside every pod, and a namespace's
// cache starts as reflink copies of them (copy-on-write: a tenant that rewrites an entry changes only
// its own namespace's copy). Where the filesystem has no reflinks the entries are read-only hard
// links instead. Process pods run under the kubelet's uid, so such a pod could still chmod and rewrite
// a shared inode; comgr itself only adds and removes content-hashed entries, never rewrites them.
std::string comgr_seed_dir() {
  if (const char* d = std::getenv("KFAMD_COMGR_SEED_DIR")) return d;
  const char* xdg = std::getenv("XDG_CACHE_HOME");
  const char* home = std::getenv("HOME");
  const std::string base = xdg && *xdg ? xdg : std::string(home && *home ? home : "/tmp") + "/.cache";
  return base + "/kfamd/comgr-seed";
}
}  // namespace

void Kubelet::seed_comgr_cache() {
  if (::access((comgr_seed_ + "/.complete").c_str(), F_OK) == 0) return;
  // one build per host (several kubelets may share it, e.g. test clusters): a live kubelet's build
  // in progress is left to finish; the leftovers of dead ones are removed
  const std::filesystem::path seed(comgr_seed_);
  const std::string prefix = seed.filename().string() + ".building-";
  std::error_code ec;
  std::vector<std::filesystem::path> stale;
  for (std::filesystem::directory_iterator it(seed.parent_path(), ec), end; !ec && it != end; it.increment(ec)) {
    const std::string name = it->path().filename().string();
    if (name.rfind(prefix, 0) != 0) continue;
    const pid_t owner = static_cast<pid_t>(std::atol(name.c_str() + prefix.size()));
    if (owner > 0 && (::kill(owner, 0) == 0 || errno == EPERM)) return;
    stale.push_back(it->path());
  }
  for (const auto& d : stale) std::filesystem::remove_all(d, ec);
  ec.clear();
  const std::string tmp = comgr_seed_ + ".building-" + std::to_string(::getpid());
  std::filesystem::remove_all(tmp, ec);
  make_dirs(tmp);
  std::vector<std::string> env;
  for (char** e = environ; *e; ++e) {
    const std::string kv = *e, k = kv.substr(0, kv.find('='));
    if (k == "PATH" || k == "LANG" || k == "LD_LIBRARY_PATH" || k == "TMPDIR" || k == "HOME" || starts_with(k, "HSA_") ||
        starts_with(k, "ROCM"))
      env.push_back(kv);
  }
  env.push_back("AMD_COMGR_CACHE_DIR=" + tmp);
  env.push_back("ROCR_VISIBLE_DEVICES=0");
  env.push_back("HIP_VISIBLE_DEVICES=0");
  std::vector<std::string> argv = {cfg_.bin_dir + "/kfamd-readiness", "--rccl-single", "--skip-ln", "--iters", "1"};
  if (::access("/usr/bin/nice", X_OK) == 0) argv.insert(argv.begin(), {"/usr/bin/nice", "-n", "10"});
  std::string err;
  seed_pid_ = spawn(argv, env, tmp, comgr_seed_ + ".log", &err);
}

// supervise tick: the seed build finished -> publish it (rename + marker); failures just leave none
void Kubelet::finish_comgr_seed() {
  if (seed_pid_ <= 0) return;
  int st = 0;
  if (::waitpid(seed_pid_, &st, WNOHANG) != seed_pid_) return;
  seed_pid_ = -1;
  const std::string tmp = comgr_seed_ + ".building-" + std::to_string(::getpid());
  std::error_code ec;
  if (WIFEXITED(st) && WEXITSTATUS(st) == 0 && ::access((comgr_seed_ + "/.complete").c_str(), F_OK) != 0) {
    std::ofstream(tmp + "/.complete") << "1\n";
    std::filesystem::remove_all(comgr_seed_, ec);  // an incomplete earlier attempt
    std::filesystem::rename(tmp, comgr_seed_, ec);  // (another kubelet may have won: then ours goes)
  }
  std::filesystem::remove_all(tmp, ec);
}

namespace {
// dst as a copy-on-write clone of src (FICLONE); false where the filesystem cannot (ext4, tmpfs,
// overlay, another device): the caller falls back
bool reflink(const std::string& src, const std::string& dst) {
  const int in = ::open(src.c_str(), O_RDONLY | O_CLOEXEC);
  if (in < 0) return false;
  const int out = ::open(dst.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
  bool ok = false;
  if (out >= 0) {
    ok = ::ioctl(out, FICLONE, in) == 0;
    ::close(out);
    if (!ok) ::unlink(dst.c_str());
  }
  ::close(in);
  return ok;
}
}  // namespace

// a namespace's new code-object cache starts as reflinks (else read-only hard links) of the node's
// seed entries
void Kubelet::link_comgr_seed(const std::string& cache_dir) {
  if (comgr_seed_.empty() || ::access((comgr_seed_ + "/.complete").c_str(), F_OK) != 0) return;
  std::error_code ec;
  for (std::filesystem::directory_iterator it(comgr_seed_, ec), end; !ec && it != end; it.increment(ec)) {
    const std::string name = it->path().filename().string();
    if (name.rfind("llvmcache-", 0) != 0) continue;
    const std::string dst = cache_dir + "/" + name;
    if (reflink(it->path().string(), dst)) continue;
    ::chmod(it->path().c_str(), 0444);
    (void)::link(it->path().c_str(), dst.c_str());
  }
}

void Kubelet::start_warm_ops() {
  const std::string bin = cfg_.bin_dir + "/kfamd-readiness";
  if (!cfg_.pod_warm_gpus || alloc_->topology().source == "synthetic" || alloc_->topology().size() == 0 ||
      ::access("/dev/kfd", R_OK | W_OK) != 0 || ::access(bin.c_str(), X_OK) != 0)
    return;
  warm_dir_ = cfg_.root_dir + "/warm-readiness";
  make_dirs(warm_dir_);
  ::chmod(warm_dir_.c_str(), 0700);
  std::lock_guard<std::mutex> g(wo_mu_);
  seed_comgr_cache();
  for (int d = 0; d < alloc_->topology().size(); ++d) {
    WarmOp w;
    w.dev = d;
    warm_ops_.push_back(w);
  }
}

void Kubelet::supervise_warm_ops() {
  std::lock_guard<std::mutex> g(wo_mu_);
  finish_comgr_seed();
  const double now = now_seconds();
  for (auto& w : warm_ops_) {
    if (w.pid > 0) {
      int st = 0;
      if (::waitpid(w.pid, &st, WNOHANG) != w.pid) continue;
      // served a pod (exit after its verdict) or failed to warm up (exit 3 within seconds)
      const bool quick = now - w.started < 5.0 && WIFEXITED(st) && WEXITSTATUS(st) == 3;
      w.failures = quick ? w.failures + 1 : 0;
      w.pid = -1;
      w.next_start = now + kWarmOpRespawnS;
    }
    if (w.pid > 0 || w.failures >= 3 || now < w.next_start) continue;
    std::vector<std::string> env;
    for (char** e = environ; *e; ++e) {
      const std::string kv = *e, k = kv.substr(0, kv.find('='));
      if (k == "PATH" || k == "LANG" || k == "LD_LIBRARY_PATH" || k == "TMPDIR" || starts_with(k, "HSA_") ||
          starts_with(k, "KFAMD_") || starts_with(k, "ROCM") || k == "HOME")
        env.push_back(kv);
    }
    // the device plugin's view of a 1-GPU pod on this device (gpu_env_for)
    env.push_back("ROCR_VISIBLE_DEVICES=" + std::to_string(w.dev));
    env.push_back("HIP_VISIBLE_DEVICES=0");
    const std::string sock = warm_dir_ + "/gpu-" + std::to_string(w.dev) + ".sock";
    std::string err;
    w.pid = spawn({cfg_.bin_dir + "/kfamd-readiness", "--warm-op", sock}, env, warm_dir_,
                  warm_dir_ + "/gpu-" + std::to_string(w.dev) + ".log", &err);
    w.started = now;
  }
}

void Kubelet::stop_warm_ops() {
  std::lock_guard<std::mutex> g(wo_mu_);
  for (auto& w : warm_ops_) {
    if (w.pid <= 0) continue;
    ::kill(w.pid, SIGKILL);
    ::waitpid(w.pid, nullptr, 0);
    w.pid = -1;
  }
}

void Kubelet::stop_zygotes() {
  std::map<std::string, Zygote> zs;
  {
    std::lock_guard<std::mutex> g(zy_mu_);
    zs = zygotes_;
  }
  for (auto& kv : zs) {
    if (kv.second.pid <= 0) continue;
    ::kill(-kv.second.pid, SIGTERM);
    int code = 0;
    std::string reason;
    const double deadline = now_seconds() + 5;
    while (!reap(kv.second.pid, code, reason)) {
      if (now_seconds() > deadline) {
        ::kill(-kv.second.pid, SIGKILL);
        ::waitpid(kv.second.pid, nullptr, 0);
        break;
      }
      ::usleep(5000);
    }
    // the entry stays as it is (reconcile workers may still read it; a connect is simply refused)
  }
}

void Kubelet::terminate_pod(PodRuntime& rt, int64_t grace_s) {
  auto kill_all = [&](int sig) {
    for (auto* v : {&rt.init, &rt.main})
      for (auto& c : *v)
        if (c.pid > 0 && c.state == "running") ::kill(-c.pid, sig);
  };
  if (grace_s <= 0) {
    kill_all(SIGKILL);
  } else {
    kill_all(SIGTERM);
  }
  for (auto* v : {&rt.init, &rt.main})
    for (auto& c : *v) {
      if (c.pid <= 0 || c.state != "running") continue;
      double deadline = now_seconds() + static_cast<double>(grace_s);
      int code = 0;
      std::string reason;
      while (!reap_container(c.pid, c.zfd, c.zorphan, code, reason)) {
        if (now_seconds() > deadline) {
          ::kill(-c.pid, SIGKILL);
          deadline = now_seconds() + 5;
        }
        ::usleep(10000);
      }
      c.state = "terminated";
      c.exit_code = code;
      c.reason = reason;
      c.finished_at = ms_now();
      c.pid = -1;
    }
  // the pod's inbound listeners and egress relays go with it (the pod IP may be handed out again)
  for (auto& srv : rt.inbound) srv->stop();
  rt.inbound.clear();
  if (relay_) relay_->remove_pod(rt.uid);
}

bool Kubelet::exec(const std::string& ns, const std::string& pod, const std::string& container,
                   const std::vector<std::string>& argv, double timeout_s, int& exit_code, std::string& output,
                   std::string& err) {
  std::shared_ptr<PodRuntime> rt;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto k = key_to_uid_.find(ns + "/" + pod);
    if (k != key_to_uid_.end()) {
      auto it = pods_.find(k->second);
      if (it != pods_.end()) rt = it->second;
    }
  }
  if (!rt) {
    err = "pod " + pod + " is not running on this node";
    return false;
  }
  std::vector<std::string> envv;
  std::string cwd, dir;
  std::vector<int> cpus;
  {
    std::lock_guard<std::mutex> pl(rt->op_mu);
    const ContainerRt* found = nullptr;
    for (const auto& c : rt->main)
      if (!found && (container.empty() || c.name == container)) found = &c;
    for (const auto& c : rt->init)  // a named native sidecar
      if (!found && !container.empty() && c.name == container) found = &c;
    if (!found) {
      err = "container " + container + " is not valid for pod " + pod;
      return false;
    }
    if (found->state != "running" || found->pid <= 0) {
      err = "container " + found->name + " is not running";
      return false;
    }
    envv = found->envv;
    cwd = found->cwd;
    cpus = found->cpus;
    dir = rt->dir;
  }
  const std::string out_path = dir + "/exec-" + random_hex(6) + ".out";
  std::string serr;
  const pid_t pid = spawn(argv, envv, cwd, out_path, &serr, cpus, rt->netns.get());
  if (pid < 0) {
    err = serr;
    ::unlink(out_path.c_str());
    return false;
  }
  std::string reason;
  double deadline = now_seconds() + timeout_s;
  bool killed = false, too_big = false;
  constexpr size_t kMaxOut = 16u << 20;       // the reply carries at most the last 16 MiB
  constexpr off_t kMaxFile = 64ll << 20;      // a command that writes more is killed (disk + RAM bound)
  double next_size_check = 0;
  while (!reap(pid, exit_code, reason)) {
    const double now = now_seconds();
    if (!killed && now > deadline) {
      ::kill(-pid, SIGKILL);
      killed = true;
      deadline = now + 5;
    }
    if (!killed && now >= next_size_check) {  // bounded output: e.g. `yes` fills 64 MiB in well under a second
      next_size_check = now + 0.01;
      struct stat st{};
      if (::stat(out_path.c_str(), &st) == 0 && st.st_size > kMaxFile) {
        ::kill(-pid, SIGKILL);
        killed = too_big = true;
        deadline = now + 5;
      }
    }
    ::usleep(2000);
  }
  // read only the tail: seek to the last kMaxOut bytes
  output.clear();
  bool truncated = false;
  if (FILE* f = std::fopen(out_path.c_str(), "rb")) {
    if (std::fseek(f, 0, SEEK_END) == 0) {
      const long size = std::ftell(f);
      const long from = size > static_cast<long>(kMaxOut) ? size - static_cast<long>(kMaxOut) : 0;
      truncated = from > 0;
      std::fseek(f, from, SEEK_SET);
      output.resize(static_cast<size_t>(size - from));
      output.resize(std::fread(output.data(), 1, output.size(), f));
    }
    std::fclose(f);
  }
  ::unlink(out_path.c_str());
  if (truncated) output = "[... output truncated ...]\n" + output;
  if (too_big) output += "\ncommand terminated: output exceeded " + std::to_string(kMaxFile >> 20) + " MiB\n";
  else if (killed) output += "\ncommand terminated: timeout after " + std::to_string(static_cast<int>(timeout_s)) + " s\n";
  return true;
}

bool Kubelet::read_logs(const std::string& ns, const std::string& pod, const std::string& container, int64_t tail,
                        std::string& out) {
  std::shared_ptr<PodRuntime> rt;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto k = key_to_uid_.find(ns + "/" + pod);
    if (k == key_to_uid_.end()) return false;
    auto it = pods_.find(k->second);
    if (it == pods_.end()) return false;
    rt = it->second;
  }
  std::string path;
  for (auto* v : {&rt->main, &rt->init})
    for (auto& c : *v)
      if (path.empty() && (container.empty() || c.name == container)) path = c.log_path;
  if (path.empty()) return false;
  if (!read_file(path, out)) out.clear();
  if (tail >= 0) {
    size_t pos = out.size();
    int64_t lines = 0;
    while (pos > 0 && lines <= tail) {
      pos = out.rfind('\n', pos - 1);
      if (pos == std::string::npos) {
        pos = 0;
        break;
      }
      lines++;
    }
    if (lines > tail && pos < out.size()) out = out.substr(pos + 1);
  }
  return true;
}

// ---- reconcile ---------------------------------------------------------------------------------
// ---- one reconcile pass, in units ------------------------------------------
// reconcile() = look up the runtime -> termination | admission (sandbox, GPUs, volumes, containers)
// -> init containers -> long-running containers (start, exit/restart, probes) -> readiness report
// -> status. Everything one pass shares is in PodSync.

namespace {
// Until a pod is Ready the kubelet re-syncs it every 5 ms (cold start is on the notebook's critical
// path; a sync of an unchanged pod costs no API call), afterwards at the 1 s relist.
constexpr double kStartupPoll = 0.005;

Json terminated_state(const ContainerRt& cr) {
  return Json{{"terminated", Json{{"exitCode", cr.exit_code}, {"reason", cr.reason}, {"startedAt", cr.started_at},
                                  {"finishedAt", cr.finished_at}, {"message", cr.message}}}};
}

// a running container whose process ended: record its termination (false when it still runs)
bool handle_exit(ContainerRt& cr) {
  int code = 0;
  std::string reason;
  if (cr.pid <= 0 || cr.state != "running" || !reap_container(cr.pid, cr.zfd, cr.zorphan, code, reason)) return false;
  cr.pid = -1;
  cr.state = "terminated";
  cr.exit_code = code;
  cr.reason = reason;
  cr.finished_at = ms_now();
  cr.ready = false;
  std::string msg;
  if (read_file(cr.term_path, msg)) cr.message = msg.substr(0, 4096);
  else cr.message.clear();
  return true;
}

Json container_status(const ContainerRt& cr, const Json& c) {
  Json state;
  if (cr.state == "running") {
    state = Json{{"running", Json{{"startedAt", cr.started_at}}}};
  } else if (cr.state == "terminated") {
    Json t{{"exitCode", cr.exit_code}, {"reason", cr.reason}, {"startedAt", cr.started_at}, {"finishedAt", cr.finished_at},
           {"containerID", "kflite://" + cr.name}};
    if (!cr.message.empty()) t["message"] = cr.message;
    state = Json{{"terminated", t}};
  } else {
    Json w{{"reason", cr.reason.empty() ? "ContainerCreating" : cr.reason}};
    if (!cr.message.empty()) w["message"] = cr.message;
    state = Json{{"waiting", w}};
  }
  Json s{{"name", cr.name}, {"state", state}, {"lastState", cr.last_state}, {"ready", cr.ready},
         {"restartCount", cr.restarts}, {"image", c["image"]}, {"imageID", "kflite-recipe://" + c["image"].as_string()},
         {"started", cr.state == "running"}};
  if (cr.pid > 0) s["containerID"] = "kflite://" + std::to_string(cr.pid);
  return s;
}

bool wants_pod_gpus(const Json& c) {
  return container_integer_request(c, GPU_RESOURCE).value_or(0) > 0 || shares_pod_gpus(c);
}
}  // namespace

struct Kubelet::PodSync {
  const Request& r;
  Json pod;
  std::shared_ptr<PodRuntime> rt;
  std::string uid, restart_policy;
  double next_wake = 1.0;
  const Json& container_spec(const ContainerRt& cr) const {
    for (const auto& c : pod["spec"][cr.init ? "initContainers" : "containers"].as_array())
      if (c["name"].as_string() == cr.name) return c;
    static const Json empty;
    return empty;
  }
};

// the runtime of r's pod; tears down a runtime whose pod is gone or was replaced (new uid)
std::shared_ptr<Kubelet::PodRuntime> Kubelet::lookup_runtime(const Request& r, const ApiError& e, const Json& pod) {
  std::shared_ptr<PodRuntime> rt;
  std::lock_guard<std::mutex> g(mu_);
  auto k = key_to_uid_.find(r.ns + "/" + r.name);
  if (k == key_to_uid_.end()) return rt;
  auto it = pods_.find(k->second);
  if (it != pods_.end()) rt = it->second;
  if (e.code == 404 || (!e && pod.str_at({"metadata", "uid"}) != k->second)) {
    if (rt) {
      std::lock_guard<std::mutex> pl(rt->op_mu);
      terminate_pod(*rt, 0);
      alloc_->release(rt->uid);
      rdzv_ports_.erase(rt->rdzv_port);
      prober_->forget_pod(rt->uid);
      pods_.erase(rt->uid);
    }
    key_to_uid_.erase(k);
    rt.reset();
  }
  return rt;
}

// deletionTimestamp set: stop the containers (grace period), release the node's resources and
// remove the object
void Kubelet::finish_deletion(const Request& r, const Json& pod, const std::shared_ptr<PodRuntime>& rt,
                              std::string* err) {
  if (rt) {
    if (!rt->announced_kill) {
      rt->announced_kill = true;
      for (auto& c : rt->main)
        if (c.state == "running") rec_->event(pod, "Normal", "Killing", "Stopping container " + c.name);
    }
    terminate_pod(*rt, pod.at_path({"metadata", "deletionGracePeriodSeconds"}).as_int(30));
    alloc_->release(rt->uid);
    std::lock_guard<std::mutex> g(mu_);
    rdzv_ports_.erase(rt->rdzv_port);
    prober_->forget_pod(rt->uid);
    pods_.erase(rt->uid);
    key_to_uid_.erase(r.ns + "/" + r.name);
  }
  ApiError de = c_->remove("v1", "Pod", r.ns, r.name, "", 0);
  if (de && de.code != 404) *err = de.message;
}

// device plugin Allocate: topology-aware GPU placement, recorded on the pod
// The count is the one the scheduler and ResourceQuota charged (pod_gpu_count: requests, which
// admission defaulted from limits and forced equal to them). A count that does not parse as a
// whole number fails the pod instead of silently allocating no GPU.
void Kubelet::allocate_gpus(PodRuntime& rt, const Json& pod) {
  auto count = pod_gpu_count(pod, GPU_RESOURCE);
  if (!count) {
    rt.gpu_ok = false;
    rt.gpu_error = "Allocate failed: amd.com/gpu is not a whole, non-negative number of devices";
    return;
  }
  const int want = static_cast<int>(*count);
  if (want <= 0) return;
  if (!alloc_->allocate(rt.uid, want, rt.gpus)) {
    rt.gpu_ok = false;
    return;
  }
  std::vector<std::string> ids, ring;
  for (int d : rt.gpus.devices) ids.push_back(std::to_string(d));
  for (int d : rt.gpus.ring) ring.push_back(std::to_string(d));
  if (rt.gpus.devices.size() > 1) rt.rdzv_port = alloc_rdzv_port();
  c_->update_with_retry("v1", "Pod", rt.ns, rt.name, [&](Json& o) {
    o["metadata"]["annotations"][ANNOTATION_GPU_IDS] = join(ids, ",");
    o["metadata"]["annotations"][ANNOTATION_XGMI_RING] = join(ring, ",");
    o["metadata"]["annotations"]["amd.com/gpu-placement"] = rt.gpus.reason;
    if (rt.rdzv_port) o["metadata"]["annotations"]["kfamd.io/rendezvous"] = rt.ip + ":" + std::to_string(rt.rdzv_port);
    return true;
  });
}

// volumes (emptyDir / PVC / hostPath / configMap / secret) under the sandbox: volume name -> host dir
std::map<std::string, std::string> Kubelet::prepare_volumes(PodRuntime& rt, const Json& pod) {
  std::map<std::string, std::string> vol_dirs;
  for (const auto& v : pod.at_path({"spec", "volumes"}).as_array()) {
    const std::string vname = v["name"].as_string();
    std::string dir;
    if (v["persistentVolumeClaim"].is_object()) {
      dir = cfg_.root_dir + "/pv/" + rt.ns + "/" + v.at_path({"persistentVolumeClaim", "claimName"}).as_string();
    } else if (v["hostPath"].is_object()) {
      dir = v.at_path({"hostPath", "path"}).as_string();
    } else {
      dir = rt.dir + "/volumes/" + vname;
    }
    make_dirs(dir);
    if (v["configMap"].is_object() || v["secret"].is_object()) {
      const bool secret = v["secret"].is_object();
      Json src;
      const std::string sname = secret ? v.at_path({"secret", "secretName"}).as_string() : v.at_path({"configMap", "name"}).as_string();
      if (!c_->get("v1", secret ? "Secret" : "ConfigMap", rt.ns, sname, src)) {
        for (const auto& m : src["data"].as_object())
          write_file(dir + "/" + m.first, secret ? base64_decode(m.second.as_string()) : m.second.as_string());
        if (secret)
          for (const auto& m : src["stringData"].as_object()) write_file(dir + "/" + m.first, m.second.as_string());
      }
    }
    vol_dirs[vname] = dir;
  }
  return vol_dirs;
}

// container runtimes in spec order, with their volume mounts; mount points materialised in the
// pod rootfs as symlinks
void Kubelet::build_containers(PodRuntime& rt, const Json& pod, const std::map<std::string, std::string>& vol_dirs) {
  auto build = [&](const Json& list, bool init, std::vector<ContainerRt>& out) {
    for (const auto& c : list.as_array()) {
      ContainerRt cr;
      cr.name = c["name"].as_string();
      cr.init = init;
      cr.sidecar = init && c["restartPolicy"].as_string() == "Always";
      cr.log_path = rt.dir + "/" + cr.name + ".log";
      cr.term_path = rt.dir + "/" + cr.name + ".termination-log";
      for (const auto& vm : c["volumeMounts"].as_array()) {
        auto it = vol_dirs.find(vm["name"].as_string());
        if (it == vol_dirs.end()) continue;
        std::string host = it->second;
        if (!vm["subPath"].as_string().empty()) {
          host += "/" + vm["subPath"].as_string();
          if (!file_exists(host)) make_dirs(host);
        }
        rt.mounts[vm["mountPath"].as_string()] = host;
      }
      out.push_back(cr);
    }
  };
  build(pod.at_path({"spec", "initContainers"}), true, rt.init);
  build(pod.at_path({"spec", "containers"}), false, rt.main);
  for (const auto& m : rt.mounts) {
    std::string link = rt.dir + "/rootfs" + m.first;
    size_t slash = link.rfind('/');
    make_dirs(link.substr(0, slash));
    ::unlink(link.c_str());
    if (::symlink(m.second.c_str(), link.c_str()) != 0) make_dirs(link);
  }
}

// Istio's injection rule: the namespace carries istio-injection=enabled and the pod does not opt out
// (profile_controller.go:71 labels every profile namespace); only with a policy enforcer on the node
bool Kubelet::wants_sidecar(const Json& pod) {
  if (!inbound_) return false;
  if (annotation(pod, "sidecar.istio.io/inject") == "false") return false;
  Json ns;
  if (c_->get("v1", "Namespace", "", pod.str_at({"metadata", "namespace"}), ns)) return false;
  return label(ns, "istio-injection") == "enabled";
}

// an ingress NetworkPolicy of the pod's namespace selects it (its traffic must pass an enforcement
// point even without a mesh sidecar: ODH's <nb>-ctrl-np / <nb>-oauth-np)
bool Kubelet::selected_by_netpol(const Json& pod) {
  Json nps;
  if (c_->list("networking.k8s.io/v1", "NetworkPolicy", pod.str_at({"metadata", "namespace"}), ListOptions(), nps)) return false;
  NetpolSource none;
  std::map<std::string, std::string> labels;
  for (const auto& kv : pod.at_path({"metadata", "labels"}).as_object()) labels[kv.first] = kv.second.as_string();
  std::vector<Json> items(nps["items"].as_array().begin(), nps["items"].as_array().end());
  return evaluate_netpol(items, pod.str_at({"metadata", "namespace"}), labels, 0, "", "TCP", none).isolated;
}

// the pod's inbound listeners: pod_ip:port (host namespace) for every TCP containerPort, each
// request through the enforcer (NetworkPolicy; Istio AuthorizationPolicy when `mesh`), then to the
// app: app_ip:port on the host, or inside the pod's network namespace
void Kubelet::start_inbound(PodRuntime& rt, const Json& pod, bool mesh) {
  InboundTarget base;
  base.ns = rt.ns;
  base.name = rt.name;
  base.app_ip = rt.app_ip;
  base.pod_ip = rt.ip;
  base.mesh = mesh;
  base.netns = rt.netns;
  for (const auto& kv : pod.at_path({"metadata", "labels"}).as_object()) base.labels[kv.first] = kv.second.as_string();
  std::map<int, std::string> ports;  // port -> name
  for (const char* list : {"containers", "initContainers"})
    for (const auto& c : pod.at_path({"spec", list}).as_array())
      for (const auto& p : c["ports"].as_array())
        if (p["protocol"].as_string_or("TCP") == "TCP" && p["containerPort"].as_int() > 0)
          ports.emplace(static_cast<int>(p["containerPort"].as_int()), p["name"].as_string());
  for (const auto& port : ports) {
    InboundTarget t = base;
    t.port = port.first;
    t.port_name = port.second;
    auto srv = std::make_unique<HttpServer>();
    InboundHandler h = inbound_;
    srv->set_handler([h, t](HttpRequest& req, HttpResponse& resp) { h(t, req, resp); });
    std::string err;
    if (!srv->listen(rt.ip, port.first, &err)) {
      rec_->event(pod, "Warning", "FailedInbound", "inbound listener " + rt.ip + ":" + std::to_string(port.first) + ": " + err);
      continue;
    }
    srv->start();
    rt.inbound.push_back(std::move(srv));
  }
}

// the pod's network: its own namespace with inbound listeners and egress relays (--pod-netns), else
// the host namespace, with the private-address convention when an enforcement point is needed
bool Kubelet::setup_pod_network(PodRuntime& rt, const Json& pod) {
  const bool mesh = wants_sidecar(pod);
  if (netns_) {
    std::string err;
    rt.netns = PodNetns::create(&err);
    if (!rt.netns) {
      rt.gpu_ok = false;  // fails admission: a pod is never started outside its isolation
      rt.gpu_error = "FailedCreatePodSandBox: network namespace: " + err;
      rec_->event(pod, "Warning", "FailedCreatePodSandBox", "network namespace: " + err);
      return false;
    }
    PodSource src;
    src.ns = rt.ns;
    src.name = rt.name;
    for (const auto& kv : pod.at_path({"metadata", "labels"}).as_object()) src.labels[kv.first] = kv.second.as_string();
    const auto eps = cfg_.egress_endpoints ? cfg_.egress_endpoints() : std::vector<std::string>{};
    for (const auto& f : relay_->add_pod(rt.uid, *rt.netns, eps, src))
      rec_->event(pod, "Warning", "FailedEgress", "egress relay for " + f + " could not be bound in the pod's namespace");
    start_inbound(rt, pod, mesh);
    return true;
  }
  if (cfg_.pod_netns == "on") {
    rt.gpu_ok = false;
    rt.gpu_error = "FailedCreatePodSandBox: --pod-netns=on and this node cannot isolate pods";
    return false;
  }
  if (inbound_ && (mesh || selected_by_netpol(pod))) {
    rt.app_ip = cfg_.app_ip_prefix + rt.ip.substr(cfg_.pod_ip_prefix.size());
    start_inbound(rt, pod, mesh);
  }
  return true;
}

// admission of a new pod: sandbox dir, pod IP, network, GPUs, volumes, containers; registered on the node
std::shared_ptr<Kubelet::PodRuntime> Kubelet::admit(const Request& r, const Json& pod) {
  auto rt = std::make_shared<PodRuntime>();
  rt->uid = pod.str_at({"metadata", "uid"});
  rt->ns = r.ns;
  rt->name = r.name;
  rt->dir = cfg_.root_dir + "/pods/" + r.ns + "_" + r.name + "_" + rt->uid.substr(0, 8);
  make_dirs(rt->dir + "/rootfs");
  {
    std::lock_guard<std::mutex> g(mu_);
    uint32_t n;
    do {  // (x.y.z.0 and .255 skipped; the range wraps)
      n = next_ip_++;
      if (next_ip_ >= 0xFFFF) next_ip_ = 2;
    } while ((n & 0xFF) == 0 || (n & 0xFF) == 0xFF);
    rt->ip = cfg_.pod_ip_prefix + "." + std::to_string((n >> 8) & 0xFF) + "." + std::to_string(n & 0xFF);
    rt->app_ip = rt->ip;
  }
  rt->start_time = ms_now();
  if (setup_pod_network(*rt, pod)) {
    allocate_gpus(*rt, pod);
    build_containers(*rt, pod, prepare_volumes(*rt, pod));
  }
  std::lock_guard<std::mutex> g(mu_);
  pods_[rt->uid] = rt;
  key_to_uid_[r.ns + "/" + r.name] = rt->uid;
  return rt;
}

// UnexpectedAdmissionError: the device plugin could not satisfy the request
void Kubelet::fail_admission(const Request& r, const std::string& why) {
  c_->update_with_retry(
      "v1", "Pod", r.ns, r.name,
      [&](Json& o) {
        if (o.at_path({"status", "phase"}).as_string() == "Failed") return false;
        o["status"]["phase"] = "Failed";
        o["status"]["reason"] = "UnexpectedAdmissionError";
        o["status"]["message"] = why.empty() ? "Allocate failed due to requested number of devices unavailable for amd.com/gpu" : why;
        return true;
      },
      true);
}

// the environment of container c (host basics, downward API, GPU wiring, envFrom, env)
void Kubelet::container_env(const PodSync& s, const Json& c, std::vector<std::string>& envv,
                            std::map<std::string, std::string>& envm) {
  const PodRuntime& rt = *s.rt;
  const Request& r = s.r;
  auto set = [&](const std::string& k, const std::string& v) { envm[k] = v; };
  for (char** e = environ; *e; ++e) {
    std::string kv = *e;
    size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    std::string k = kv.substr(0, eq);
    // pass through the host runtime basics only (containers do not inherit the kubelet env)
    if (k == "PATH" || k == "LANG" || k == "LD_LIBRARY_PATH" || k == "TMPDIR" || starts_with(k, "HSA_") ||
        starts_with(k, "KFAMD_") || starts_with(k, "ROCM") || k == "OMP_NUM_THREADS" || k == "PYTHONUNBUFFERED")
      set(k, kv.substr(eq + 1));
  }
  const std::string rootfs = rt.dir + "/rootfs";
  std::string home = rootfs + "/home/jovyan";
  auto hm = rt.mounts.find("/home/jovyan");
  if (hm != rt.mounts.end()) home = hm->second;
  make_dirs(home);
  set("HOME", home);
  set("HOSTNAME", r.name);
  set("POD_NAME", r.name);
  set("POD_NAMESPACE", r.ns);
  set("POD_IP", rt.ip);
  // a mesh-injected pod's apps listen on its private address, behind the inbound listeners
  if (rt.app_ip != rt.ip) set("KFAMD_BIND_IP", rt.app_ip);
  set("KFAMD_POD_DIR", rt.dir);
  if (!warm_dir_.empty()) set("KFAMD_WARM_READINESS_DIR", warm_dir_);  // the gpu-readiness sidecar's warm ops
  set("KFAMD_ROOTFS", rootfs);
  set("KFAMD_TERMINATION_LOG", rt.dir + "/" + c["name"].as_string() + ".termination-log");
  Json mounts = Json::object();
  for (const auto& m : rt.mounts) mounts[m.first] = m.second;
  set("KFAMD_VOLUME_MOUNTS", mounts.dump());
  set("PYTHONPATH", cfg_.repo_root);
  set("PYTHONUNBUFFERED", "1");
  {
    std::vector<std::string> ports;
    for (const auto& p : c["ports"].as_array()) ports.push_back(std::to_string(p["containerPort"].as_int()));
    set("KFAMD_CONTAINER_PORTS", join(ports, ","));
    set("KFAMD_CONTAINER_NAME", c["name"].as_string());
  }
  Url u;
  if (Url::parse(cfg_.api_url, u)) {
    set("KUBERNETES_SERVICE_HOST", u.host);
    set("KUBERNETES_SERVICE_PORT", std::to_string(u.port));
    set("KFAMD_API_URL", cfg_.api_url);
  }
  // GPU wiring from the device plugin allocation (and for a container that shares the pod's GPUs
  // without a second allocation: the gpu-readiness sidecar)
  if (wants_pod_gpus(c) && !rt.gpus.devices.empty()) {
    const Json genv = gpu_env_for(rt.gpus, alloc_->topology(), rt.gpus.devices.size() > 1, rt.ip, rt.rdzv_port);
    for (const auto& ev : genv.as_array()) set(ev["name"].as_string(), ev["value"].as_string());
    const auto local = alloc_->topology().local_cpus(rt.gpus.devices);
    if (cfg_.numa_pinning && !local.empty()) set("KFAMD_CPU_AFFINITY", format_cpulist(local));
    // Node-level code-object cache shared by every GPU container (the device plugin's Allocate
    // response carries this env + mount). comgr caches the runtime's device-code builds under
    // $HOME/.cache/comgr by default, and every pod starts with an empty HOME: that miss cost
    // ~140 ms of each cold start on MI355X (profiles/r1_coldstart2/README.md).
    // Keyed per namespace: profiles are tenants, and a cache one tenant can write must never
    // feed code objects to another tenant's pods (a namespace's own pods share its warm cache).
    const std::string cache = cfg_.root_dir + "/gpu-cache/comgr/" + r.ns;
    if (::access(cache.c_str(), F_OK) != 0) {
      make_dirs(cache);
      link_comgr_seed(cache);
    }
    set("AMD_COMGR_CACHE_DIR", cache);
  }
  for (const auto& ef : c["envFrom"].as_array()) {
    const bool secret = ef["secretRef"].is_object();
    const std::string name = secret ? ef.at_path({"secretRef", "name"}).as_string() : ef.at_path({"configMapRef", "name"}).as_string();
    Json src;
    if (c_->get("v1", secret ? "Secret" : "ConfigMap", r.ns, name, src)) continue;
    for (const auto& m : src["data"].as_object())
      set(ef["prefix"].as_string() + m.first, secret ? base64_decode(m.second.as_string()) : m.second.as_string());
  }
  for (const auto& ev : c["env"].as_array()) {
    const std::string name = ev["name"].as_string();
    if (ev.has("value")) {
      set(name, expand_vars(ev["value"].as_string(), envm));
      continue;
    }
    const Json& vf = ev["valueFrom"];
    if (vf["fieldRef"].is_object()) {
      const std::string path = vf.at_path({"fieldRef", "fieldPath"}).as_string();
      if (path == "metadata.name") set(name, r.name);
      else if (path == "metadata.namespace") set(name, r.ns);
      else if (path == "status.podIP") set(name, rt.ip);
      else if (path == "spec.nodeName") set(name, cfg_.node_name);
      else if (path == "metadata.uid") set(name, s.uid);
      else if (starts_with(path, "metadata.annotations['")) set(name, annotation(s.pod, path.substr(22, path.size() - 24)));
      else if (starts_with(path, "metadata.labels['")) set(name, label(s.pod, path.substr(17, path.size() - 19)));
    } else if (vf["configMapKeyRef"].is_object() || vf["secretKeyRef"].is_object()) {
      const bool secret = vf["secretKeyRef"].is_object();
      const Json& ref = secret ? vf["secretKeyRef"] : vf["configMapKeyRef"];
      Json src;
      if (!c_->get("v1", secret ? "Secret" : "ConfigMap", r.ns, ref["name"].as_string(), src)) {
        const Json& v = src["data"][ref["key"].as_string()];
        if (v.is_string()) set(name, secret ? base64_decode(v.as_string()) : v.as_string());
      }
    } else if (vf["resourceFieldRef"].is_object()) {
      const std::string res = vf.at_path({"resourceFieldRef", "resource"}).as_string();
      auto parts = split(res, '.');
      if (parts.size() == 2) set(name, c.at_path({"resources", parts[0].c_str(), parts[1].c_str()}).as_string());
    }
  }
  envv.clear();
  for (auto& kv : envm) envv.push_back(kv.first + "=" + kv.second);
}

// a container's process: forked from the recipe's zygote when one serves it, else a fresh exec
void Kubelet::start_container(PodSync& s, ContainerRt& cr) {
  PodRuntime& rt = *s.rt;
  const Json& c = s.container_spec(cr);
  std::vector<std::string> envv;
  std::map<std::string, std::string> envm;
  container_env(s, c, envv, envm);
  std::string why, zygote;
  std::vector<std::string> argv = resolve_argv(c, &why, &zygote);
  for (auto& a : argv) a = expand_vars(a, envm);
  std::string wd = c["workingDir"].as_string();
  std::string cwd = rt.dir + "/rootfs";
  if (!wd.empty()) {
    auto m = rt.mounts.find(wd);
    cwd = m != rt.mounts.end() ? m->second : rt.dir + "/rootfs" + wd;
    make_dirs(cwd);
    // follow a symlinked mount point
    char buf[4096];
    if (!realpath(cwd.c_str(), buf)) make_dirs(cwd);
  }
  ::unlink(cr.term_path.c_str());
  std::string serr;
  {
    std::ofstream lf(cr.log_path, std::ios::app);
    lf << "# kflite: starting " << cr.name << " (" << why << "): " << join(argv, " ") << "\n";
  }
  // topology-manager "single-numa-node"-style placement for GPU containers: the process tree runs
  // on the CPUs local to its GPUs (host<->HBM copies, RCCL proxy threads, data loaders)
  std::vector<int> cpus;
  if (cfg_.numa_pinning && !rt.gpus.devices.empty() && wants_pod_gpus(c)) cpus = alloc_->topology().local_cpus(rt.gpus.devices);
  pid_t pid = -1;
  cr.zfd = -1;
  cr.zorphan = false;
  // a recipe with a zygote forks from the pre-imported interpreter when one serves it ('python -m'
  // containers only); otherwise, or when it does not answer, a fresh interpreter as always
  Zygote zy;
  bool warm = false;  // the process is a zygote's warm GPU child
  if (!zygote.empty()) {
    std::lock_guard<std::mutex> g(zy_mu_);
    auto it = zygotes_.find(zygote);
    if (it != zygotes_.end()) zy = it->second;
  }
  if (zy.pid > 0 && argv.size() >= 3 && argv[0] == cfg_.python && argv[1] == "-m") {
    std::string zerr;
    // a 1-GPU container may take the zygote's warm child of its device (GPU already initialised)
    const int warm_dev = rt.gpus.devices.size() == 1 && wants_pod_gpus(c) ? rt.gpus.devices[0] : -1;
    pid = zygote_spawn(zy.sock, argv, envv, cwd, cr.log_path, cpus, &cr.zfd, &zerr, rt.netns ? rt.netns->path() : "",
                       warm_dev, &warm);
    if (pid > 0) {
      std::ofstream lf(cr.log_path, std::ios::app);
      lf << "# kflite: " << (warm ? "warm child of zygote " : "forked from zygote ") << zy.pid << " (preloaded " << zygote
         << (warm ? ", GPU " + std::to_string(warm_dev) + " initialised" : std::string()) << ")\n";
    } else if (!zerr.empty()) {
      std::ofstream lf(cr.log_path, std::ios::app);
      lf << "# kflite: " << zerr << "; starting a fresh interpreter\n";
    }
  }
  static const auto starts = Registry::global().counter(
      "kubelet_container_starts_total", "container processes started, by how: zygote fork or fresh exec", {"mode"});
  if (pid > 0) starts->inc({warm ? "zygote-warm" : "zygote"});
  if (pid < 0) {
    pid = spawn(argv, envv, cwd, cr.log_path, &serr, cpus, rt.netns.get());
    if (pid > 0) starts->inc({"fresh"});
  }
  if (pid < 0) {
    cr.state = "waiting";
    cr.reason = "CreateContainerError";
    cr.message = serr;
    rec_->event(s.pod, "Warning", "Failed", "Error: " + serr);
    cr.backoff_until = now_seconds() + cfg_.restart_backoff;
    return;
  }
  cr.pid = pid;
  cr.state = "running";
  cr.reason = "";
  cr.envv = envv;
  cr.cwd = cwd;
  cr.cpus = cpus;
  cr.started_at = ms_now();
  if (cr.zfd >= 0) {
    const int dfd = ::fcntl(cr.zfd, F_DUPFD_CLOEXEC, 0);  // the watch closes its own copy
    if (dfd >= 0) watch_fd(dfd, s.r.ns, s.r.name);
  } else {
    watch_exit(pid, s.r.ns, s.r.name);
  }
  cr.run_started = now_seconds();
  cr.probe_gen = Prober::next_generation();
  cr.ready = false;
  cr.ready_ok = cr.ready_fail = cr.live_fail = cr.startup_ok = cr.startup_fail = 0;
  const Json& sp = c["startupProbe"];
  cr.started_probe_ok = !sp.is_object();
  cr.next_startup_probe = now_seconds() + static_cast<double>(probe_i(sp, "initialDelaySeconds", 0));
  cr.next_ready_probe = now_seconds() + static_cast<double>(probe_i(c["readinessProbe"], "initialDelaySeconds", 0));
  cr.next_live_probe = now_seconds() + static_cast<double>(probe_i(c["livenessProbe"], "initialDelaySeconds", 0));
  rec_->event(s.pod, "Normal", "Started", "Started container " + cr.name);
}

// The probe as a self-contained closure (copies of the spec, the pod IP and the container env): it
// runs on a Prober thread, never on a reconcile worker.
std::function<bool()> Kubelet::make_probe(const PodSync& s, const Json& probe, const Json& c) {
  const PodRuntime& rt = *s.rt;
  const int timeout = static_cast<int>(probe_i(probe, "timeoutSeconds", 1)) * 1000;
  auto port_of = [&](const Json& p) -> int {
    if (p.is_number()) return static_cast<int>(p.as_int());
    for (const auto& cp : c["ports"].as_array())
      if (cp["name"].as_string() == p.as_string()) return static_cast<int>(cp["containerPort"].as_int());
    return std::atoi(p.as_string().c_str());
  };
  if (probe["httpGet"].is_object()) {
    const Json& hg = probe["httpGet"];
    // probes go to the app itself (the inbound listener exempts the kubelet as Istio's probe
    // rewrite does)
    const std::string host = hg["host"].as_string_or(rt.app_ip);
    std::string url = "http://" + host + ":" + std::to_string(port_of(hg["port"])) + hg["path"].as_string_or("/");
    Headers h;
    for (const auto& hh : hg["httpHeaders"].as_array()) h[hh["name"].as_string()] = hh["value"].as_string();
    std::shared_ptr<const PodNetns> ns = rt.netns;  // probes connect inside the pod's namespace
    return [url, h, timeout, ns] {
      NetnsScope in(ns.get());
      HttpResult res = in.ok() ? http_request("GET", url, "", h, timeout) : HttpResult{};
      return res.status >= 200 && res.status < 400;
    };
  }
  if (probe["tcpSocket"].is_object()) {
    const std::string ip = rt.app_ip;
    const int port = port_of(probe.at_path({"tcpSocket", "port"}));
    std::shared_ptr<const PodNetns> ns = rt.netns;
    return [ip, port, timeout, ns] {
      NetnsScope in(ns.get());
      return in.ok() && tcp_connect(ip, port, timeout);
    };
  }
  if (probe["exec"].is_object()) {
    std::vector<std::string> argv;
    for (const auto& a : probe.at_path({"exec", "command"}).as_array()) argv.push_back(a.as_string());
    if (argv.empty()) return [] { return false; };
    std::vector<std::string> envv;
    std::map<std::string, std::string> envm;
    container_env(s, c, envv, envm);
    const std::string cwd = rt.dir + "/rootfs", log = rt.dir + "/probe.log";
    std::shared_ptr<const PodNetns> ns = rt.netns;
    return [argv, envv, cwd, log, timeout, ns] {
      pid_t pid = spawn(argv, envv, cwd, log, nullptr, {}, ns.get());
      if (pid < 0) return false;
      return wait_probe_process(pid, timeout) == 0;
    };
  }
  return [] { return true; };
}

// The verdict of this container's last `kind` probe, if one finished; starts one when `due`.
std::optional<bool> Kubelet::probe_verdict(PodSync& s, ContainerRt& cr, const char* kind, const Json& probe,
                                           const Json& c, bool due) {
  const std::string key = s.rt->uid + "/" + (cr.init ? "init:" : "") + cr.name + "/" + kind;
  const bool start = due && !prober_->in_flight(key);
  return prober_->poll(key, cr.probe_gen, start, s.r.ns, s.r.name, start ? make_probe(s, probe, c) : nullptr);
}

// Probes of one running container (startup gates readiness/liveness); lowers s.next_wake.
void Kubelet::tick_probes(PodSync& s, ContainerRt& cr, const Json& c) {
  const double now = now_seconds();
  const Json& sp = c["startupProbe"];
  if (!cr.started_probe_ok) {
    if (auto v = probe_verdict(s, cr, "startup", sp, c, now >= cr.next_startup_probe)) {
      if (*v) {
        if (++cr.startup_ok >= probe_i(sp, "successThreshold", 1)) cr.started_probe_ok = true;
      } else if (++cr.startup_fail >= probe_i(sp, "failureThreshold", 3)) {
        rec_->event(s.pod, "Warning", "Unhealthy", "Startup probe failed");
        ::kill(-cr.pid, SIGKILL);
      }
      cr.next_startup_probe = now + static_cast<double>(probe_i(sp, "periodSeconds", 10));
    }
  }
  if (!cr.started_probe_ok) {
    s.next_wake = std::min(s.next_wake, 0.1);
    return;
  }
  const Json& rp = c["readinessProbe"];
  if (!rp.is_object()) {
    cr.ready = true;
  } else if (auto v = probe_verdict(s, cr, "readiness", rp, c, now >= cr.next_ready_probe)) {
    if (*v) {
      cr.ready_fail = 0;
      if (++cr.ready_ok >= probe_i(rp, "successThreshold", 1)) cr.ready = true;
    } else {
      cr.ready_ok = 0;
      if (++cr.ready_fail >= probe_i(rp, "failureThreshold", 3)) {
        if (cr.ready) rec_->event(s.pod, "Warning", "Unhealthy", "Readiness probe failed");
        cr.ready = false;
      }
    }
    // probe fast until the first success (cold-start latency: the readiness sidecar's verdict or the
    // server's first answer is seen within ~5 ms), then at periodSeconds
    cr.next_ready_probe = now + (cr.ready ? static_cast<double>(probe_i(rp, "periodSeconds", 10)) : kStartupPoll);
  }
  const Json& lp = c["livenessProbe"];
  if (lp.is_object()) {
    if (auto v = probe_verdict(s, cr, "liveness", lp, c, now >= cr.next_live_probe)) {
      if (*v) {
        cr.live_fail = 0;
      } else if (++cr.live_fail >= probe_i(lp, "failureThreshold", 3)) {
        rec_->event(s.pod, "Warning", "Unhealthy", "Liveness probe failed; container will be restarted");
        ::kill(-cr.pid, SIGKILL);
      }
      cr.next_live_probe = now + static_cast<double>(probe_i(lp, "periodSeconds", 10));
    }
  }
  if (!cr.ready) {
    s.next_wake = std::min(s.next_wake, kStartupPoll);
  } else {
    // wake for the next due probe; a container without probes only needs the 1 s exit-detection
    // relist (PLEG-like), not a 0.2 s spin on "probe due at t=0"
    double due = 1e30;
    if (rp.is_object()) due = std::min(due, cr.next_ready_probe);
    if (lp.is_object()) due = std::min(due, cr.next_live_probe);
    if (due < 1e30) s.next_wake = std::min(s.next_wake, std::max(0.2, due - now));
  }
}

// a long-running container (main, or started sidecar): exit -> restart per policy with back-off, probes
void Kubelet::tick_long_running(PodSync& s, ContainerRt& cr, bool always_restart) {
  const Json& c = s.container_spec(cr);
  if (cr.state == "running") {
    if (!handle_exit(cr)) {
      tick_probes(s, cr, c);
      return;
    }
  }
  if (cr.state == "terminated") {
    const bool restart = always_restart || s.restart_policy == "Always" ||
                         (s.restart_policy == "OnFailure" && cr.exit_code != 0);
    if (!restart) return;
    cr.last_state = terminated_state(cr);
    cr.restarts++;
    cr.state = "waiting";
    cr.reason = "CrashLoopBackOff";
    double ran = now_seconds() - cr.run_started;
    double backoff = ran > 600 ? cfg_.restart_backoff : std::min(300.0, cfg_.restart_backoff * (1 << std::min(cr.restarts - 1, 5)));
    cr.backoff_until = now_seconds() + backoff;
    rec_->event(s.pod, "Warning", "BackOff", "Back-off restarting failed container " + cr.name);
  }
  if (cr.state == "waiting") {
    if (now_seconds() >= cr.backoff_until) {
      start_container(s, cr);
      // no startup / readiness probe: Ready as soon as it runs (Kubernetes' default Success), in
      // this pass rather than the next re-sync
      if (cr.state == "running" && !c["startupProbe"].is_object() && !c["readinessProbe"].is_object()) {
        cr.started_probe_ok = true;
        cr.ready = true;
      }
      s.next_wake = std::min(s.next_wake, kStartupPoll);
    } else {
      s.next_wake = std::min(s.next_wake, cr.backoff_until - now_seconds());
    }
  }
}

// init containers, sequentially. A native sidecar (restartPolicy: Always) counts as done once it is
// STARTED (running, startup probe passed): the next init container / the main containers start
// while it keeps running, and it is restarted whenever it exits (KEP-753 semantics).
void Kubelet::run_init_containers(PodSync& s) {
  PodRuntime& rt = *s.rt;
  while (rt.init_done < rt.init.size() && !rt.init_failed) {
    ContainerRt& ic = rt.init[rt.init_done];
    if (ic.state == "waiting") {
      if (now_seconds() < ic.backoff_until) {
        s.next_wake = std::min(s.next_wake, ic.backoff_until - now_seconds());
        break;
      }
      start_container(s, ic);
      s.next_wake = kStartupPoll;
      if (ic.sidecar && ic.state == "running" && !s.container_spec(ic)["startupProbe"].is_object()) {
        ic.started_probe_ok = true;
        rt.init_done++;
        continue;
      }
      break;
    }
    if (ic.state == "running") {
      if (handle_exit(ic)) continue;
      if (ic.sidecar) {
        tick_probes(s, ic, s.container_spec(ic));
        if (ic.started_probe_ok) {
          rt.init_done++;
          continue;
        }
      }
      s.next_wake = kStartupPoll;  // init containers gate the pod: notice their exit within ~10 ms
      break;
    }
    // terminated
    if (ic.exit_code == 0 && !ic.sidecar) {
      rt.init_done++;
      continue;
    }
    if (s.restart_policy == "Never" && !ic.sidecar) {
      rt.init_failed = true;
      break;
    }
    ic.last_state = terminated_state(ic);
    ic.restarts++;
    ic.state = "waiting";
    ic.reason = "CrashLoopBackOff";
    ic.backoff_until = now_seconds() + std::min(300.0, cfg_.restart_backoff * (1 << std::min(ic.restarts - 1, 5)));
    rec_->event(s.pod, "Warning", "BackOff", "Back-off restarting failed container " + ic.name);
    break;
  }
}

// the gpu-readiness sidecar's report (its termination-log file, written before it turns Ready) goes
// onto the pod as notebooks.kubeflow.org/gpu-readiness, where the notebook controller surfaces it as
// status.gpuReadiness; written before the status update that makes the pod Ready
void Kubelet::publish_readiness(PodSync& s) {
  PodRuntime& rt = *s.rt;
  for (const auto& cr : rt.init) {
    if (!cr.sidecar || cr.name != "gpu-readiness" || !cr.ready || rt.readiness_published) continue;
    std::string rep;
    if (!read_file(cr.term_path, rep) || rep.empty()) continue;
    rt.readiness_published = true;
    c_->update_with_retry("v1", "Pod", s.r.ns, s.r.name, [&](Json& o) {
      if (o.str_at({"metadata", "uid"}) != s.uid) return false;
      o["metadata"]["annotations"][ANNOTATION_GPU_READINESS] = rep.substr(0, 4096);
      o["metadata"]["annotations"]["notebooks.kubeflow.org/gpu-readiness-at"] = ms_now();
      return true;
    });
  }
}

// phase, conditions and container statuses; written only when they changed
ApiError Kubelet::write_status(PodSync& s) {
  const PodRuntime& rt = *s.rt;
  const bool initialized = rt.init_done == rt.init.size();
  Json init_st = Json::array(), main_st = Json::array();
  for (const auto& cr : rt.init) init_st.push_back(container_status(cr, s.container_spec(cr)));
  for (const auto& cr : rt.main) main_st.push_back(container_status(cr, s.container_spec(cr)));
  bool all_ready = initialized && !rt.main.empty(), any_running = false, all_done = initialized, any_failed = rt.init_failed;
  for (const auto& cr : rt.init)
    if (cr.sidecar) all_ready = all_ready && cr.ready;  // sidecar readiness gates the pod's
  for (const auto& cr : rt.main) {
    all_ready = all_ready && cr.ready;
    any_running = any_running || cr.state == "running";
    all_done = all_done && cr.state == "terminated";
    any_failed = any_failed || (cr.state == "terminated" && cr.exit_code != 0);
  }
  std::string new_phase = "Pending";
  if (rt.init_failed) new_phase = "Failed";
  else if (initialized && all_done && s.restart_policy != "Always") new_phase = any_failed ? "Failed" : "Succeeded";
  else if (initialized && (any_running || all_done)) new_phase = "Running";

  if (!s.pod.has("apiVersion")) s.pod["apiVersion"] = "v1";
  if (!s.pod.has("kind")) s.pod["kind"] = "Pod";
  return c_->update_with_retry_from(
      std::move(s.pod),
      [&](Json& o) {
        if (o.str_at({"metadata", "uid"}) != s.uid) return false;
        Json st = o["status"];
        const Json old_st = st;
        st["phase"] = new_phase;
        st["hostIP"] = "127.0.0.1";
        st["podIP"] = rt.ip;
        st["podIPs"] = Json::array({Json{{"ip", rt.ip}}});
        st["startTime"] = rt.start_time;
        st["containerStatuses"] = main_st;
        if (!rt.init.empty()) st["initContainerStatuses"] = init_st;
        auto cond = [&](const char* type, bool ok, const std::string& reason) {
          Json conds = Json::array();
          std::string ts = ms_now();
          for (const auto& c : st["conditions"].as_array()) {
            if (c["type"].as_string() == type) {
              if (c["status"].as_string() == (ok ? "True" : "False")) ts = c["lastTransitionTime"].as_string();
              continue;
            }
            conds.push_back(c);
          }
          Json c{{"type", type}, {"status", ok ? "True" : "False"}, {"lastProbeTime", Json()}, {"lastTransitionTime", ts}};
          if (!ok && !reason.empty()) c["reason"] = reason;
          conds.push_back(c);
          st["conditions"] = conds;
        };
        cond("Initialized", initialized, "ContainersNotInitialized");
        cond("ContainersReady", all_ready, "ContainersNotReady");
        cond("Ready", all_ready, "ContainersNotReady");
        if (st == old_st) return false;
        o["status"] = st;
        return true;
      },
      true);
}

Result Kubelet::reconcile(const Request& r, std::string* err) {
  if (stopping_) return {};
  Json pod;
  ApiError e = c_->get("v1", "Pod", r.ns, r.name, pod);
  std::shared_ptr<PodRuntime> rt = lookup_runtime(r, e, pod);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  if (pod.at_path({"spec", "nodeName"}).as_string() != cfg_.node_name) return {};
  std::unique_lock<std::mutex> pod_lock;
  if (rt) {
    pod_lock = std::unique_lock<std::mutex>(rt->op_mu);
    if (stopping_) return {};
  }
  if (pod.at_path({"metadata", "deletionTimestamp"}).is_string()) {
    finish_deletion(r, pod, rt, err);
    return {};
  }
  const std::string phase = pod.at_path({"status", "phase"}).as_string();
  if (!rt && (phase == "Succeeded" || phase == "Failed")) return {};
  if (!rt) rt = admit(r, pod);
  if (!pod_lock.owns_lock()) {
    pod_lock = std::unique_lock<std::mutex>(rt->op_mu);
    if (stopping_) return {};
  }
  if (!rt->gpu_ok) {
    fail_admission(r, rt->gpu_error);
    return {};
  }
  PodSync s{r, std::move(pod), rt, rt->uid, ""};
  s.restart_policy = s.pod.at_path({"spec", "restartPolicy"}).as_string_or("Always");
  run_init_containers(s);
  // started sidecars run alongside everything after them
  for (size_t i = 0; i < rt->init_done && i < rt->init.size(); ++i)
    if (rt->init[i].sidecar) tick_long_running(s, rt->init[i], true);
  if (rt->init_done == rt->init.size())
    for (auto& cr : rt->main) tick_long_running(s, cr, false);
  publish_readiness(s);
  ApiError ue = write_status(s);
  if (ue && ue.code != 404) *err = ue.message;
  return Result::after(std::max(kStartupPoll, s.next_wake));
}

// GPU metrics (SURVEY §5.5 build additions), scraped from the kubelet's registry: which pod holds
// which MI355X, HBM allocated per namespace (what amd.com/gpu-memory quota charges), and the live
// amdgpu sysfs counters of every discovered GPU (VRAM used/total, busy %).
void Kubelet::register_gpu_metrics() {
  auto& reg = Registry::global();
  reg.add_collector(std::make_shared<CollectorFamily>(
      "kfamd_gpu_allocated", "1 for every MI355X allocated to a pod by the device plugin", "gauge",
      std::vector<std::string>{"gpu", "namespace", "pod"}, [this]() {
        std::vector<std::pair<Labels, double>> out;
        const auto allocs = alloc_->allocations();
        std::lock_guard<std::mutex> g(mu_);
        for (const auto& a : allocs) {
          auto it = pods_.find(a.first);
          const std::string ns = it != pods_.end() ? it->second->ns : "", name = it != pods_.end() ? it->second->name : a.first;
          for (int d : a.second) out.push_back({{std::to_string(d), ns, name}, 1.0});
        }
        return out;
      }));
  reg.add_collector(std::make_shared<CollectorFamily>(
      "kfamd_gpu_hbm_allocated_bytes", "HBM of the MI355X GPUs allocated to pods, per namespace", "gauge",
      std::vector<std::string>{"namespace"}, [this]() {
        std::vector<std::pair<Labels, double>> out;
        const auto allocs = alloc_->allocations();
        const auto& topo = alloc_->topology();
        std::map<std::string, double> per_ns;
        std::lock_guard<std::mutex> g(mu_);
        for (const auto& a : allocs) {
          auto it = pods_.find(a.first);
          const std::string ns = it != pods_.end() ? it->second->ns : "";
          for (int d : a.second)
            if (d >= 0 && d < topo.size()) per_ns[ns] += static_cast<double>(topo.gpus[d].hbm_bytes);
        }
        for (auto& kv : per_ns) out.push_back({{kv.first}, kv.second});
        return out;
      }));
  struct SysfsMetric {
    const char* name;
    const char* help;
    const char* file;
  };
  static const SysfsMetric kSysfs[] = {
      {"kfamd_gpu_vram_used_bytes", "amdgpu mem_info_vram_used", "mem_info_vram_used"},
      {"kfamd_gpu_vram_total_bytes", "amdgpu mem_info_vram_total", "mem_info_vram_total"},
      {"kfamd_gpu_busy_percent", "amdgpu gpu_busy_percent", "gpu_busy_percent"},
  };
  for (const auto& m : kSysfs) {
    const std::string file = m.file;
    reg.add_collector(std::make_shared<CollectorFamily>(
        m.name, m.help, "gauge", std::vector<std::string>{"gpu"}, [this, file]() {
          std::vector<std::pair<Labels, double>> out;
          for (const auto& g : alloc_->topology().gpus) {
            if (g.drm_render_minor < 0) continue;
            std::string v;
            if (read_file("/sys/class/drm/renderD" + std::to_string(g.drm_render_minor) + "/device/" + file, v))
              out.push_back({{std::to_string(g.index)}, std::atof(v.c_str())});
          }
          return out;
        }));
  }
  register_telemetry_metrics();
  metrics_registered_ = true;
}

namespace {

// one discovered GPU's latest sample: device index, telemetry, the sample before (throttle residency
// is a delta), and the pod holding it
struct TelemetryRow {
  int gpu;
  GpuTelemetry t;
  bool has_prev;
  GpuTelemetry prev;
  std::string ns, pod;
};
using TelemetryRows = std::function<std::vector<TelemetryRow>()>;

// the metric families over one (cached) telemetry source
void add_telemetry_families(const TelemetryRows& rows) {
  auto& reg = Registry::global();
  using Field = double (*)(const GpuTelemetry&);
  struct PerPod {
    const char* name;
    const char* help;
    Field f;
  };
  static const PerPod kPerPod[] = {
      {"kfamd_gpu_gfx_activity_percent", "GFX engine activity (SMU average), labelled with the holding pod",
       [](const GpuTelemetry& t) { return t.gfx_activity; }},
      {"kfamd_gpu_hbm_activity_percent", "HBM memory-controller (UMC) activity, labelled with the holding pod",
       [](const GpuTelemetry& t) { return t.umc_activity; }},
  };
  for (const auto& m : kPerPod) {
    const Field f = m.f;
    reg.add_collector(std::make_shared<CollectorFamily>(
        m.name, m.help, "gauge", std::vector<std::string>{"gpu", "namespace", "pod"}, [rows, f]() {
          std::vector<std::pair<Labels, double>> out;
          for (const auto& r : rows()) {
            const double v = f(r.t);
            if (v >= 0) out.push_back({{std::to_string(r.gpu), r.ns, r.pod}, v});
          }
          return out;
        }));
  }
  struct PerGpu {
    const char* name;
    const char* help;
    const char* type;
    Field f;
  };
  static const PerGpu kPerGpu[] = {
      {"kfamd_gpu_power_watts", "socket power", "gauge", [](const GpuTelemetry& t) { return t.power_w; }},
      {"kfamd_gpu_gfxclk_mhz", "current GFX clock: the clock the GPU holds under load", "gauge",
       [](const GpuTelemetry& t) { return t.gfxclk_mhz; }},
      {"kfamd_gpu_energy_joules_total", "energy accumulated since driver load", "counter",
       [](const GpuTelemetry& t) { return t.energy_j; }},
  };
  for (const auto& m : kPerGpu) {
    const Field f = m.f;
    reg.add_collector(std::make_shared<CollectorFamily>(
        m.name, m.help, m.type, std::vector<std::string>{"gpu"}, [rows, f]() {
          std::vector<std::pair<Labels, double>> out;
          for (const auto& r : rows()) {
            const double v = f(r.t);
            if (v >= 0) out.push_back({{std::to_string(r.gpu)}, v});
          }
          return out;
        }));
  }
  reg.add_collector(std::make_shared<CollectorFamily>(
      "kfamd_gpu_temperature_celsius", "hotspot and HBM temperature", "gauge", std::vector<std::string>{"gpu", "sensor"},
      [rows]() {
        std::vector<std::pair<Labels, double>> out;
        for (const auto& r : rows()) {
          if (r.t.temp_hotspot_c >= 0) out.push_back({{std::to_string(r.gpu), "hotspot"}, r.t.temp_hotspot_c});
          if (r.t.temp_mem_c >= 0) out.push_back({{std::to_string(r.gpu), "hbm"}, r.t.temp_mem_c});
        }
        return out;
      }));
  for (int dir = 0; dir < 2; ++dir) {
    reg.add_collector(std::make_shared<CollectorFamily>(
        dir == 0 ? "kfamd_gpu_xgmi_read_bytes_total" : "kfamd_gpu_xgmi_write_bytes_total",
        dir == 0 ? "bytes read over each xGMI link since driver load" : "bytes written over each xGMI link since driver load",
        "counter", std::vector<std::string>{"gpu", "link"}, [rows, dir]() {
          std::vector<std::pair<Labels, double>> out;
          for (const auto& r : rows())
            for (int l = 0; l < r.t.xgmi_links; ++l)
              out.push_back({{std::to_string(r.gpu), std::to_string(l)},
                             dir == 0 ? r.t.xgmi_read_bytes[l] : r.t.xgmi_write_bytes[l]});
          return out;
        }));
  }
  reg.add_collector(std::make_shared<CollectorFamily>(
      "kfamd_gpu_throttle_residency_ratio",
      "share of the last sampling interval spent power-limited (PVIOL) or thermally limited (TVIOL)", "gauge",
      std::vector<std::string>{"gpu", "cause"}, [rows]() {
        std::vector<std::pair<Labels, double>> out;
        for (const auto& r : rows()) {
          // counters restart with the driver: only a forward step of every accumulator is a sample
          if (!r.has_prev || r.t.accumulation_counter <= r.prev.accumulation_counter ||
              r.t.ppt_residency_acc < r.prev.ppt_residency_acc ||
              r.t.thermal_residency_acc < r.prev.thermal_residency_acc)
            continue;
          const double dt = static_cast<double>(r.t.accumulation_counter - r.prev.accumulation_counter);
          out.push_back({{std::to_string(r.gpu), "power"},
                         static_cast<double>(r.t.ppt_residency_acc - r.prev.ppt_residency_acc) / dt});
          out.push_back({{std::to_string(r.gpu), "thermal"},
                         static_cast<double>(r.t.thermal_residency_acc - r.prev.thermal_residency_acc) / dt});
        }
        return out;
      }));
}

}  // namespace

// Live SMU telemetry per MI355X (AMD SMI gpu_metrics, gpu/smi.h), labelled with the pod that holds
// the device: what a notebook's GPUs are doing (GFX / HBM-controller activity), the clock they
// hold under load (MFMA-dense kernels are clock-limited on this part), power, temperatures,
// energy, xGMI traffic per link (RCCL rings over xGMI) and power/thermal throttle residency. One
// AMD SMI sample serves every family of a scrape (cached 1 s).
void Kubelet::register_telemetry_metrics() {
  struct Cache {
    std::mutex mu;
    double at = -1e9;
    std::vector<GpuTelemetry> last, prev;  // prev: the sample before, for throttle-residency deltas
  };
  auto cache = std::make_shared<Cache>();
  auto rows = [this, cache]() {
    std::vector<TelemetryRow> out;
    std::vector<GpuTelemetry> cur, prev;
    {
      std::lock_guard<std::mutex> g(cache->mu);
      const double t = now_seconds();
      if (t - cache->at > 1.0) {
        auto s = AmdSmi::instance().sample();
        if (!s.empty()) {
          cache->prev = std::move(cache->last);
          cache->last = std::move(s);
        }
        cache->at = t;
      }
      cur = cache->last;
      prev = cache->prev;
    }
    if (cur.empty()) return out;
    std::map<int, std::pair<std::string, std::string>> owner;
    const auto allocs = alloc_->allocations();
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& a : allocs) {
        auto it = pods_.find(a.first);
        for (int d : a.second)
          owner[d] = it != pods_.end() ? std::make_pair(it->second->ns, it->second->name) : std::make_pair(std::string(), a.first);
      }
    }
    for (const auto& gdev : alloc_->topology().gpus) {
      for (const auto& t : cur) {
        if (t.bdf != gdev.pci_bus) continue;
        TelemetryRow r{gdev.index, t, false, {}, "", ""};
        for (const auto& p : prev)
          if (p.bdf == t.bdf) {
            r.has_prev = true;
            r.prev = p;
          }
        auto o = owner.find(gdev.index);
        if (o != owner.end()) {
          r.ns = o->second.first;
          r.pod = o->second.second;
        }
        out.push_back(r);
        break;
      }
    }
    return out;
  };
  add_telemetry_families(rows);
}

void Kubelet::setup(Manager& mgr) {
  register_gpu_metrics();
  ctl_ = std::make_shared<Controller>("kubelet", [this](const Request& r, std::string* e) { return reconcile(r, e); }, 4);
  const std::string node = cfg_.node_name;
  ctl_->For(mgr.informer("v1", "Pod"), [node](const std::string& type, const Json& p, const Json* old) {
    if (type == "DELETED") return true;
    const std::string& n = p.at_path({"spec", "nodeName"}).as_string();
    if (n != node) return false;
    // status-only writes of our own do not need a new pass (the periodic requeue drives probes)
    if (type == "MODIFIED" && old && p["spec"] == (*old)["spec"] && p["metadata"]["deletionTimestamp"] == (*old)["metadata"]["deletionTimestamp"])
      return false;
    return true;
  });
  mgr.add(ctl_);
}

}  // namespace kf
