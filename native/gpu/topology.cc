// topology.cc — see topology.h.
#include "gpu/topology.h"

#include <dirent.h>

#include <algorithm>
#include <cstdlib>
#include <functional>
#include <sstream>

#include "core/util.h"

namespace kf {

namespace {
std::map<std::string, std::string> read_props(const std::string& path) {
  std::map<std::string, std::string> out;
  std::string text;
  if (!read_file(path, text)) return out;
  std::istringstream in(text);
  std::string k, v;
  while (in >> k >> v) out[k] = v;
  return out;
}
std::vector<std::string> list_dir(const std::string& path) {
  std::vector<std::string> out;
  DIR* d = ::opendir(path.c_str());
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    std::string n = e->d_name;
    if (n != "." && n != "..") out.push_back(n);
  }
  ::closedir(d);
  std::sort(out.begin(), out.end(), [](const std::string& a, const std::string& b) { return std::atoi(a.c_str()) < std::atoi(b.c_str()); });
  return out;
}
int64_t to_i(const std::map<std::string, std::string>& m, const std::string& k, int64_t def = 0) {
  auto it = m.find(k);
  return it == m.end() ? def : std::atoll(it->second.c_str());
}
}  // namespace

GpuTopology GpuTopology::synthetic(int n, int numa_nodes) {
  GpuTopology t;
  t.source = "synthetic";
  for (int i = 0; i < n; ++i) {
    GpuDevice d;
    d.index = i;
    d.numa_node = numa_nodes > 0 ? i * numa_nodes / std::max(1, n) : 0;
    char bus[32];
    std::snprintf(bus, sizeof bus, "0000:%02x:00.0", 0x05 + i * 0x10);
    d.pci_bus = bus;
    d.physical = i;
    t.gpus.push_back(d);
  }
  t.link.assign(n, std::vector<int>(n, 1));
  t.bandwidth_gbps.assign(n, std::vector<double>(n, 153.0));
  for (int i = 0; i < n; ++i) {
    t.link[i][i] = 0;
    t.bandwidth_gbps[i][i] = 0;
  }
  return t;
}

std::vector<int> parse_cpulist(const std::string& s) {
  std::set<int> out;
  for (const auto& part : split(trim(s), ',', true)) {
    const size_t dash = part.find('-');
    const int a = std::atoi(part.c_str());
    const int b = dash == std::string::npos ? a : std::atoi(part.c_str() + dash + 1);
    for (int c = a; c <= b && c - a < 65536; ++c) out.insert(c);
  }
  return {out.begin(), out.end()};
}

std::string format_cpulist(const std::vector<int>& cpus) {
  std::vector<int> v(cpus);
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  std::string out;
  for (size_t i = 0; i < v.size();) {
    size_t j = i;
    while (j + 1 < v.size() && v[j + 1] == v[j] + 1) ++j;
    if (!out.empty()) out += ",";
    out += std::to_string(v[i]);
    if (j > i) out += "-" + std::to_string(v[j]);
    i = j + 1;
  }
  return out;
}

SysfsRoots SysfsRoots::under(const std::string& prefix) {
  SysfsRoots r;
  r.kfd = prefix + "/class/kfd/kfd/topology/nodes";
  r.pci = prefix + "/bus/pci/devices";
  r.node = prefix + "/devices/system/node";
  return r;
}

std::vector<int> GpuTopology::local_cpus(const std::vector<int>& devices) const {
  std::vector<int> out;
  for (int d : devices) {
    if (d < 0 || d >= size()) continue;
    for (int c : parse_cpulist(gpus[d].cpulist)) out.push_back(c);
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

int GpuTopology::physical_count() const {
  std::set<int> p;
  for (const auto& g : gpus) p.insert(g.physical);
  return static_cast<int>(p.size());
}

GpuTopology GpuTopology::discover(const std::string& root) {
  SysfsRoots r;
  r.kfd = root;
  return discover(r);
}

GpuTopology GpuTopology::discover(const SysfsRoots& roots) {
  const std::string fake = getenv_or("KFAMD_FAKE_GPUS", "");
  if (!fake.empty()) return synthetic(std::atoi(fake.c_str()));
  const std::string& root = roots.kfd;
  GpuTopology t;
  t.source = "kfd-sysfs";
  std::map<int, int> node_to_gpu;  // kfd node id -> gpu index
  std::vector<int> cpu_nodes;
  for (const auto& n : list_dir(root)) {
    auto props = read_props(root + "/" + n + "/properties");
    if (props.empty()) continue;
    int node = std::atoi(n.c_str());
    if (to_i(props, "simd_count") == 0) {
      cpu_nodes.push_back(node);
      continue;
    }
    GpuDevice d;
    d.index = static_cast<int>(t.gpus.size());
    d.kfd_node = node;
    d.simd_count = static_cast<int>(to_i(props, "simd_count"));
    d.xcc_count = static_cast<int>(to_i(props, "num_xcc", 1));
    if (props.count("drm_render_minor")) d.drm_render_minor = static_cast<int>(to_i(props, "drm_render_minor"));
    int64_t gfx = to_i(props, "gfx_target_version");
    if (gfx) {
      char buf[32];
      std::snprintf(buf, sizeof buf, "gfx%lld%llx", static_cast<long long>(gfx / 10000),
                    static_cast<unsigned long long>(gfx % 10000 / 100 * 16 + gfx % 100));
      // 90500 -> gfx950 (major 9, minor 5, stepping 0)
      std::snprintf(buf, sizeof buf, "gfx%lld%lld%llx", static_cast<long long>(gfx / 10000),
                    static_cast<long long>((gfx / 100) % 100), static_cast<unsigned long long>(gfx % 100));
      d.gfx = buf;
    }
    int64_t loc = to_i(props, "location_id");
    int64_t dom = to_i(props, "domain");
    char bus[32];
    std::snprintf(bus, sizeof bus, "%04llx:%02llx:%02llx.%llx", static_cast<long long>(dom), static_cast<long long>((loc >> 8) & 0xff),
                  static_cast<long long>((loc >> 3) & 0x1f), static_cast<long long>(loc & 0x7));
    d.pci_bus = bus;
    int64_t hbm = 0;
    for (const auto& b : list_dir(root + "/" + n + "/mem_banks")) {
      auto mp = read_props(root + "/" + n + "/mem_banks/" + b + "/properties");
      hbm += to_i(mp, "size_in_bytes");
    }
    if (hbm > 0) d.hbm_bytes = hbm;
    // the PCI function: partition modes, NUMA node and the CPUs local to it
    const std::string pdir = roots.pci + "/" + d.pci_bus;
    std::string v;
    if (read_file(pdir + "/current_compute_partition", v) && !trim(v).empty()) d.compute_partition = to_upper(trim(v));
    if (read_file(pdir + "/current_memory_partition", v) && !trim(v).empty()) d.memory_partition = to_upper(trim(v));
    if (read_file(pdir + "/local_cpulist", v)) d.cpulist = trim(v);
    if (read_file(pdir + "/numa_node", v) && std::atoi(trim(v).c_str()) >= 0) d.numa_node = std::atoi(trim(v).c_str());
    node_to_gpu[node] = d.index;
    t.gpus.push_back(d);
  }
  if (t.gpus.empty()) return synthetic(8);
  // partitions of one package share its PCI function: number packages and partitions in order
  {
    std::map<std::string, int> phys, parts;
    for (auto& g : t.gpus) {
      if (!phys.count(g.pci_bus)) phys[g.pci_bus] = static_cast<int>(phys.size());
      g.physical = phys[g.pci_bus];
      g.partition = parts[g.pci_bus]++;
    }
    // KFD reports each node's memory partition (NPSn: 1/n of the package); compute partitions
    // sharing it split it for accounting: CPX/NPS2 -> 288 / 8 = 36 GiB per device
    for (auto& g : t.gpus) {
      g.hbm_visible_bytes = g.hbm_bytes;
      int nps = std::atoi(g.memory_partition.c_str() + (starts_with(g.memory_partition, "NPS") ? 3 : 0));
      if (nps <= 0) nps = 1;
      const int np = std::max(1, parts[g.pci_bus]);
      g.hbm_bytes = g.hbm_visible_bytes * nps / np;
    }
  }
  const int n = t.size();
  t.link.assign(n, std::vector<int>(n, 2));
  t.bandwidth_gbps.assign(n, std::vector<double>(n, 0.0));
  for (int i = 0; i < n; ++i) t.link[i][i] = 0;
  for (const auto& kv : node_to_gpu) {
    const std::string links = root + "/" + std::to_string(kv.first) + "/io_links";
    for (const auto& l : list_dir(links)) {
      auto lp = read_props(links + "/" + l + "/properties");
      int to = static_cast<int>(to_i(lp, "node_to", -1));
      int type = static_cast<int>(to_i(lp, "type"));
      auto it = node_to_gpu.find(to);
      if (it != node_to_gpu.end() && type == 11) {
        t.link[kv.second][it->second] = 1;
        double bw = static_cast<double>(to_i(lp, "max_bandwidth")) / 1000.0;  // MB/s -> GB/s
        t.bandwidth_gbps[kv.second][it->second] = bw > 0 ? bw : 153.0;
      } else if (std::find(cpu_nodes.begin(), cpu_nodes.end(), to) != cpu_nodes.end()) {
        t.gpus[kv.second].numa_node = to;
      }
    }
  }
  for (auto& g : t.gpus) {
    std::string v;
    if (g.cpulist.empty() && read_file(roots.node + "/node" + std::to_string(g.numa_node) + "/cpulist", v)) g.cpulist = trim(v);
  }
  return t;
}

int GpuTopology::xgmi_degree(int a) const {
  int d = 0;
  for (int j = 0; j < size(); ++j) d += xgmi(a, j) ? 1 : 0;
  return d;
}

Json GpuTopology::to_json() const {
  Json devs = Json::array();
  for (const auto& g : gpus)
    devs.push_back(Json{{"index", g.index}, {"gfx", g.gfx}, {"product", g.product}, {"numa", g.numa_node},
                        {"hbmBytes", g.hbm_bytes}, {"hbmVisibleBytes", g.hbm_visible_bytes}, {"pciBus", g.pci_bus}, {"xgmiDegree", xgmi_degree(g.index)},
                        {"computePartition", g.compute_partition}, {"memoryPartition", g.memory_partition},
                        {"physical", g.physical}, {"partition", g.partition}, {"simdCount", g.simd_count},
                        {"cpulist", g.cpulist}});
  Json m = Json::array();
  for (const auto& row : link) {
    Json r = Json::array();
    for (int v : row) r.push_back(v);
    m.push_back(r);
  }
  return Json{{"source", source}, {"gpus", devs}, {"links", m}};
}

std::string GpuTopology::describe() const {
  if (gpus.empty()) return "no GPUs";
  bool mesh = true;
  std::set<int> numa;
  for (int i = 0; i < size(); ++i) {
    numa.insert(gpus[i].numa_node);
    for (int j = 0; j < size(); ++j)
      if (i != j && !xgmi(i, j)) mesh = false;
  }
  std::string parts;
  if (gpus[0].compute_partition != "SPX" || gpus[0].memory_partition != "NPS1")
    parts = " (" + std::to_string(physical_count()) + " packages in " + gpus[0].compute_partition + "/" +
            gpus[0].memory_partition + ")";
  return std::to_string(size()) + "x " + gpus[0].gfx + parts + (mesh ? " full-mesh xGMI" : " partial xGMI") + ", " +
         std::to_string(numa.size()) + " NUMA node(s)";
}

// ---- placement ---------------------------------------------------------------------------------
std::vector<int> GpuAllocator::ring_order(const GpuTopology& t, const std::vector<int>& devs) {
  if (devs.size() <= 2) return devs;
  // DFS for a Hamiltonian cycle over direct xGMI links (n <= 8 -> trivial cost)
  std::vector<int> path{devs[0]};
  std::vector<bool> used(devs.size(), false);
  used[0] = true;
  std::function<bool()> dfs = [&]() -> bool {
    if (path.size() == devs.size()) return t.xgmi(path.back(), path.front());
    for (size_t i = 1; i < devs.size(); ++i) {
      if (used[i] || !t.xgmi(path.back(), devs[i])) continue;
      used[i] = true;
      path.push_back(devs[i]);
      if (dfs()) return true;
      path.pop_back();
      used[i] = false;
    }
    return false;
  };
  if (dfs()) return path;
  return devs;  // no direct-link cycle: fall back to index order (RCCL will route via PCIe/host)
}

bool GpuAllocator::choose(const GpuTopology& t, const std::set<int>& free, int n, Placement& out) {
  if (n <= 0) {
    out = Placement{};
    out.reason = "no GPUs requested";
    return true;
  }
  if (static_cast<int>(free.size()) < n) return false;
  // group free devices by NUMA node
  std::map<int, std::vector<int>> by_numa;
  for (int d : free) by_numa[t.gpus[d].numa_node].push_back(d);
  // pairwise-connected subset test
  auto connected = [&](const std::vector<int>& s) {
    for (size_t i = 0; i < s.size(); ++i)
      for (size_t j = i + 1; j < s.size(); ++j)
        if (!t.xgmi(s[i], s[j])) return false;
    return true;
  };
  // 1) best-fit single NUMA node
  int best_numa = -1;
  size_t best_free = SIZE_MAX;
  for (auto& kv : by_numa) {
    if (static_cast<int>(kv.second.size()) < n) continue;
    std::vector<int> cand(kv.second.begin(), kv.second.begin() + n);
    if (n > 1 && !connected(cand)) continue;
    if (kv.second.size() < best_free) {
      best_free = kv.second.size();
      best_numa = kv.first;
    }
  }
  if (best_numa >= 0) {
    out.devices.assign(by_numa[best_numa].begin(), by_numa[best_numa].begin() + n);
    out.numa_node = best_numa;
    out.reason = "numa-local best fit (numa " + std::to_string(best_numa) + ")";
  } else {
    // 2) span NUMA nodes: greedy, prefer keeping whole-node holes (take from fullest-free first),
    //    only xGMI-connected additions
    std::vector<std::pair<int, std::vector<int>>> nodes(by_numa.begin(), by_numa.end());
    std::sort(nodes.begin(), nodes.end(), [](auto& a, auto& b) { return a.second.size() > b.second.size(); });
    std::vector<int> pick;
    for (auto& nd : nodes)
      for (int d : nd.second) {
        if (static_cast<int>(pick.size()) == n) break;
        bool ok = true;
        for (int p : pick) ok = ok && t.xgmi(p, d);
        if (ok) pick.push_back(d);
      }
    if (static_cast<int>(pick.size()) < n) {
      // 3) last resort: any free devices (PCIe between some pairs)
      pick.assign(free.begin(), free.end());
      pick.resize(n);
      out.reason = "fragmented: not all pairs xGMI-connected";
    } else {
      out.reason = "spans NUMA nodes (xGMI-connected)";
    }
    std::sort(pick.begin(), pick.end());
    out.devices = pick;
    out.numa_node = -1;
  }
  out.ring = ring_order(t, out.devices);
  return true;
}

bool GpuAllocator::allocate(const std::string& owner, int n, Placement& out) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = alloc_.find(owner);
  if (it != alloc_.end()) {
    out.devices = it->second;
    out.ring = ring_order(topo_, out.devices);
    out.reason = "existing allocation";
    return true;
  }
  std::set<int> free;
  for (int i = 0; i < topo_.size(); ++i) free.insert(i);
  for (auto& kv : alloc_)
    for (int d : kv.second) free.erase(d);
  if (!choose(topo_, free, n, out)) return false;
  if (n > 0) alloc_[owner] = out.devices;
  return true;
}

void GpuAllocator::release(const std::string& owner) {
  std::lock_guard<std::mutex> g(mu_);
  alloc_.erase(owner);
}

void GpuAllocator::adopt(const std::string& owner, const std::vector<int>& devices) {
  std::lock_guard<std::mutex> g(mu_);
  alloc_[owner] = devices;
}

std::vector<int> GpuAllocator::free_devices() const {
  std::lock_guard<std::mutex> g(mu_);
  std::set<int> free;
  for (int i = 0; i < topo_.size(); ++i) free.insert(i);
  for (auto& kv : alloc_)
    for (int d : kv.second) free.erase(d);
  return std::vector<int>(free.begin(), free.end());
}

int GpuAllocator::free_count() const { return static_cast<int>(free_devices().size()); }

std::map<std::string, std::vector<int>> GpuAllocator::allocations() const {
  std::lock_guard<std::mutex> g(mu_);
  return alloc_;
}

Json gpu_env_for(const Placement& p, const GpuTopology& t, bool multi_gpu, const std::string& master_addr,
                 int master_port) {
  Json env = Json::array();
  auto add = [&](const std::string& k, const std::string& v) { env.push_back(Json{{"name", k}, {"value", v}}); };
  std::vector<std::string> ids, ring;
  for (int d : p.devices) ids.push_back(std::to_string(d));
  // devices are renumbered 0..n-1 inside the pod; the ring is expressed in pod-local ordinals
  for (int d : p.ring) {
    auto pos = std::find(p.devices.begin(), p.devices.end(), d) - p.devices.begin();
    ring.push_back(std::to_string(pos));
  }
  // the container view of a device-plugin allocation: ROCr brings up only these agents (a process
  // pod otherwise initialises, and at exit tears down, every GPU of the node), renumbered 0..n-1
  // for HIP; KFAMD_GPU_IDS keeps the node-level ids
  std::vector<std::string> local;
  for (size_t i = 0; i < ids.size(); ++i) local.push_back(std::to_string(i));
  add("ROCR_VISIBLE_DEVICES", join(ids, ","));
  add("HIP_VISIBLE_DEVICES", join(local, ","));
  add("KFAMD_GPU_IDS", join(ids, ","));
  add("KFAMD_XGMI_RING", join(ring, ","));
  add("KFAMD_GPU_TOPOLOGY", t.describe());
  if (t.source == "synthetic") add("KFAMD_SIMULATED_GPUS", "1");  // CI node: no /dev/kfd behind these ids
  if (multi_gpu) {
    // single-node torchrun / RCCL wiring: one process per GPU, a rendezvous endpoint
    // private to this pod, xGMI P2P enabled, no IB/socket fallbacks inside the pod.
    add("LOCAL_WORLD_SIZE", std::to_string(p.devices.size()));
    add("WORLD_SIZE", std::to_string(p.devices.size()));
    add("MASTER_ADDR", master_addr.empty() ? "127.0.0.1" : master_addr);
    add("MASTER_PORT", std::to_string(master_port > 0 ? master_port : 29500));
    add("NCCL_IB_DISABLE", "1");
    add("NCCL_P2P_LEVEL", "SYS");
    add("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1");
    add("HSA_ENABLE_IPC_MODE_LEGACY", "0");
  }
  return env;
}

}  // namespace kf
