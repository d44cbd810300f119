// topology.h — K6/K7: MI355X node topology discovery, xGMI-aware GPU placement and HBM accounting.
//
// Discovery reads the KFD topology in sysfs (/sys/class/kfd/kfd/topology/nodes/*): GPU nodes have
// simd_count > 0; their io_links of type 11 (HSA_IOLINK_TYPE_XGMI) give the xGMI graph (an 8-GPU
// MI355X platform is a full mesh: 7 links per GPU), the PCIe link to a CPU node gives the NUMA
// affinity, mem_banks give the HBM size. Without a GPU (CI, this container) a synthetic 8 x MI355X
// full mesh is used, or KFAMD_FAKE_GPUS=N.
//
// Placement (the device-plugin "GetPreferredAllocation" equivalent) picks, for a request of n GPUs:
//   1. sets whose members are pairwise xGMI-connected (always true on a full mesh);
//   2. within one NUMA node when possible (host <-> device traffic and RCCL proxy threads local);
//   3. best fit: the NUMA node / hive with the fewest free GPUs that still fits (anti-fragmentation,
//      so an 8-GPU request can still be served later);
//   4. lowest device ids as tie-break (deterministic).
// It returns the device ids and a ring order (a Hamiltonian cycle over direct xGMI links) that is
// exported to the pod as RCCL/torch env so collectives run ring-by-link.
#pragma once

#include <cstdint>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

struct GpuDevice {
  int index = 0;          // HIP device ordinal (order of KFD GPU nodes)
  int kfd_node = -1;
  int numa_node = 0;
  std::string gfx = "gfx950";
  std::string product = "AMD Instinct MI355X";
  int64_t hbm_bytes = 288LL << 30;          // this device's share of its package's HBM (quota unit)
  int64_t hbm_visible_bytes = 288LL << 30;  // what a process on it can address (its memory partition)
  int simd_count = 1024;  // 256 CUs x 4 SIMDs
  int xcc_count = 8;
  std::string pci_bus;
  int drm_render_minor = -1;  // /sys/class/drm/renderD<minor>: amdgpu sysfs (VRAM use, busy %)
  std::string compute_partition = "SPX";  // SPX | DPX | QPX | CPX
  std::string memory_partition = "NPS1";  // NPS1 | NPS2 | NPS4 | NPS8
  int physical = 0;   // physical MI355X package this device (partition) belongs to
  int partition = 0;  // partition index within the package
  std::string cpulist;  // NUMA-local CPUs ("0-47,96-143"); "" = unknown
};

// "0-3,8,10-11" <-> sorted CPU ids
std::vector<int> parse_cpulist(const std::string& s);
std::string format_cpulist(const std::vector<int>& cpus);

struct SysfsRoots {
  std::string kfd = "/sys/class/kfd/kfd/topology/nodes";
  std::string pci = "/sys/bus/pci/devices";
  std::string node = "/sys/devices/system/node";
  // all three under one prefix (tests: a fake tree)
  static SysfsRoots under(const std::string& prefix);
};

struct GpuTopology {
  std::vector<GpuDevice> gpus;
  // link[i][j]: 0 = none, 1 = xGMI direct, 2 = PCIe / via CPU
  std::vector<std::vector<int>> link;
  // per-link bandwidth estimate (GB/s, one direction) for the xGMI links
  std::vector<std::vector<double>> bandwidth_gbps;
  std::string source;  // "kfd-sysfs" | "synthetic"

  static GpuTopology discover(const std::string& sysfs_root = "/sys/class/kfd/kfd/topology/nodes");
  static GpuTopology discover(const SysfsRoots& roots);
  // CPUs local to a set of devices (union of their cpulists); empty = unknown
  std::vector<int> local_cpus(const std::vector<int>& devices) const;
  int physical_count() const;
  static GpuTopology synthetic(int n, int numa_nodes = 2);
  int size() const { return static_cast<int>(gpus.size()); }
  bool xgmi(int a, int b) const { return a != b && link[a][b] == 1; }
  int xgmi_degree(int a) const;
  Json to_json() const;
  std::string describe() const;  // "8x gfx950 full-mesh xGMI, 2 NUMA nodes"
};

struct Placement {
  std::vector<int> devices;  // chosen device indices
  std::vector<int> ring;     // ring order over xGMI links
  int numa_node = -1;
  std::string reason;
};

class GpuAllocator {
 public:
  explicit GpuAllocator(GpuTopology topo) : topo_(std::move(topo)) {}
  const GpuTopology& topology() const { return topo_; }
  // Allocate n devices to `owner` (pod uid). Idempotent per owner. False when not enough free.
  bool allocate(const std::string& owner, int n, Placement& out);
  void release(const std::string& owner);
  // Restore an allocation recorded in a pod annotation (kubelet restart).
  void adopt(const std::string& owner, const std::vector<int>& devices);
  std::vector<int> free_devices() const;
  int free_count() const;
  std::map<std::string, std::vector<int>> allocations() const;

  // pure placement function (unit-tested)
  static bool choose(const GpuTopology& t, const std::set<int>& free, int n, Placement& out);
  static std::vector<int> ring_order(const GpuTopology& t, const std::vector<int>& devs);

 private:
  GpuTopology topo_;
  mutable std::mutex mu_;
  std::map<std::string, std::vector<int>> alloc_;
};

// Env for a pod's containers given its placement (HIP_VISIBLE_DEVICES, RCCL/torch rendezvous).
// master_addr/master_port: the pod's own rendezvous endpoint (multi-GPU pods only)
Json gpu_env_for(const Placement& p, const GpuTopology& t, bool multi_gpu, const std::string& master_addr = "127.0.0.1",
                 int master_port = 29500);

}  // namespace kf
