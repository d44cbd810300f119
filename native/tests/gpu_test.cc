// gpu_test.cc — MI355X topology, xGMI placement, quota accounting.
#include <set>

#include "admission/admission.h"
#include "gpu/topology.h"
#include "tests/harness.h"

using kf::GpuAllocator;
using kf::GpuTopology;
using kf::Json;
using kf::Placement;

TEST(gpu, cpulist_parse_format) {
  CHECK(kf::parse_cpulist("0-3,8,10-11\n") == std::vector<int>({0, 1, 2, 3, 8, 10, 11}));
  CHECK_EQ(kf::format_cpulist({11, 0, 1, 2, 3, 8, 10, 3}), std::string("0-3,8,10-11"));
  CHECK(kf::parse_cpulist("").empty());
}

TEST(gpu, placement_numa_best_fit_and_ring) {
  const GpuTopology t = GpuTopology::synthetic(8, 2);  // GPUs 0-3 on NUMA 0, 4-7 on NUMA 1
  Placement p;
  // a 2-GPU request prefers the NUMA node with the fewest free GPUs that still fits (anti-fragmentation)
  REQUIRE(GpuAllocator::choose(t, {1, 2, 3, 4, 5, 6, 7}, 2, p));
  CHECK_EQ(p.devices.size(), static_cast<size_t>(2));
  for (int d : p.devices) CHECK(d >= 1 && d <= 3);
  REQUIRE(GpuAllocator::choose(t, {0, 1, 2, 3, 4, 5, 6, 7}, 8, p));
  CHECK_EQ(p.ring.size(), static_cast<size_t>(8));
  std::set<int> ring(p.ring.begin(), p.ring.end());
  CHECK_EQ(ring.size(), static_cast<size_t>(8));
  for (size_t i = 0; i < p.ring.size(); ++i) CHECK(t.xgmi(p.ring[i], p.ring[(i + 1) % p.ring.size()]));
  CHECK(!GpuAllocator::choose(t, {0, 1}, 3, p));
}

TEST(gpu, allocator_is_idempotent_per_owner_and_releases) {
  GpuAllocator a(GpuTopology::synthetic(8, 2));
  Placement p1, p2;
  REQUIRE(a.allocate("pod-a", 4, p1));
  REQUIRE(a.allocate("pod-a", 4, p2));
  CHECK(p1.devices == p2.devices);
  CHECK_EQ(a.free_count(), 4);
  Placement q;
  CHECK(!a.allocate("pod-b", 5, q));
  a.release("pod-a");
  CHECK_EQ(a.free_count(), 8);
}

TEST(gpu, quota_usage_charges_hbm_per_gpu) {
  const Json pod = Json::parse(R"({"spec":{"containers":[{"name":"c","resources":{"limits":{"amd.com/gpu":"2","cpu":"4"}}}],
                                           "initContainers":[{"name":"i","resources":{"requests":{"cpu":"8"}}}]}})");
  auto u = kf::pod_quota_usage(pod, 288);
  CHECK_EQ(u["amd.com/gpu"], 2.0);
  CHECK_EQ(u["amd.com/gpu-memory"], 576.0);
  CHECK_EQ(u["requests.cpu"], 8.0);  // init containers: max, not sum
  CHECK_EQ(u["limits.cpu"], 4.0);
  auto cpx = kf::pod_quota_usage(pod, 36);  // CPX/NPS2 partitions: 288 / 8
  CHECK_EQ(cpx["amd.com/gpu-memory"], 72.0);
}
