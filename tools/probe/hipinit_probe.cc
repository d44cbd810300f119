// Start-up cost probe: where does a fresh process's GPU runtime start-up go on MI355X?
//   hipinit_probe hsa   -> open(/dev/kfd) + hsa_init() + agent iteration
//   hipinit_probe hip   -> hipGetDeviceCount() (HIP platform init on top of ROCr)
//   hipinit_probe alloc -> hipGetDeviceCount() then the first hipMalloc + hipMemset + sync
// Prints one JSON line of millisecond timings.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "hip";
  auto t0 = std::chrono::steady_clock::now();
  if (!std::strcmp(mode, "hsa")) {
    int fd = open("/dev/kfd", O_RDWR);
    double kfd_ms = ms_since(t0);
    if (fd >= 0) close(fd);
    auto t1 = std::chrono::steady_clock::now();
    hsa_status_t st = hsa_init();
    double init_ms = ms_since(t1);
    int agents = 0;
    hsa_iterate_agents([](hsa_agent_t, void* p) { ++*static_cast<int*>(p); return HSA_STATUS_SUCCESS; }, &agents);
    auto t2 = std::chrono::steady_clock::now();
    hsa_shut_down();
    std::printf("{\"mode\":\"hsa\",\"open_kfd_ms\":%.2f,\"hsa_init_ms\":%.2f,\"status\":%d,\"agents\":%d,\"shutdown_ms\":%.2f}\n",
                kfd_ms, init_ms, (int)st, agents, ms_since(t2));
    return 0;
  }
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  double count_ms = ms_since(t0);
  double alloc_ms = 0, memset_ms = 0;
  if (!std::strcmp(mode, "alloc") && e == hipSuccess && n > 0) {
    auto t1 = std::chrono::steady_clock::now();
    void* p = nullptr;
    (void)hipMalloc(&p, 64 << 20);
    alloc_ms = ms_since(t1);
    auto t2 = std::chrono::steady_clock::now();
    (void)hipMemset(p, 0, 64 << 20);
    (void)hipDeviceSynchronize();
    memset_ms = ms_since(t2);
    (void)hipFree(p);
  }
  std::printf("{\"mode\":\"%s\",\"devices\":%d,\"hipGetDeviceCount_ms\":%.2f,\"first_malloc_ms\":%.2f,\"first_memset_sync_ms\":%.2f}\n",
              mode, n, count_ms, alloc_ms, memset_ms);
  return 0;
}
