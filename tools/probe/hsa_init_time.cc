// time the ROCr (HSA) runtime bring-up stages in a fresh process, to size what HIP adds on top
#include <hsa/hsa.h>
#include <chrono>
#include <cstdio>
static double ms(std::chrono::steady_clock::time_point a) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}
static hsa_status_t find_gpu(hsa_agent_t a, void* d) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) { *static_cast<hsa_agent_t*>(d) = a; return HSA_STATUS_INFO_BREAK; }
  return HSA_STATUS_SUCCESS;
}
int main() {
  auto t0 = std::chrono::steady_clock::now();
  if (hsa_init() != HSA_STATUS_SUCCESS) { std::printf("hsa_init failed\n"); return 1; }
  double t_init = ms(t0);
  auto t1 = std::chrono::steady_clock::now();
  hsa_agent_t gpu{};
  hsa_iterate_agents(find_gpu, &gpu);
  double t_agents = ms(t1);
  auto t2 = std::chrono::steady_clock::now();
  hsa_queue_t* q = nullptr;
  hsa_status_t st = hsa_queue_create(gpu, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q);
  double t_queue = ms(t2);
  std::printf("{\"hsa_init_ms\": %.2f, \"agents_ms\": %.2f, \"queue_create_ms\": %.2f, \"queue_ok\": %d}\n", t_init, t_agents, t_queue, st == HSA_STATUS_SUCCESS);
  if (q) hsa_queue_destroy(q);
  hsa_shut_down();
  return 0;
}
