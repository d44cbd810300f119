#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
static double ms(std::chrono::steady_clock::time_point a) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}
int main() {
  auto t0 = std::chrono::steady_clock::now();
  int n = 0;
  hipGetDeviceCount(&n);
  double t_init = ms(t0);
  auto t1 = std::chrono::steady_clock::now();
  hipStream_t s;
  hipSetDevice(0);
  hipStreamCreate(&s);
  double t_stream = ms(t1);
  std::printf("{\"hip_init_ms\": %.2f, \"stream_ms\": %.2f, \"devices\": %d}\n", t_init, t_stream, n);
  return 0;
}
