// Stream-K timing A/B build (tools/sk_ab.py): the plain-epilogue SK instantiation only, compiled with
// -DKFW4_SK_AB=<n> (gemm_w4.h) into its own library.
#include "gemm_w4.h"

using namespace kfw4;

extern "C" int skab_launch(const void* A, const void* B, void* C, int M, int N, int K, float* W, unsigned* flags,
                           unsigned epoch, int grid, int splits, void* stream) {
  hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, 0, 0, 256, false, false, 0, true>), dim3(grid),
                     dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream), static_cast<const __bf16*>(A),
                     static_cast<const __bf16*>(B), static_cast<__bf16*>(C), nullptr, nullptr, nullptr, M, N, K,
                     (long long)K, (long long)K, (long long)N, 0LL, 0LL, 0LL, 0LL, 0LL, 1.0f, nullptr, W, splits, flags,
                     epoch);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
