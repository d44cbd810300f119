// gemm_w4_sk.h — one stream-K kernel variant per translation unit (kernels/tu/w4_sk_*.hip): the
// persistent-schedule kernels are the slowest of the library to compile (~40 s each), so each builds
// on its own core. The dispatcher with the argument checks is kernels/gemm_bf16_w4_sk.hip.
#pragma once
#include "gemm_w4.h"

#define KFW4_SK_ENTRY(NAME, ACT, HB, HR)                                                                            \
  extern "C" int NAME(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,   \
                      long long lda, long long ldb, long long ldc, long long ldr, float alpha, float* W,            \
                      unsigned* flags, unsigned epoch, int grid, int splits, void* stream) {                         \
    using namespace kfw4;                                                                                          \
    hipLaunchKernelGGL((gemm_w4<ACT, HB, HR, false, 0, 0, 256, false, false, 0, true>), dim3(grid), dim3(kThreads), \
                       0, reinterpret_cast<hipStream_t>(stream), static_cast<const __bf16*>(A),                      \
                       static_cast<const __bf16*>(B), static_cast<__bf16*>(C), static_cast<const __bf16*>(bias),     \
                       static_cast<const __bf16*>(R), nullptr, M, N, K, lda, ldb, ldc, ldr, 0LL, 0LL, 0LL, 0LL, alpha, \
                       nullptr, W, splits, flags, epoch);                                                            \
    const hipError_t e = hipGetLastError();                                                                          \
    return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);                                                         \
  }
