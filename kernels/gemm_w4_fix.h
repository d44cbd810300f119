// gemm_w4_fix.h — split-K with the in-kernel fixup (gemm_w4.h SPLIT == 2), one operand layout per
// translation unit (kernels/tu/w4_fix_*.hip); the dispatcher with the argument checks is
// kfamd_w4_splitk_fix in kernels/gemm_bf16_w4_t.hip.
#pragma once
#include "gemm_w4.h"

#define KFW4_FIX_ENTRY(NAME, LA, LB)                                                                                 \
  extern "C" int NAME(const void* A, const void* B, void* C, const void* R, int M, int N, int K, int batch,          \
                      long long lda, long long ldb, long long ldc, long long ldr, long long sa, long long sb,         \
                      long long sc, long long sr, float alpha, float* W, unsigned* cnt, int splits, int kper,          \
                      void* stream) {                                                                                 \
    using namespace kfw4;                                                                                             \
    const dim3 grid(((M + 255) / 256) * ((N + 255) / 256), batch, splits), block(kThreads);                          \
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);                                                           \
    const __bf16* a = static_cast<const __bf16*>(A);                                                                 \
    const __bf16* b = static_cast<const __bf16*>(B);                                                                 \
    __bf16* c = static_cast<__bf16*>(C);                                                                             \
    const __bf16* r = static_cast<const __bf16*>(R);                                                                 \
    if (R)                                                                                                            \
      hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, true, false, LA, LB, 256, 2>), grid, block, 0, s, a, b, c,   \
                         nullptr, r, nullptr, M, N, K, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, nullptr, W, kper,   \
                         cnt, 0u);                                                                                    \
    else                                                                                                              \
      hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, LA, LB, 256, 2>), grid, block, 0, s, a, b, c,  \
                         nullptr, nullptr, nullptr, M, N, K, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, nullptr, W,   \
                         kper, cnt, 0u);                                                                              \
    const hipError_t e = hipGetLastError();                                                                           \
    return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);                                                          \
  }
