// tu/w4_wgrad_pair.hip — two weight gradients in one launch (gemm_w4.h GRP): a transformer block's
// QKV and output-projection wgrads are 192 + 64 tiles of 256 x 256 at gpt-1b, 75 % and 25 % of the
// 256 CUs alone (the second one ran split-K); together one full wave (ops.attention attn_block).
#include "gemm_w4.h"

using namespace kfw4;

// C_i[M_i][N] = A_i^T . B_i with A_i [K][M_i] (row stride lda_i) and B_i [K][N] (ldb_i), both read
// k-major (LA = LB = 1, the wgrad layout of gemm_bf16_w4_t.hip); C_i row stride ldc_i.
// splits > 1: the K range in `splits` pieces of kper (kper % 64 == 0, every piece non-empty) with the
// in-kernel fixup (gemm_w4.h SPLIT == 2) over both problems' tiles: W holds splits x (tiles 1 + 2)
// fp32 partial tiles of 256 x 256 (16-B aligned), cnt (tiles 1 + 2) arrival counters, zero on entry
// and left zero (one pair per stream) — for pairs that under-fill the chip even together.
extern "C" int kfamd_w4_wgrad_pair_v2(const void* A1, const void* B1, void* C1, int M1, long long lda1, long long ldb1,
                                      long long ldc1, const void* A2, const void* B2, void* C2, int M2, long long lda2,
                                      long long ldb2, long long ldc2, int N, int N2, int K, int splits, int kper,
                                      float* W, unsigned* cnt, void* stream);

extern "C" int kfamd_w4_wgrad_pair(const void* A1, const void* B1, void* C1, int M1, long long lda1, long long ldb1,
                                   long long ldc1, const void* A2, const void* B2, void* C2, int M2, long long lda2,
                                   long long ldb2, long long ldc2, int N, int K, void* stream) {
  return kfamd_w4_wgrad_pair_v2(A1, B1, C1, M1, lda1, ldb1, ldc1, A2, B2, C2, M2, lda2, ldb2, ldc2, N, N, K, 1, 0,
                                nullptr, nullptr, stream);
}

extern "C" int kfamd_w4_wgrad_pair_v2(const void* A1, const void* B1, void* C1, int M1, long long lda1, long long ldb1,
                                      long long ldc1, const void* A2, const void* B2, void* C2, int M2, long long lda2,
                                      long long ldb2, long long ldc2, int N, int N2, int K, int splits, int kper,
                                      float* W, unsigned* cnt, void* stream) {
  int rc = check_shape(1, 1, 256, A1, B1, C1, nullptr, nullptr, nullptr, M1, N, K, lda1, ldb1, ldc1, 0, 0, 0, 0, 0);
  if (rc != KFAMD_OK) return rc;
  rc = check_shape(1, 1, 256, A2, B2, C2, nullptr, nullptr, nullptr, M2, N2, K, lda2, ldb2, ldc2, 0, 0, 0, 0, 0);
  if (rc != KFAMD_OK) return rc;
  const long long t1 = (long long)((M1 + 255) / 256) * ((N + 255) / 256);
  const long long t2 = (long long)((M2 + 255) / 256) * ((N2 + 255) / 256);
  if (t1 + t2 >= (1LL << 31)) return KFAMD_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const W4Grp g2{static_cast<const __bf16*>(A2), static_cast<const __bf16*>(B2), static_cast<__bf16*>(C2), M2, N2,
                 lda2, ldb2, ldc2};
  if (splits > 1) {
    if (!W || !cnt || splits > 64 || kper < kBK || kper % kBK || (long long)kper * (splits - 1) >= K) return KFAMD_EINVAL;
    if ((reinterpret_cast<uintptr_t>(W) & 15) || (reinterpret_cast<uintptr_t>(cnt) & 3)) return KFAMD_EALIGN;
    hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, 1, 1, 256, 2, false, 0, false, false, false, true>),
                       dim3((unsigned)(t1 + t2), 1, splits), dim3(kThreads), 0, s, static_cast<const __bf16*>(A1),
                       static_cast<const __bf16*>(B1), static_cast<__bf16*>(C1), nullptr, nullptr, nullptr, M1, N, K,
                       lda1, ldb1, ldc1, 0LL, 0LL, 0LL, 0LL, 0LL, 1.0f, nullptr, W, kper, cnt, 0u, g2);
  } else {
    hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, 1, 1, 256, 0, false, 0, false, false, false, true>),
                       dim3((unsigned)(t1 + t2)), dim3(kThreads), 0, s, static_cast<const __bf16*>(A1),
                       static_cast<const __bf16*>(B1), static_cast<__bf16*>(C1), nullptr, nullptr, nullptr, M1, N, K,
                       lda1, ldb1, ldc1, 0LL, 0LL, 0LL, 0LL, 0LL, 1.0f, nullptr, nullptr, 0, nullptr, 0u, g2);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
