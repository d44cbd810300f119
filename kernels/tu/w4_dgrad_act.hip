// tu/w4_dgrad_act.hip — a linear layer's dgrad through the previous layer's activation in one GEMM
// (gemm_w4.h DACT): G = (dY . W) * act'(Z) plus the column-sum partials of G, then the partials'
// fold (act_grad_bf16.hip colsum_finalize). Replaces, on an MLP's backward (ops.mlp), the fc2 dgrad
// GEMM followed by act_grad_bf16.hip's pass over dH and Z (profiles/r5ze_mlp).
#include "gemm_w4.h"

using namespace kfw4;

// KFW4_DACT_BM: the tile. 128 runs two workgroups per CU, so one workgroup's epilogue (the
// pre-activation reads and the G stores) overlaps the other's K loop (A/B runs, profiles/r5ze_mlp)
#ifndef KFW4_DACT_BM
#define KFW4_DACT_BM 256
#endif
constexpr int kDactBM = KFW4_DACT_BM;

extern "C" long long kfamd_w4_dgrad_act_workspace(int M, int N) {
  return (long long)((M + kDactBM / 2 - 1) / (kDactBM / 2)) * N * (long long)sizeof(float);
}

extern "C" int kfamd_w4_dgrad_act(const void* dy, const void* w, void* g, const void* z, int M, int N, int K,
                                  long long lda, long long ldb, long long ldg, long long ldz, int act, float* ws,
                                  void* db, int db_bf16, void* stream) {
  // kernel A = dY [M][K] (LA = 0), kernel B = W [K][N] read k-major (LB = 1), R = Z
  const int rc = check_shape(0, 1, kDactBM, dy, w, g, nullptr, z, nullptr, M, N, K, lda, ldb, ldg, ldz, 0, 0, 0, 0);
  if (rc != KFAMD_OK) return rc;
  if (M % kDactBM || N % kDactBM || K % kBK || !z || (db && !ws)) return KFAMD_EINVAL;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al16(g) || !al16(z) || (ws && !al16(ws)) || ldg % 8 || ldz % 8) return KFAMD_EALIGN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((M / kDactBM) * (N / kDactBM), 1), block(kThreads);
  const __bf16* a = static_cast<const __bf16*>(dy);
  const __bf16* b = static_cast<const __bf16*>(w);
  const __bf16* r = static_cast<const __bf16*>(z);
  __bf16* c = static_cast<__bf16*>(g);
  float* W = db ? ws : nullptr;
#define DACT_GO(ACTV)                                                                                             \
  hipLaunchKernelGGL((gemm_w4<ACTV, false, true, false, 0, 1, kDactBM, 0, false, 0, false, false, true>), grid, block, 0, \
                     s, a, b, c, nullptr, r, nullptr, M, N, K, lda, ldb, ldg, ldz, 0LL, 0LL, 0LL, 0LL, 1.0f, nullptr, W)
  switch (act) {
    case KFAMD_ACT_GELU_TANH: DACT_GO(KFAMD_ACT_GELU_TANH); break;
    case KFAMD_ACT_SILU: DACT_GO(KFAMD_ACT_SILU); break;
    case KFAMD_ACT_RELU: DACT_GO(KFAMD_ACT_RELU); break;
    default: return KFAMD_EINVAL;
  }
#undef DACT_GO
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return static_cast<int>(e);
  if (db) return kfamd_colsum_finalize(ws, db, db_bf16, M / (kDactBM / 2), N, stream);
  return KFAMD_OK;
}
