// gemm_bf16_w4.hip — K1 variant "w4" in the forward ("NT") layout: C = act(alpha * A B^T + bias)
// (+ R), A [M][K], B [N][K], on the 4-wave template of gemm_w4.h (256x256 tile "w4" or 128x128
// "w4s"), with in-kernel edge tiles (any M, N >= the tile, N % 8, K % 8) and an optional second
// output Aux = the pre-activation (gelu/silu backward without recomputing the GEMM).
// The backward layouts live in gemm_bf16_w4_t.hip.
//
// History kept out of this file: profiles/r1_gemm_w4 (register placement: asm MFMA with tied AGPR
// accumulators, buffer_load..lds with SGPR row offsets), profiles/r1_gemm_w4c (5-slot ring),
// profiles/r2_gemm_knobs + r2_gemm_stalls (knob A/Bs, issue-stall diagnosis).
#include "gemm_w4.h"

using namespace kfw4;

namespace {

template <int BM>
int launch_nt(const void* A, const void* B, void* C, const void* bias, const void* R, void* Aux, int M, int N, int K,
              int batch, long long lda, long long ldb, long long ldc, long long ldr, long long sa, long long sb,
              long long sc, long long sr, float alpha, int act, void* stream) {
  const int rc = check_shape(0, 0, BM, A, B, C, bias, R, Aux, M, N, K, lda, ldb, ldc, ldr, sa, sb, sc, sr);
  if (rc != KFAMD_OK) return rc;
  if (Aux && (act == KFAMD_ACT_NONE || R)) return KFAMD_EINVAL;
  if (R && act != KFAMD_ACT_NONE) return KFAMD_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(((M + BM - 1) / BM) * ((N + BM - 1) / BM), batch), block(kThreads);
  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
  __bf16* c = static_cast<__bf16*>(C);
  const __bf16* bs = static_cast<const __bf16*>(bias);
  const __bf16* r = static_cast<const __bf16*>(R);
  __bf16* x = static_cast<__bf16*>(Aux);
  const bool hb = bias != nullptr, hr = R != nullptr, hx = Aux != nullptr;
#define W4_LAUNCH(ACTV, HB, HR, HX)                                                                                \
  hipLaunchKernelGGL((gemm_w4<ACTV, HB, HR, HX, 0, 0, BM>), grid, block, 0, s, a, b, c, bs, r, x, M, N, K, lda, ldb, \
                     ldc, ldr, sa, sb, sc, sr, alpha, nullptr)
#define W4_ACT(ACTV)                                       \
  if (hx) {                                                \
    if (hb) W4_LAUNCH(ACTV, true, false, true);            \
    else W4_LAUNCH(ACTV, false, false, true);              \
  } else {                                                 \
    if (hb) W4_LAUNCH(ACTV, true, false, false);           \
    else W4_LAUNCH(ACTV, false, false, false);             \
  }
  switch (act) {
    case KFAMD_ACT_NONE:
      if (hb && hr) W4_LAUNCH(KFAMD_ACT_NONE, true, true, false);
      else if (hb) W4_LAUNCH(KFAMD_ACT_NONE, true, false, false);
      else if (hr) W4_LAUNCH(KFAMD_ACT_NONE, false, true, false);
      else W4_LAUNCH(KFAMD_ACT_NONE, false, false, false);
      break;
    case KFAMD_ACT_RELU:
      if (hx) return KFAMD_EINVAL;  // relu's backward needs only the output's sign
      if (hb) W4_LAUNCH(KFAMD_ACT_RELU, true, false, false);
      else W4_LAUNCH(KFAMD_ACT_RELU, false, false, false);
      break;
    case KFAMD_ACT_GELU_TANH:
      W4_ACT(KFAMD_ACT_GELU_TANH);
      break;
    case KFAMD_ACT_SILU:
      W4_ACT(KFAMD_ACT_SILU);
      break;
    default:
      return KFAMD_EINVAL;
  }
#undef W4_ACT
#undef W4_LAUNCH
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

}  // namespace

// NT layout on the w4 template; bm = 256 ("w4") or 128 ("w4s"). Shapes/alignment: check_shape.
extern "C" int kfamd_w4_launch_nt(int bm, const void* A, const void* B, void* C, const void* bias, const void* R,
                                  void* Aux, int M, int N, int K, int batch, long long lda, long long ldb, long long ldc,
                                  long long ldr, long long sa, long long sb, long long sc, long long sr, float alpha,
                                  int act, void* stream) {
  if (bm == 256)
    return launch_nt<256>(A, B, C, bias, R, Aux, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, act, stream);
  if (bm == 128)
    return launch_nt<128>(A, B, C, bias, R, Aux, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, act, stream);
  return KFAMD_EINVAL;
}

#ifdef KFAMD_DIAG
// Diagnostic build only (libkfamd_kernels_diag.so, kubeflow_rm_amd._build.build_diag_kernels; never
// in the production library): per-wave K-loop segment cycle sums into diag
// [(M/256)*(N/256) blocks][4 waves][16 words] (tools/w4_diag.py).
extern "C" int kfamd_gemm_nt_bf16_w4_diag(const void* A, const void* B, void* C, int M, int N, int K,
                                          unsigned long long* diag, int abl, void* stream) {
  if (M % 256 || N % 256 || K % kBK || !diag) return KFAMD_EINVAL;
  dim3 grid((M / 256) * (N / 256), 1), block(kThreads);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
  __bf16* c = static_cast<__bf16*>(C);
#define W4_DIAG(AB)                                                                                           \
  hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, 0, 0, 256, true, AB>), grid, block, 0, s, a, b, \
                     c, nullptr, nullptr, nullptr, M, N, K, (long long)K, (long long)K, (long long)N, 0LL, 0LL, 0LL,  \
                     0LL, 0LL, 1.0f, diag)
  if (abl == 0) W4_DIAG(0);
  else if (abl == 1) W4_DIAG(1);
  else if (abl == 2) W4_DIAG(2);
  else return KFAMD_EINVAL;
#undef W4_DIAG
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
#endif  // KFAMD_DIAG
