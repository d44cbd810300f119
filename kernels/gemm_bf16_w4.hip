// gemm_bf16_w4.hip — K1 variant "w4" in the forward ("NT") layout: C = act(alpha * A B^T + bias)
// (+ R), A [M][K], B [N][K], on the 4-wave template of gemm_w4.h (256x256 tile "w4" or 128x128
// "w4s"), with in-kernel edge tiles (any M, N >= the tile, N % 8, K % 8) and an optional second
// output Aux = the pre-activation (gelu/silu backward without recomputing the GEMM).
// The backward layouts live in gemm_bf16_w4_t.hip; the kernels of each activation in
// tu/w4_nt_<act>.hip and stream-K in gemm_bf16_w4_sk.hip (separate translation units that the
// library build compiles in parallel). This file: the dispatcher, split-K partials + reduce, diag.
//
// History kept out of this file: profiles/r1_gemm_w4 (register placement: asm MFMA with tied AGPR
// accumulators, buffer_load..lds with SGPR row offsets), profiles/r1_gemm_w4c (5-slot ring),
// profiles/r2_gemm_knobs + r2_gemm_stalls (knob A/Bs, issue-stall diagnosis).
#include "gemm_w4.h"

using namespace kfw4;

#ifndef KFAMD_DIAG  // (the diagnostic library holds only the stamped kernel below)
extern "C" {
int kfw4_nt_none(int, const void*, const void*, void*, const void*, const void*, void*, int, int, int, int, long long,
                 long long, long long, long long, long long, long long, long long, long long, float, void*);
int kfw4_nt_relu(int, const void*, const void*, void*, const void*, const void*, void*, int, int, int, int, long long,
                 long long, long long, long long, long long, long long, long long, long long, float, void*);
int kfw4_nt_gelu(int, const void*, const void*, void*, const void*, const void*, void*, int, int, int, int, long long,
                 long long, long long, long long, long long, long long, long long, long long, float, void*);
int kfw4_nt_silu(int, const void*, const void*, void*, const void*, const void*, void*, int, int, int, int, long long,
                 long long, long long, long long, long long, long long, long long, long long, float, void*);
}

// NT layout on the w4 template; bm = 256 ("w4") or 128 ("w4s"). Shapes/alignment: check_shape.
// One translation unit per activation (tu/w4_nt_<act>.hip, launcher gemm_w4_nt.h).
extern "C" int kfamd_w4_launch_nt(int bm, const void* A, const void* B, void* C, const void* bias, const void* R,
                                  void* Aux, int M, int N, int K, int batch, long long lda, long long ldb, long long ldc,
                                  long long ldr, long long sa, long long sb, long long sc, long long sr, float alpha,
                                  int act, void* stream) {
  switch (act) {
    case KFAMD_ACT_NONE:
      return kfw4_nt_none(bm, A, B, C, bias, R, Aux, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, stream);
    case KFAMD_ACT_RELU:
      return kfw4_nt_relu(bm, A, B, C, bias, R, Aux, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, stream);
    case KFAMD_ACT_GELU_TANH:
      return kfw4_nt_gelu(bm, A, B, C, bias, R, Aux, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, stream);
    case KFAMD_ACT_SILU:
      return kfw4_nt_silu(bm, A, B, C, bias, R, Aux, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, stream);
    default:
      return KFAMD_EINVAL;
  }
}

// Split-K partials on the 128x128 w4s tile (NT layout): W[splits][batch][M][N] fp32, K range
// [z*kper, (z+1)*kper) per split (kper % 64 == 0); the epilogue runs in kfamd_splitk_reduce.
extern "C" int kfamd_w4_splitk_nt(const void* A, const void* B, float* W, int M, int N, int K, int batch, int splits,
                                  int kper, long long lda, long long ldb, long long sa, long long sb, void* stream) {
  const int rc = check_shape(0, 0, 128, A, B, W, nullptr, nullptr, nullptr, M, N, K, lda, ldb, N, 0, sa, sb, 0, 0);
  if (rc != KFAMD_OK) return rc;
  if (splits < 1 || kper < kBK || kper % kBK || (long long)kper * (splits - 1) >= K || !W || N % 8) return KFAMD_EINVAL;
  if (reinterpret_cast<uintptr_t>(W) & 15) return KFAMD_EALIGN;
  dim3 grid(((M + 127) / 128) * ((N + 127) / 128), batch, splits), block(kThreads);
  hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, 0, 0, 128, true>), grid, block, 0,
                     reinterpret_cast<hipStream_t>(stream), static_cast<const __bf16*>(A), static_cast<const __bf16*>(B),
                     nullptr, nullptr, nullptr, nullptr, M, N, K, lda, ldb, 0LL, 0LL, sa, sb, 0LL, 0LL, 1.0f, nullptr, W,
                     kper);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

namespace {

// C[b][m][n] = epilogue(alpha * sum_z W[z][b][m][n]); 8 columns per thread (two float4 per split).
template <int ACT, bool HAS_BIAS, bool HAS_RES, bool HAS_AUX>
__global__ void __launch_bounds__(256) splitk_reduce(const float* __restrict__ W, __bf16* C, const __bf16* __restrict__ bias,
                                                     const __bf16* R, __bf16* __restrict__ Aux, int M, int N, int batch,
                                                     int splits, long long ldc, long long ldr, long long sc, long long sr,
                                                     float alpha) {
  const long long n8 = N / 8, per = (long long)M * n8;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= per * batch) return;
  const long long b = t / per, rem = t - b * per;
  const int m = (int)(rem / n8), col = (int)(rem - (long long)m * n8) * 8;
  const long long mn = (long long)M * N, zs = mn * batch;
  const float* w = W + b * mn + (long long)m * N + col;
  f32x4 lo = *reinterpret_cast<const f32x4*>(w), hi = *reinterpret_cast<const f32x4*>(w + 4);
  for (int z = 1; z < splits; ++z) {
    lo += *reinterpret_cast<const f32x4*>(w + z * zs);
    hi += *reinterpret_cast<const f32x4*>(w + z * zs + 4);
  }
  float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] *= alpha;
  if (HAS_BIAS) {
    const bf16x8 bb = *reinterpret_cast<const bf16x8*>(bias + col);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += (float)bb[r];
  }
  const long long coff = b * sc + (long long)m * ldc + col;
  if (HAS_AUX) {
    bf16x8 p;
#pragma unroll
    for (int r = 0; r < 8; ++r) p[r] = (__bf16)v[r];
    *reinterpret_cast<bf16x8*>(Aux + coff) = p;
  }
  if (ACT != KFAMD_ACT_NONE) {
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = act_fn(v[r], ACT);
  }
  if (HAS_RES) {
    const bf16x8 rr = *reinterpret_cast<const bf16x8*>(R + b * sr + (long long)m * ldr + col);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += (float)rr[r];
  }
  bf16x8 o;
#pragma unroll
  for (int r = 0; r < 8; ++r) o[r] = (__bf16)v[r];
  *reinterpret_cast<bf16x8*>(C + coff) = o;
}

}  // namespace

// Split-K epilogue over W[splits][batch][M][N] (kfamd_w4_splitk_*): alpha, bias, activation (Aux =
// the pre-activation), residual (R may alias C) into bf16 C. N % 8, 16-B aligned C/R/Aux/bias rows.
extern "C" int kfamd_splitk_reduce(const float* W, void* C, const void* bias, const void* R, void* Aux, int M, int N,
                                   int batch, int splits, long long ldc, long long ldr, long long sc, long long sr,
                                   float alpha, int act, void* stream) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!W || !C || M <= 0 || N <= 0 || batch <= 0 || splits < 1 || N % 8 || ldc % 8 || sc % 8) return KFAMD_EINVAL;
  if (!al16(W) || !al16(C) || (bias && !al16(bias)) || (Aux && !al16(Aux))) return KFAMD_EINVAL;
  if (R && (!al16(R) || ldr % 8 || sr % 8)) return KFAMD_EINVAL;
  if (Aux && (act == KFAMD_ACT_NONE || R)) return KFAMD_EINVAL;
  if (R && act != KFAMD_ACT_NONE) return KFAMD_EINVAL;
  const long long total = (long long)batch * M * (N / 8);
  dim3 grid((unsigned)((total + 255) / 256)), block(256);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  __bf16* c = static_cast<__bf16*>(C);
  const __bf16* bs = static_cast<const __bf16*>(bias);
  const __bf16* r = static_cast<const __bf16*>(R);
  __bf16* x = static_cast<__bf16*>(Aux);
  const bool hb = bias != nullptr, hr = R != nullptr, hx = Aux != nullptr;
#define SK(ACTV, HB, HR, HX)                                                                                       \
  hipLaunchKernelGGL((splitk_reduce<ACTV, HB, HR, HX>), grid, block, 0, s, W, c, bs, r, x, M, N, batch, splits, ldc, \
                     ldr, sc, sr, alpha)
#define SK_ACT(ACTV)                                         \
  if (hx) {                                                  \
    if (hb) SK(ACTV, true, false, true);                     \
    else SK(ACTV, false, false, true);                       \
  } else {                                                   \
    if (hb) SK(ACTV, true, false, false);                    \
    else SK(ACTV, false, false, false);                      \
  }
  switch (act) {
    case KFAMD_ACT_NONE:
      if (hb && hr) SK(KFAMD_ACT_NONE, true, true, false);
      else if (hb) SK(KFAMD_ACT_NONE, true, false, false);
      else if (hr) SK(KFAMD_ACT_NONE, false, true, false);
      else SK(KFAMD_ACT_NONE, false, false, false);
      break;
    case KFAMD_ACT_RELU:
      if (hx) return KFAMD_EINVAL;
      if (hb) SK(KFAMD_ACT_RELU, true, false, false);
      else SK(KFAMD_ACT_RELU, false, false, false);
      break;
    case KFAMD_ACT_GELU_TANH:
      SK_ACT(KFAMD_ACT_GELU_TANH);
      break;
    case KFAMD_ACT_SILU:
      SK_ACT(KFAMD_ACT_SILU);
      break;
    default:
      return KFAMD_EINVAL;
  }
#undef SK_ACT
#undef SK
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

#endif  // !KFAMD_DIAG

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
  hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, 0, 0, 256, false, true, AB>), grid, block, 0, s, a, b, \
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
