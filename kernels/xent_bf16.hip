// xent_bf16.hip — softmax cross-entropy over a vocabulary row, for the LM head of the in-notebook
// model (kubeflow_rm_amd.ops.cross_entropy): the bf16 logits are never widened to an fp32 copy.
//   forward:  lse[r] = log sum_j exp(x[r][j]);  loss[r] = lse[r] - x[r][t[r]]  (0 where t = ignore)
//   backward: dx[r][j] = (exp(x[r][j] - lse[r]) - [j == t[r]]) * scale,  scale = *g / *count read on
//             the device (no host sync for the upstream gradient or the number of counted rows)
// One 256-thread block per row; 16-B loads (8 bf16 per lane per step), the row max / sum meet
// through wave shuffles and LDS. The forward reads the logits once, the backward reads them once
// and writes the gradient once: ~1.5x the logits' bytes in total, against widen + softmax forward +
// softmax backward + narrow (~7x) for torch's fp32 path.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "kfamd_kernels.h"
#include "wave_ops.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kThreads = 256, kWaves = kThreads / 64;

using kfw::wave_max;  // DPP + permlane swaps (wave_ops.h)
using kfw::wave_sum;

// row max and sum of exp(x - max) over [0, V), online (one pass); result in every thread
__device__ __forceinline__ void row_stats(const __bf16* __restrict__ x, int V, bool vec, float& mx, float& sm) {
  __shared__ float red_m[kWaves], red_s[kWaves];
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  float m = -INFINITY, s = 0.f;
  const int nv = vec ? V / 8 : 0;  // rows off the 16-B grid (V or ld % 8) take the element loop
  for (int i = t; i < nv; i += kThreads) {
    const bf16x8 v = reinterpret_cast<const bf16x8*>(x)[i];
    float vm = (float)v[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) vm = fmaxf(vm, (float)v[k]);
    if (vm > m) { s *= __expf(m - vm); m = vm; }
#pragma unroll
    for (int k = 0; k < 8; ++k) s += __expf((float)v[k] - m);
  }
  for (int j = nv * 8 + t; j < V; j += kThreads) {
    const float v = (float)x[j];
    if (v > m) { s *= __expf(m - v); m = v; }
    s += __expf(v - m);
  }
  // combine (m, s) pairs: wave, then across the block's waves
  float wm = wave_max(m);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - wm);
  s = wave_sum(s);
  if (l == 0) { red_m[w] = wm; red_s[w] = s; }
  __syncthreads();
  float bm = red_m[0];
#pragma unroll
  for (int k = 1; k < kWaves; ++k) bm = fmaxf(bm, red_m[k]);
  float bs = 0.f;
#pragma unroll
  for (int k = 0; k < kWaves; ++k) bs += red_m[k] == -INFINITY ? 0.f : red_s[k] * __expf(red_m[k] - bm);
  mx = bm;
  sm = bs;
}

__global__ __launch_bounds__(kThreads) void xent_fwd(const __bf16* __restrict__ logits, long long ld,
                                                     const long long* __restrict__ target, float* __restrict__ loss,
                                                     float* __restrict__ lse, int V, long long ignore, int vec) {
  const long long r = blockIdx.x;
  const __bf16* x = logits + r * ld;
  float mx, sm;
  row_stats(x, V, vec != 0, mx, sm);
  if (threadIdx.x == 0) {
    const float l = mx + __logf(sm);
    lse[r] = l;
    const long long tg = target[r];
    loss[r] = (tg == ignore || tg < 0 || tg >= V) ? 0.f : l - (float)x[tg];
  }
}

__global__ __launch_bounds__(kThreads) void xent_bwd(const __bf16* __restrict__ logits, long long ld,
                                                     const long long* __restrict__ target,
                                                     const float* __restrict__ lse, __bf16* __restrict__ grad,
                                                     long long ldg, int V, long long ignore,
                                                     const float* __restrict__ g, const float* __restrict__ count,
                                                     int vec) {
  const long long r = blockIdx.x;
  const __bf16* x = logits + r * ld;
  __bf16* d = grad + r * ldg;
  const long long tg = target[r];
  const bool skip = tg == ignore || tg < 0 || tg >= V;
  const float c = *count;
  const float scale = (skip || c <= 0.f) ? 0.f : *g / c;
  const float l = lse[r];
  const int nv = vec ? V / 8 : 0;
  for (int i = threadIdx.x; i < nv; i += kThreads) {
    const bf16x8 v = reinterpret_cast<const bf16x8*>(x)[i];
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int j = i * 8 + k;
      o[k] = (__bf16)((__expf((float)v[k] - l) - (j == tg ? 1.f : 0.f)) * scale);
    }
    reinterpret_cast<bf16x8*>(d)[i] = o;
  }
  for (int j = nv * 8 + threadIdx.x; j < V; j += kThreads)
    d[j] = (__bf16)((__expf((float)x[j] - l) - (j == tg ? 1.f : 0.f)) * scale);
}

}  // namespace

// rows x V bf16 logits (row stride ld; 16-B rows take the vector loop), int64 targets -> per-row loss and lse (fp32)
extern "C" int kfamd_xent_fwd_bf16(const void* logits, long long ld, const long long* target, float* loss, float* lse,
                                   int rows, int V, long long ignore_index, void* stream) {
  if (!logits || !target || !loss || !lse || rows <= 0 || V <= 0 || ld < V) return KFAMD_EINVAL;
  const int vec = !(reinterpret_cast<uintptr_t>(logits) & 15) && ld % 8 == 0;
  hipLaunchKernelGGL(xent_fwd, dim3(rows), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const __bf16*>(logits), ld, target, loss, lse, V, ignore_index, vec);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

// dlogits = (softmax - onehot) * (*g / *count), written to grad (row stride ldg)
extern "C" int kfamd_xent_bwd_bf16(const void* logits, long long ld, const long long* target, const float* lse,
                                   void* grad, long long ldg, int rows, int V, long long ignore_index, const float* g,
                                   const float* count, void* stream) {
  if (!logits || !target || !lse || !grad || !g || !count || rows <= 0 || V <= 0 || ld < V || ldg < V)
    return KFAMD_EINVAL;
  const int vec = !((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(grad)) & 15) && ld % 8 == 0 &&
                  ldg % 8 == 0;
  hipLaunchKernelGGL(xent_bwd, dim3(rows), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const __bf16*>(logits), ld, target, lse, static_cast<__bf16*>(grad), ldg, V,
                     ignore_index, g, count, vec);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
