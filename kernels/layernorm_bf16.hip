// layernorm_bf16.hip — K2: LayerNorm / RMSNorm (bf16 I/O, fp32 statistics) for MI355X (gfx950).
//
// SURVEY.md §2.7.2 K2. Memory-bound: the target is the HBM3E roof (~6.3 TB/s achievable).
//  * Fast path: one 64-lane wave per row, the whole row resident in VGPRs (hidden = 512*VPL,
//    VPL in {1,2,3,4,5,6,8,10,12,16} -> hidden 512..8192), 16-byte bf16x8 loads/stores,
//    exact two-pass mean/variance from registers (no re-read of HBM), wave-only reductions
//    (no LDS, no barriers), 4 rows per 256-thread workgroup -> rows/4 workgroups (>>256 CUs).
//  * Generic path: one workgroup per row, any hidden size, LDS block reduction.
//  * Backward: dx per row (same wave-per-row structure), dgamma/dbeta by a column-strip
//    partial-sum kernel + a finalize kernel (deterministic, no float atomics).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>
#include "kfamd_kernels.h"
#include "wave_ops.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

using kfw::wave_sum;  // DPP + permlane swaps, no LDS round trips (wave_ops.h)

// Block reduction for the generic (one workgroup per row) kernels. 256 threads = 4 waves.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) t += red[i];
  return t;
}

// W bf16 per lane per unit: 8 (16-byte loads, hidden = 512 * VPL) or 4 (8-byte loads, hidden =
// 256 * VPL for the widths 256 / 768 / 1280 that are not multiples of 512)
// PF: gamma / beta are loaded with the row, before the reductions (their L2 latency overlaps the
// statistics instead of following them), at the cost of their registers: used at VPL 16 (hidden
// 8192), +3.5 % at 8192 x 8192 and +4.6 % at 32768 x 8192; at VPL <= 8 it measured 1-5 % slower
// (profiles/r5j_ln_ab)
template <int VPL, bool RMS, int W = 8, bool PF = false>
__global__ __launch_bounds__(256) void norm_fwd_wave(const __bf16* __restrict__ x,
                                                    const __bf16* __restrict__ gamma,
                                                    const __bf16* __restrict__ beta,
                                                    __bf16* __restrict__ y, float* __restrict__ mean_out,
                                                    float* __restrict__ rstd_out, int rows, float eps) {
  using vec_t = __bf16 __attribute__((ext_vector_type(W)));
  constexpr int H = VPL * 64 * W;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;  // wave-uniform; no barriers below
  const vec_t* xr = reinterpret_cast<const vec_t*>(x + (long long)row * H);
  // hidden 8192: the row stays resident as packed bf16 (64 data VGPRs instead of 128 fp32), so 4
  // waves per SIMD instead of 2 keep more rows in flight: +6-8 % at 8192 / 32768 x 8192. At
  // hidden <= 4096 the fp32 copy already allows 4+ waves and re-widening measured 0-8 % slower
  // (profiles/r2_ln_occupancy), so there the compiler keeps the widened values.
  constexpr bool kRepack = VPL >= 16;
  vec_t v[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) v[j] = __builtin_nontemporal_load(&xr[j * 64 + lane]);  // streamed once
  const vec_t* g8 = reinterpret_cast<const vec_t*>(gamma);
  const vec_t* b8 = reinterpret_cast<const vec_t*>(beta);
  vec_t gpre[PF ? VPL : 1], bpre[PF ? VPL : 1];
  if constexpr (PF) {
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      gpre[j] = g8[j * 64 + lane];
      if (!RMS && beta) bpre[j] = b8[j * 64 + lane];
    }
  }
  float mean = 0.f;
  if (!RMS) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j)
#pragma unroll
      for (int e = 0; e < W; ++e) s += (float)v[j][e];
    mean = wave_sum(s) * (1.f / H);
  }
  // an empty asm "redefines" the packed row before each later pass, so the compiler widens it again
  // instead of keeping the first pass's fp32 copies live (which is what costs the registers)
  if constexpr (kRepack)
#pragma unroll
    for (int j = 0; j < VPL; ++j) asm volatile("" : "+v"(v[j]));
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j)
#pragma unroll
    for (int e = 0; e < W; ++e) {
      const float d = (float)v[j][e] - mean;
      ss += d * d;
    }
  const float rstd = rsqrtf(wave_sum(ss) * (1.f / H) + eps);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
  if constexpr (kRepack)
#pragma unroll
    for (int j = 0; j < VPL; ++j) asm volatile("" : "+v"(v[j]));
  vec_t* yr = reinterpret_cast<vec_t*>(y + (long long)row * H);
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const vec_t g = PF ? gpre[PF ? j : 0] : g8[j * 64 + lane];
    vec_t b;
    if (!RMS && beta) b = PF ? bpre[PF ? j : 0] : b8[j * 64 + lane];
    vec_t o;
#pragma unroll
    for (int e = 0; e < W; ++e) {
      float r = ((float)v[j][e] - mean) * rstd * (float)g[e];
      if (!RMS && beta) r += (float)b[e];
      o[e] = (__bf16)r;
    }
    __builtin_nontemporal_store(o, &yr[j * 64 + lane]);
  }
}

// Streaming forward (hidden = 512 * VPL): a grid of resident waves, each sweeping rows wave,
// wave + nw, ... with the NEXT row in flight while this one is reduced and stored (no
// generation-by-generation load / compute / store phases, no tail of late rows). VPL <= 8 double-
// buffers the row (the next row's loads go out before this row's statistics); ROLL (VPL 16, where a
// second buffer does not fit) reloads each 16-B piece for the next row right after its output is
// stored. gamma / beta sit in LDS (one copy per workgroup): their reads wait on lgkmcnt, so no vmcnt
// wait for them also waits for the prefetched row.
template <int VPL, bool RMS, bool ROLL = false>
__global__ __launch_bounds__(256) void norm_fwd_stream(const __bf16* __restrict__ x,
                                                      const __bf16* __restrict__ gamma,
                                                      const __bf16* __restrict__ beta,
                                                      __bf16* __restrict__ y, float* __restrict__ mean_out,
                                                      float* __restrict__ rstd_out, int rows, float eps) {
  constexpr int H = VPL * 512;
  __shared__ bf16x8 sg[H / 8], sb[RMS ? 1 : H / 8];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < H / 8; i += 256) {
    sg[i] = reinterpret_cast<const bf16x8*>(gamma)[i];
    if (!RMS) sb[i] = beta ? reinterpret_cast<const bf16x8*>(beta)[i] : bf16x8{};
  }
  __syncthreads();
  const int nw = gridDim.x * 4;
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // wave-uniform; no barriers below
  auto load = [&](bf16x8 (&v)[VPL], int r) __attribute__((always_inline)) {
    const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (long long)r * H);
#pragma unroll
    for (int j = 0; j < VPL; ++j) v[j] = __builtin_nontemporal_load(&xr[j * 64 + lane]);
  };
  // the empty asms "redefine" the packed row before each pass, so the compiler widens it per pass
  // instead of keeping fp32 copies of both buffers live
  auto opaque = [&](bf16x8 (&v)[VPL]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < VPL; ++j) asm volatile("" : "+v"(v[j]));
  };
  auto finish = [&](bf16x8 (&v)[VPL], int r, int rnext) __attribute__((always_inline)) {
    opaque(v);
    float mean = 0.f;
    if (!RMS) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < VPL; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) s += (float)v[j][e];
      mean = wave_sum(s) * (1.f / H);
    }
    opaque(v);
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = (float)v[j][e] - mean;
        ss += d * d;
      }
    const float rstd = rsqrtf(wave_sum(ss) * (1.f / H) + eps);
    if (lane == 0) {
      if (mean_out) mean_out[r] = mean;
      if (rstd_out) rstd_out[r] = rstd;
    }
    opaque(v);
    bf16x8* yr = reinterpret_cast<bf16x8*>(y + (long long)r * H);
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const bf16x8 g = sg[j * 64 + lane];
      bf16x8 b{};
      if (!RMS) b = sb[j * 64 + lane];
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = ((float)v[j][e] - mean) * rstd * (float)g[e];
        if (!RMS) t += (float)b[e];
        o[e] = (__bf16)t;
      }
      __builtin_nontemporal_store(o, &yr[j * 64 + lane]);
      if (ROLL && rnext >= 0)
        v[j] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(x + (long long)rnext * H) + j * 64 + lane);
    }
  };
  if constexpr (ROLL) {
    bf16x8 va[VPL];
    load(va, row);
    while (true) {
      const int rn = row + nw;
      finish(va, row, rn < rows ? rn : -1);
      if (rn >= rows) break;
      row = rn;
    }
  } else {
    bf16x8 va[VPL], vb[VPL];
    load(va, row);
    while (true) {
      const int r1 = row + nw;
      if (r1 < rows) load(vb, r1);
      finish(va, row, -1);
      if (r1 >= rows) break;
      const int r2 = r1 + nw;
      if (r2 < rows) load(va, r2);
      finish(vb, r1, -1);
      if (r2 >= rows) break;
      row = r2;
    }
  }
}

template <bool RMS>
__global__ __launch_bounds__(256) void norm_fwd_block(const __bf16* __restrict__ x,
                                                     const __bf16* __restrict__ gamma,
                                                     const __bf16* __restrict__ beta,
                                                     __bf16* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int hidden, float eps) {
  __shared__ float red[4];
  const long long row = blockIdx.x;
  const __bf16* xr = x + row * hidden;
  float mean = 0.f;
  if (!RMS) {
    float s = 0.f;
    for (int i = threadIdx.x; i < hidden; i += 256) s += (float)xr[i];
    mean = block_sum(s, red) / hidden;
  }
  float ss = 0.f;
  for (int i = threadIdx.x; i < hidden; i += 256) {
    const float d = (float)xr[i] - mean;
    ss += d * d;
  }
  const float rstd = rsqrtf(block_sum(ss, red) / hidden + eps);
  if (threadIdx.x == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
  __bf16* yr = y + row * hidden;
  for (int i = threadIdx.x; i < hidden; i += 256) {
    float r = ((float)xr[i] - mean) * rstd * (float)gamma[i];
    if (!RMS && beta) r += (float)beta[i];
    yr[i] = (__bf16)r;
  }
}

// ---- backward: dx ---------------------------------------------------------------------------
template <int VPL, int W = 8>  // W as in norm_fwd_wave
__global__ __launch_bounds__(256) void ln_bwd_dx_wave(const __bf16* __restrict__ dy,
                                                     const __bf16* __restrict__ x,
                                                     const __bf16* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     const __bf16* __restrict__ dres,
                                                     __bf16* __restrict__ dx, int rows) {
  using vec_t = __bf16 __attribute__((ext_vector_type(W)));
  constexpr int H = VPL * 64 * W;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const vec_t* xr = reinterpret_cast<const vec_t*>(x + (long long)row * H);
  const vec_t* dyr = reinterpret_cast<const vec_t*>(dy + (long long)row * H);
  const vec_t* g8 = reinterpret_cast<const vec_t*>(gamma);
  const float mu = mean[row], rs = rstd[row];
  vec_t* dxr = reinterpret_cast<vec_t*>(dx + (long long)row * H);
  // dres: the residual stream's own gradient, added in the store (one pass instead of an add kernel)
  const vec_t* rr = dres ? reinterpret_cast<const vec_t*>(dres + (long long)row * H) : nullptr;
  if constexpr (VPL < 16) {
    // the widened row (xhat, gamma * dy) stays in registers between the passes
    float xh[VPL][W], gd[VPL][W];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const vec_t xv = xr[j * 64 + lane], dv = dyr[j * 64 + lane], gv = g8[j * 64 + lane];
#pragma unroll
      for (int e = 0; e < W; ++e) {
        xh[j][e] = ((float)xv[e] - mu) * rs;
        gd[j][e] = (float)dv[e] * (float)gv[e];
        s1 += gd[j][e] * xh[j][e];
        s2 += gd[j][e];
      }
    }
    const float c1 = wave_sum(s1) * (1.f / H), c2 = wave_sum(s2) * (1.f / H);
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      vec_t o;
      if (rr) {
        const vec_t rv = rr[j * 64 + lane];
#pragma unroll
        for (int e = 0; e < W; ++e) o[e] = (__bf16)(fmaf(rs, gd[j][e] - xh[j][e] * c1 - c2, (float)rv[e]));
      } else {
#pragma unroll
        for (int e = 0; e < W; ++e) o[e] = (__bf16)(rs * (gd[j][e] - xh[j][e] * c1 - c2));
      }
      dxr[j * 64 + lane] = o;
    }
  } else {
    // hidden 8192: x and dy stay packed bf16 between the two passes (8 VGPRs per 8 columns
    // instead of 16 fp32: 2 waves per SIMD instead of 1); the second pass widens them again and
    // re-reads gamma, which every row shares (L2-resident)
    vec_t xv[VPL], dv[VPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      xv[j] = xr[j * 64 + lane];
      dv[j] = dyr[j * 64 + lane];
    }
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const vec_t gv = g8[j * 64 + lane];
#pragma unroll
      for (int e = 0; e < W; ++e) {
        const float xh = ((float)xv[j][e] - mu) * rs, gd = (float)dv[j][e] * (float)gv[e];
        s1 += gd * xh;
        s2 += gd;
      }
    }
    const float c1 = wave_sum(s1) * (1.f / H), c2 = wave_sum(s2) * (1.f / H);
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      asm volatile("" : "+v"(xv[j]));  // widen again below rather than keep pass one's fp32 values
      asm volatile("" : "+v"(dv[j]));
    }
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const vec_t gv = g8[j * 64 + lane];
      vec_t rv = {};
      if (rr) rv = rr[j * 64 + lane];
      vec_t o;
#pragma unroll
      for (int e = 0; e < W; ++e) {
        const float xh = ((float)xv[j][e] - mu) * rs, gd = (float)dv[j][e] * (float)gv[e];
        o[e] = (__bf16)(fmaf(rs, gd - xh * c1 - c2, (float)rv[e]));
      }
      dxr[j * 64 + lane] = o;
    }
  }
}

__global__ __launch_bounds__(256) void ln_bwd_dx_block(const __bf16* __restrict__ dy,
                                                      const __bf16* __restrict__ x,
                                                      const __bf16* __restrict__ gamma,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ rstd,
                                                      const __bf16* __restrict__ dres,
                                                      __bf16* __restrict__ dx, int hidden) {
  __shared__ float red[4];
  const long long row = blockIdx.x;
  const float mu = mean[row], rs = rstd[row];
  const __bf16* xr = x + row * hidden;
  const __bf16* dyr = dy + row * hidden;
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < hidden; i += 256) {
    const float xh = ((float)xr[i] - mu) * rs, g = (float)dyr[i] * (float)gamma[i];
    s1 += g * xh;
    s2 += g;
  }
  const float c1 = block_sum(s1, red) / hidden;
  const float c2 = block_sum(s2, red) / hidden;
  __bf16* dxr = dx + row * hidden;
  for (int i = threadIdx.x; i < hidden; i += 256) {
    const float xh = ((float)xr[i] - mu) * rs, g = (float)dyr[i] * (float)gamma[i];
    dxr[i] = (__bf16)(fmaf(rs, g - xh * c1 - c2, dres ? (float)dres[row * hidden + i] : 0.f));
  }
}

// ---- backward, fused: dx and the dgamma / dbeta partials in one pass -----------------------------
// kFusedWaves waves per block walk a contiguous chunk of rows, one row per wave at a time, as
// ln_bwd_dx_wave does; each lane also keeps its columns' sums of dy * xhat and dy in registers
// across its rows, so dy and x are read once for all three gradients (the split path reads them a
// second time in ln_bwd_dgb_partial: 16.9 of 46.8 us per gpt-1b LayerNorm backward,
// profiles/r5zc_ln_bwd). At the end the block's waves meet in LDS, 64 W columns at a time, summed
// in wave order (deterministic), and one [2][hidden] partial row per block goes to the workspace for
// ln_bwd_dgb_finalize. Widths up to 32 columns per lane (hidden <= 2048 at W = 8): the sums take
// 2 x VPL x W registers beside the row.
constexpr int kFusedWaves = 8, kFusedBlocks = 256;

template <int VPL, int W>
__global__ __launch_bounds__(64 * kFusedWaves) void ln_bwd_fused(const __bf16* __restrict__ dy,
                                                                const __bf16* __restrict__ x,
                                                                const __bf16* __restrict__ gamma,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                const __bf16* __restrict__ dres,
                                                                __bf16* __restrict__ dx, float* __restrict__ ws,
                                                                int rows, int rpb) {
  using vec_t = __bf16 __attribute__((ext_vector_type(W)));
  constexpr int H = VPL * 64 * W, CW = 64 * W;
  static_assert(VPL * W <= 32, "ln_bwd_fused: at most 32 columns per lane");
  __shared__ __attribute__((aligned(16))) float red[kFusedWaves][CW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  const vec_t* g8 = reinterpret_cast<const vec_t*>(gamma);
  float ag[VPL][W], ab[VPL][W];
#pragma unroll
  for (int j = 0; j < VPL; ++j)
#pragma unroll
    for (int e = 0; e < W; ++e) ag[j][e] = ab[j][e] = 0.f;
  for (int row = r0 + wv; row < r1; row += kFusedWaves) {
    const vec_t* xr = reinterpret_cast<const vec_t*>(x + (long long)row * H);
    const vec_t* dyr = reinterpret_cast<const vec_t*>(dy + (long long)row * H);
    const float mu = mean[row], rs = rstd[row];
    float xh[VPL][W], gd[VPL][W];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const vec_t xv = xr[j * 64 + lane], dv = dyr[j * 64 + lane], gv = g8[j * 64 + lane];
#pragma unroll
      for (int e = 0; e < W; ++e) {
        const float d = (float)dv[e];
        xh[j][e] = ((float)xv[e] - mu) * rs;
        gd[j][e] = d * (float)gv[e];
        s1 += gd[j][e] * xh[j][e];
        s2 += gd[j][e];
        ag[j][e] = fmaf(d, xh[j][e], ag[j][e]);
        ab[j][e] += d;
      }
    }
    const float c1 = wave_sum(s1) * (1.f / H), c2 = wave_sum(s2) * (1.f / H);
    vec_t* dxr = reinterpret_cast<vec_t*>(dx + (long long)row * H);
    const vec_t* rr = dres ? reinterpret_cast<const vec_t*>(dres + (long long)row * H) : nullptr;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      vec_t rv = {};
      if (rr) rv = rr[j * 64 + lane];
      vec_t o;
#pragma unroll
      for (int e = 0; e < W; ++e) o[e] = (__bf16)(fmaf(rs, gd[j][e] - xh[j][e] * c1 - c2, (float)rv[e]));
      dxr[j * 64 + lane] = o;
    }
  }
  float* og = ws + (long long)blockIdx.x * H;
  float* ob = ws + ((long long)gridDim.x + blockIdx.x) * H;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
#pragma unroll
    for (int which = 0; which < 2; ++which) {
#pragma unroll
      for (int e = 0; e < W; ++e) red[wv][lane * W + e] = which ? ab[j][e] : ag[j][e];
      __syncthreads();
      for (int c = threadIdx.x; c < CW; c += 64 * kFusedWaves) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kFusedWaves; ++w) t += red[w][c];
        (which ? ob : og)[j * CW + c] = t;
      }
      __syncthreads();
    }
  }
}

// ---- backward: dgamma / dbeta partials over row chunks ---------------------------------------
// Block: 64 column lanes x 4 row lanes; each column lane owns one column of the strip, so a
// wave reads 64 consecutive bf16 (128 B) of one row per step; partials land in ws[chunk][col].
constexpr int kColsPerBlock = 64, kRowLanes = 4, kRowsPerChunk = 64;

__global__ __launch_bounds__(256) void ln_bwd_dgb_partial(const __bf16* __restrict__ dy,
                                                         const __bf16* __restrict__ x,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd,
                                                         float* __restrict__ ws, int rows, int hidden) {
  __shared__ float sg[kRowLanes][kColsPerBlock], sb[kRowLanes][kColsPerBlock];
  const int c = blockIdx.x * kColsPerBlock + (threadIdx.x & (kColsPerBlock - 1));
  const int rl = threadIdx.x / kColsPerBlock;
  const int chunk = blockIdx.y;
  const int r0 = chunk * kRowsPerChunk, r1 = min(rows, r0 + kRowsPerChunk);
  float dg = 0.f, db = 0.f;
  if (c < hidden) {
    for (int r = r0 + rl; r < r1; r += kRowLanes) {
      const float d = (float)dy[(long long)r * hidden + c];
      const float xh = ((float)x[(long long)r * hidden + c] - mean[r]) * rstd[r];
      dg += d * xh;
      db += d;
    }
  }
  sg[rl][threadIdx.x & (kColsPerBlock - 1)] = dg;
  sb[rl][threadIdx.x & (kColsPerBlock - 1)] = db;
  __syncthreads();
  if (rl == 0 && c < hidden) {
    float tg = 0.f, tb = 0.f;
#pragma unroll
    for (int i = 0; i < kRowLanes; ++i) {
      tg += sg[i][threadIdx.x];
      tb += sb[i][threadIdx.x];
    }
    const long long nch = gridDim.y;
    ws[(long long)chunk * hidden + c] = tg;
    ws[(nch + chunk) * (long long)hidden + c] = tb;
  }
}

// Sum of the chunk partials: 64 columns x 4 chunk lanes per block, each lane's loads independent (8 in
// flight), then a 4-way LDS reduce. (One thread per column summing all chunks in order was latency
// bound: 37.6 us for 128 chunks x 2048 columns on 8 blocks, profiles/r4_train_trace.)
// OB: write bf16 (the parameter dtype), else fp32
template <bool OB>
__global__ __launch_bounds__(256) void ln_bwd_dgb_finalize(const float* __restrict__ ws, void* __restrict__ dgamma,
                                                          void* __restrict__ dbeta, int nchunks, int hidden) {
  __shared__ float sg[kRowLanes][kColsPerBlock], sb[kRowLanes][kColsPerBlock];
  const int cl = threadIdx.x & (kColsPerBlock - 1), kl = threadIdx.x / kColsPerBlock;
  const int c = blockIdx.x * kColsPerBlock + cl;
  float tg = 0.f, tb = 0.f;
  if (c < hidden) {
#pragma unroll 8
    for (int k = kl; k < nchunks; k += kRowLanes) {
      tg += ws[(long long)k * hidden + c];
      tb += ws[(long long)(nchunks + k) * hidden + c];
    }
  }
  sg[kl][cl] = tg;
  sb[kl][cl] = tb;
  __syncthreads();
  if (kl == 0 && c < hidden) {
    tg = sg[0][cl] + sg[1][cl] + sg[2][cl] + sg[3][cl];
    tb = sb[0][cl] + sb[1][cl] + sb[2][cl] + sb[3][cl];
    if (OB) {
      if (dgamma) static_cast<__bf16*>(dgamma)[c] = (__bf16)tg;
      if (dbeta) static_cast<__bf16*>(dbeta)[c] = (__bf16)tb;
    } else {
      if (dgamma) static_cast<float*>(dgamma)[c] = tg;
      if (dbeta) static_cast<float*>(dbeta)[c] = tb;
    }
  }
}

inline bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline bool a8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }

// wave-per-row widths: hidden = 512 * VPL, the powers of two plus the common model widths
// 1536 / 2560 / 3072 / 5120 / 6144 (VPL 3, 5, 6, 10, 12); anything else takes the block kernel
inline int vpl_for(int hidden) {
  if (hidden % 512) return 0;
  switch (hidden / 512) {
    case 1: case 2: case 3: case 4: case 5: case 6: case 8: case 10: case 12: case 16: return hidden / 512;
    default: return 0;
  }
}

#define KFAMD_FOR_EACH_VPL(X) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(10) X(12) X(16)

// hidden = 256 * {1, 3, 5} with 8-byte rows (e.g. 768, the BERT-base / GPT-2 width)
inline int vpl4_for(int hidden) {
  if (hidden % 256 || hidden % 512 == 0) return 0;
  const int v = hidden / 256;
  return (v == 1 || v == 3 || v == 5) ? v : 0;
}

// rows the device holds at once for a one-wave-per-row kernel of 256-thread blocks (occupancy x CUs
// x 4 waves), per kernel, queried once
template <auto kernel>
long long resident_rows() {
  static const long long n = [] {
    int occ = 0, cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, 256, 0) != hipSuccess) occ = 1;
    return 4LL * (occ > 0 ? occ : 1) * (cus > 0 ? cus : 256);
  }();
  return n;
}

// Forward launch policy (profiles/r5_ln, kbench A/B runs on one box): the one-shot wave-per-row
// kernel, except when its grid would take between one and two generations of resident waves (of the
// plain kernel: the gamma / beta prefetch variant holds half as many): there
// the second generation's load / compute / store phases do not overlap the first's, and the
// streaming kernel (resident waves, next row in flight) is faster: 8192 x 4096 24.1 -> 22.1 us
// (6.06 TB/s). At one generation (8192 x 2048: equal) or four (16384 x 4096: 46.3 vs 47.4 us) the
// one-shot kernel stays. Hidden 8192 streams with the rolling reload up to two generations
// (4096 x 8192 26.6 -> 24.7 us, 8192 x 8192 48.3-49.3 -> 47.7 us) and is 2.5-6 % slower beyond, where
// the one-shot kernel with gamma / beta prefetched runs (32768 x 8192: 178.8 us, 6.0 TB/s).
template <bool RMS>
int norm_fwd(const void* x, const void* gamma, const void* beta, void* y, float* mean, float* rstd,
             int rows, int hidden, float eps, void* stream) {
  if (!x || !gamma || !y || rows <= 0 || hidden <= 0) return KFAMD_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* xp = static_cast<const __bf16*>(x);
  const __bf16* gp = static_cast<const __bf16*>(gamma);
  const __bf16* bp = static_cast<const __bf16*>(beta);
  __bf16* yp = static_cast<__bf16*>(y);
  const int vpl = vpl_for(hidden);
  const bool vec = vpl && a16(x) && a16(gamma) && a16(y) && (!beta || a16(beta));
  if (vec) {
    dim3 grid((rows + 3) / 4), block(256);
    switch (vpl) {
#define KFAMD_NORM_FWD_CASE(V)                                                                                   \
  case V:                                                                                                      \
    if (V == 16 && rows <= 2 * resident_rows<norm_fwd_wave<V, RMS>>()) {                        \
      const long long waves = resident_rows<norm_fwd_stream<16, RMS, true>>();                                  \
      const long long rpw = (rows + waves - 1) / waves;                                                        \
      hipLaunchKernelGGL((norm_fwd_stream<16, RMS, true>), dim3((int)((rows + 4 * rpw - 1) / (4 * rpw))),     \
                         block, 0, s, xp, gp, bp, yp, mean, rstd, rows, eps);                                  \
    } else if (V <= 8 && rows > resident_rows<norm_fwd_wave<V, RMS>>() &&                       \
        rows <= 2 * resident_rows<norm_fwd_wave<V, RMS>>()) {                                       \
      const long long waves = resident_rows<norm_fwd_stream<V <= 8 ? V : 8, RMS>>();                             \
      const long long rpw = (rows + waves - 1) / waves; /* rows per wave, the same for every wave */          \
      hipLaunchKernelGGL((norm_fwd_stream<V <= 8 ? V : 8, RMS>), dim3((int)((rows + 4 * rpw - 1) / (4 * rpw))), \
                         block, 0, s, xp, gp, bp, yp, mean, rstd, rows, eps);                                  \
    } else {                                                                                                   \
      hipLaunchKernelGGL((norm_fwd_wave<V, RMS, 8, V == 16>), grid, block, 0, s, xp, gp, bp, yp, mean, rstd, rows, eps); \
    }                                                                                                          \
    break;
      KFAMD_FOR_EACH_VPL(KFAMD_NORM_FWD_CASE)
#undef KFAMD_NORM_FWD_CASE
    }
  } else if (const int v4 = vpl4_for(hidden); v4 && a8(x) && a8(gamma) && a8(y) && (!beta || a8(beta))) {
    dim3 grid((rows + 3) / 4), block(256);
    switch (v4) {
      case 1: hipLaunchKernelGGL((norm_fwd_wave<1, RMS, 4>), grid, block, 0, s, xp, gp, bp, yp, mean, rstd, rows, eps); break;
      case 3: hipLaunchKernelGGL((norm_fwd_wave<3, RMS, 4>), grid, block, 0, s, xp, gp, bp, yp, mean, rstd, rows, eps); break;
      case 5: hipLaunchKernelGGL((norm_fwd_wave<5, RMS, 4>), grid, block, 0, s, xp, gp, bp, yp, mean, rstd, rows, eps); break;
    }
  } else {
    hipLaunchKernelGGL((norm_fwd_block<RMS>), dim3(rows), dim3(256), 0, s, xp, gp, bp, yp, mean, rstd, hidden, eps);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

}  // namespace

extern "C" int kfamd_layernorm_fwd_bf16(const void* x, const void* gamma, const void* beta, void* y,
                                        float* mean, float* rstd, int rows, int hidden, float eps,
                                        void* stream) {
  return norm_fwd<false>(x, gamma, beta, y, mean, rstd, rows, hidden, eps, stream);
}

extern "C" int kfamd_rmsnorm_fwd_bf16(const void* x, const void* gamma, void* y, float* rstd,
                                      int rows, int hidden, float eps, void* stream) {
  return norm_fwd<true>(x, gamma, nullptr, y, nullptr, rstd, rows, hidden, eps, stream);
}

extern "C" long long kfamd_layernorm_bwd_workspace(int rows, int hidden) {
  const long long nch = (rows + kRowsPerChunk - 1) / kRowsPerChunk;
  return 2LL * (nch > kFusedBlocks ? nch : kFusedBlocks) * hidden * (long long)sizeof(float);
}

// dgamma / dbeta: fp32, or bf16 (the parameter dtype) when dgb_bf16; sums accumulate in fp32 either way.
// dres (optional, same layout as dx): dx = dres + the LayerNorm input gradient — the pre-norm
// residual stream's two gradient contributions summed in the dx store.
extern "C" int kfamd_layernorm_bwd_bf16_v3(const void* dy, const void* dres, const void* x, const void* gamma,
                                           const float* mean, const float* rstd, void* dx, void* dgamma, void* dbeta,
                                           int dgb_bf16, float* workspace, int rows, int hidden, void* stream) {
  if (!dy || !x || !gamma || !mean || !rstd || !dx || rows <= 0 || hidden <= 0) return KFAMD_EINVAL;
  if (dres == dx) return KFAMD_EINVAL;
  if ((dgamma || dbeta) && !workspace) return KFAMD_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* dyp = static_cast<const __bf16*>(dy);
  const __bf16* xp = static_cast<const __bf16*>(x);
  const __bf16* gp = static_cast<const __bf16*>(gamma);
  __bf16* dxp = static_cast<__bf16*>(dx);
  const __bf16* rp = static_cast<const __bf16*>(dres);
  const int vpl = vpl_for(hidden);
  const bool vec = vpl && a16(dy) && a16(x) && a16(gamma) && a16(dx) && (!dres || a16(dres));
  const int v4 = vec ? 0 : vpl4_for(hidden);
  const bool vec4 = v4 && a8(dy) && a8(x) && a8(gamma) && a8(dx) && (!dres || a8(dres));
  // dx + dgamma / dbeta in one pass (ln_bwd_fused) where the sums fit beside the row: hidden <= 2048
  // (W = 8) or 256 x {1, 3, 5} (W = 4); KFAMD_LN_BWD_SPLIT=1 forces the split path (A/B runs)
  static const bool force_split = [] { const char* e = getenv("KFAMD_LN_BWD_SPLIT"); return e && *e == '1'; }();
  const bool fused = (dgamma || dbeta) && !force_split && ((vec && vpl <= 4) || vec4);
  if (fused) {
    int nblk = (rows + kFusedWaves - 1) / kFusedWaves;
    if (nblk > kFusedBlocks) nblk = kFusedBlocks;
    const int rpb = (rows + nblk - 1) / nblk;
    nblk = (rows + rpb - 1) / rpb;
    const dim3 grid(nblk), block(64 * kFusedWaves);
    const int key = vec ? vpl : 100 + v4;
    switch (key) {
#define KFAMD_LN_FUSED(K, V, WW) \
  case K: hipLaunchKernelGGL((ln_bwd_fused<V, WW>), grid, block, 0, s, dyp, xp, gp, mean, rstd, rp, dxp, workspace, rows, rpb); break;
      KFAMD_LN_FUSED(1, 1, 8) KFAMD_LN_FUSED(2, 2, 8) KFAMD_LN_FUSED(3, 3, 8) KFAMD_LN_FUSED(4, 4, 8)
      KFAMD_LN_FUSED(101, 1, 4) KFAMD_LN_FUSED(103, 3, 4) KFAMD_LN_FUSED(105, 5, 4)
#undef KFAMD_LN_FUSED
    }
    const dim3 fg((hidden + kColsPerBlock - 1) / kColsPerBlock);
    if (dgb_bf16) hipLaunchKernelGGL(ln_bwd_dgb_finalize<true>, fg, dim3(256), 0, s, workspace, dgamma, dbeta, nblk, hidden);
    else hipLaunchKernelGGL(ln_bwd_dgb_finalize<false>, fg, dim3(256), 0, s, workspace, dgamma, dbeta, nblk, hidden);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
  }
  if (vec) {
    dim3 grid((rows + 3) / 4), block(256);
    switch (vpl) {
#define KFAMD_LN_BWD_CASE(V) \
  case V: hipLaunchKernelGGL((ln_bwd_dx_wave<V>), grid, block, 0, s, dyp, xp, gp, mean, rstd, rp, dxp, rows); break;
      KFAMD_FOR_EACH_VPL(KFAMD_LN_BWD_CASE)
#undef KFAMD_LN_BWD_CASE
    }
  } else if (vec4) {
    dim3 grid((rows + 3) / 4), block(256);
    switch (v4) {
      case 1: hipLaunchKernelGGL((ln_bwd_dx_wave<1, 4>), grid, block, 0, s, dyp, xp, gp, mean, rstd, rp, dxp, rows); break;
      case 3: hipLaunchKernelGGL((ln_bwd_dx_wave<3, 4>), grid, block, 0, s, dyp, xp, gp, mean, rstd, rp, dxp, rows); break;
      case 5: hipLaunchKernelGGL((ln_bwd_dx_wave<5, 4>), grid, block, 0, s, dyp, xp, gp, mean, rstd, rp, dxp, rows); break;
    }
  } else {
    hipLaunchKernelGGL(ln_bwd_dx_block, dim3(rows), dim3(256), 0, s, dyp, xp, gp, mean, rstd, rp, dxp, hidden);
  }
  if (dgamma || dbeta) {
    const int nch = (rows + kRowsPerChunk - 1) / kRowsPerChunk;
    dim3 grid((hidden + kColsPerBlock - 1) / kColsPerBlock, nch);
    hipLaunchKernelGGL(ln_bwd_dgb_partial, grid, dim3(256), 0, s, dyp, xp, mean, rstd, workspace, rows, hidden);
    const dim3 fg((hidden + kColsPerBlock - 1) / kColsPerBlock);
    if (dgb_bf16) hipLaunchKernelGGL(ln_bwd_dgb_finalize<true>, fg, dim3(256), 0, s, workspace, dgamma, dbeta, nch, hidden);
    else hipLaunchKernelGGL(ln_bwd_dgb_finalize<false>, fg, dim3(256), 0, s, workspace, dgamma, dbeta, nch, hidden);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

extern "C" int kfamd_layernorm_bwd_bf16_v2(const void* dy, const void* x, const void* gamma, const float* mean,
                                           const float* rstd, void* dx, void* dgamma, void* dbeta, int dgb_bf16,
                                           float* workspace, int rows, int hidden, void* stream) {
  return kfamd_layernorm_bwd_bf16_v3(dy, nullptr, x, gamma, mean, rstd, dx, dgamma, dbeta, dgb_bf16, workspace, rows,
                                     hidden, stream);
}

extern "C" int kfamd_layernorm_bwd_bf16(const void* dy, const void* x, const void* gamma, const float* mean,
                                        const float* rstd, void* dx, float* dgamma, float* dbeta, float* workspace,
                                        int rows, int hidden, void* stream) {
  return kfamd_layernorm_bwd_bf16_v2(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, 0, workspace, rows, hidden, stream);
}
