// gemm_bf16.hip — K1: bf16 GEMM on CDNA4 MFMA for MI355X (gfx950).
//
// SURVEY.md §2.7.2 K1 / §7.1 C. The reference has no GPU code at all; this kernel is
// the in-pod readiness op and the notebook-facing matmul of the MI355X build.
//
// Default fast path: gemm_bf16_w4.hip (4 waves x 128x128, one wave per SIMD, asm MFMA with AGPR
//   accumulators, buffer_load...lds into a 5-slot LDS ring). The 8-wave kernels below are the
//   previous fast paths (variants pipe / pipe_sched) and the fallback for >= 2 GiB panels.
// 8-wave path (gemm_nt_256): 256x256 output tile per 512-thread workgroup (8 waves, 2(M) x 4(N)),
//   BK = 64, one workgroup per CU (128 KiB LDS: two stages of A+B), operands staged HBM -> LDS with
//   global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip), XOR-swizzled LDS image (the swizzle is
//   applied to the per-lane SOURCE address because the DMA destination is lane-linear), counted
//   `s_waitcnt vmcnt(8)` so one K-tile stays in flight across the barrier, raw s_barrier (a
//   __syncthreads() would drain vmcnt to 0), XCD-aware bijective block remap + grouped tile order
//   so the 32 co-resident blocks of an XCD share A/B panels in that XCD's private 4 MiB L2.
//   MFMA: v_mfma_f32_16x16x32_bf16 with the operands swapped (B-tile as the MFMA "A"), which puts
//   4 consecutive output columns in each lane -> 8-byte packed bf16 stores in the fused epilogue
//   (alpha, bias, ReLU/GELU/SiLU, residual).
// Generic path (gemm_nt_128): 128x128 tile, 4 waves, register-staged and fully bounds-checked,
//   for any M/N/K/alignment (small or ragged shapes).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "kfamd_kernels.h"
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))
#define COMPILER_FENCE() asm volatile("" ::: "memory")

namespace {

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case KFAMD_ACT_RELU: return v > 0.f ? v : 0.f;
    case KFAMD_ACT_GELU_TANH: {
      const float u = 0.7978845608028654f * (v + 0.044715f * v * v * v);
      return 0.5f * v * (1.f + tanhf(u));
    }
    case KFAMD_ACT_SILU: return v / (1.f + __expf(-v));
    default: return v;
  }
}

// -------------------------------------------------------------------------------------------
// Fast path: 256 x 256 x 64, 8 waves, LDS-DMA double buffer.
// -------------------------------------------------------------------------------------------
constexpr int kBM = 256, kBN = 256, kBK = 64, kThreads = 512;
constexpr int kTileBytes = kBM * kBK * 2;          // 32 KiB per operand tile
constexpr int kStageBytes = 2 * kTileBytes;        // A + B
constexpr int kLdsBytes = 2 * kStageBytes;         // two stages = 128 KiB

// Bijective XCD remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"): blocks
// b, b+8, b+16, ... are dispatched to the same XCD; give each XCD a contiguous run of tile ids.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <int ACT, bool HAS_BIAS, bool HAS_RES>
__global__ __launch_bounds__(kThreads, 2) void gemm_nt_256(
    const __bf16* __restrict__ A, const __bf16* __restrict__ B, __bf16* __restrict__ C,
    const __bf16* __restrict__ bias, const __bf16* __restrict__ R, int M, int N, int K,
    long long lda, long long ldb, long long ldc, long long ldr, long long sa, long long sb,
    long long sc, long long sr, float alpha) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;

  // ---- tile selection: XCD remap, then grouped (GROUP_M rows of tiles) order -----------------
  const int tiles_m = M / kBM, tiles_n = N / kBN, nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  constexpr int kGroupM = 4;
  const int per_group = kGroupM * tiles_n;
  const int g = wg / per_group, first_m = g * kGroupM;
  const int gm = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (wg % per_group) % gm;
  const int tn = (wg % per_group) / gm;
  const int m0 = tm * kBM, n0 = tn * kBN;

  const long long bz = blockIdx.y;
  A += bz * sa;
  B += bz * sb;
  C += bz * sc;
  if (HAS_RES) R += bz * sr;

  // ---- per-lane LDS-DMA source pointers (4 A pieces + 4 B pieces of 1 KiB per wave) ---------
  // Piece p covers tile rows 8p..8p+7; lane i lands at LDS byte p*1024 + 16*i, i.e. row
  // 8p + (i>>3), swizzled chunk (i&7). It must fetch global chunk (i&7) ^ ((row>>1)&7).
  const char* a_src[4];
  const char* b_src[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = wid * 4 + j;
    const int row = p * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    a_src[j] = reinterpret_cast<const char*>(A + (long long)(m0 + row) * lda + chunk * 8);
    b_src[j] = reinterpret_cast<const char*>(B + (long long)(n0 + row) * ldb + chunk * 8);
  }

  auto stage = [&](int kt, int buf) {
    char* base = smem + buf * kStageBytes;
    const long long koff = (long long)kt * kBK * 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = wid * 4 + j;
      __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + koff), LDS_PTR(base + p * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = wid * 4 + j;
      __builtin_amdgcn_global_load_lds((const void*)(b_src[j] + koff), LDS_PTR(base + kTileBytes + p * 1024), 16, 0, 0);
    }
  };

  // ---- per-lane fragment read offsets (swizzle term is lane-constant, see header) -----------
  const int lr = lane & 15, lh = lane >> 4;
  const int sw = lh ^ (lr >> 1);
  const int off0 = lr * 128 + (sw << 4);
  const int off1 = lr * 128 + ((sw ^ 4) << 4);
  const int a_base = (wm * 128) * 128;
  const int b_base = kTileBytes + (wn * 64) * 128;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / kBK;
  stage(0, 0);
  if (nk > 1) stage(1, 1);

  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    COMPILER_FENCE();
    __builtin_amdgcn_s_barrier();
    COMPILER_FENCE();

    const char* sbuf = smem + (kt & 1) * kStageBytes;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int off = s ? off1 : off0;
      bf16x8 bf[4], af[8];
#pragma unroll
      for (int n = 0; n < 4; ++n)
        bf[n] = *reinterpret_cast<const bf16x8*>(sbuf + b_base + n * 16 * 128 + off);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(sbuf + a_base + i * 16 * 128 + off);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[n], af[i], acc[i][n], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }

    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    COMPILER_FENCE();
    __builtin_amdgcn_s_barrier();
    COMPILER_FENCE();
    if (kt + 2 < nk) stage(kt + 2, kt & 1);
  }

  // ---- fused epilogue: lane owns C[m][n..n+3] for each (i, n) fragment ----------------------
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + lr;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = n0 + wn * 64 + n * 16 + lh * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][n][r] * alpha;
      if (HAS_BIAS) {
        const bf16x4 bb = *reinterpret_cast<const bf16x4*>(bias + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)bb[r];
      }
      if (ACT != KFAMD_ACT_NONE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], ACT);
      }
      if (HAS_RES) {
        const bf16x4 rr = *reinterpret_cast<const bf16x4*>(R + (long long)m * ldr + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)rr[r];
      }
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (__bf16)v[r];
      *reinterpret_cast<bf16x4*>(C + (long long)m * ldc + col) = o;
    }
  }
}

// -------------------------------------------------------------------------------------------
// Fast path v2 (pipelined): the fragments of the NEXT k-substep are read from LDS while the
// MFMAs of the current one run (two register sets F0/F1), one barrier per K-tile, and the
// LDS-DMA of tile kt+2 is issued right after that barrier beside the MFMAs of substep 1.
//   per K-tile:  [ds_read F1(kt) || MFMA F0(kt)] -> lgkm(0), vmcnt(0) (tile kt+1 landed)
//                -> s_barrier -> [glds kt+2 -> buf(kt) || ds_read F0(kt+1) || MFMA F1(kt)]
// SCHED = 1 additionally pins a fine ds_read/glds : MFMA interleave with sched_group_barrier.
// -------------------------------------------------------------------------------------------
template <int ACT, bool HAS_BIAS, bool HAS_RES, int SCHED>
__global__ __launch_bounds__(kThreads, 2) void gemm_nt_256p(
    const __bf16* __restrict__ A, const __bf16* __restrict__ B, __bf16* __restrict__ C,
    const __bf16* __restrict__ bias, const __bf16* __restrict__ R, int M, int N, int K,
    long long lda, long long ldb, long long ldc, long long ldr, long long sa, long long sb,
    long long sc, long long sr, float alpha) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;

  const int tiles_m = M / kBM, tiles_n = N / kBN, nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  constexpr int kGroupM = 4;
  const int per_group = kGroupM * tiles_n;
  const int g = wg / per_group, first_m = g * kGroupM;
  const int gm = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (wg % per_group) % gm;
  const int tn = (wg % per_group) / gm;
  const int m0 = tm * kBM, n0 = tn * kBN;

  const long long bz = blockIdx.y;
  A += bz * sa;
  B += bz * sb;
  C += bz * sc;
  if (HAS_RES) R += bz * sr;

  const char* a_src[4];
  const char* b_src[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = wid * 4 + j;
    const int row = p * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    a_src[j] = reinterpret_cast<const char*>(A + (long long)(m0 + row) * lda + chunk * 8);
    b_src[j] = reinterpret_cast<const char*>(B + (long long)(n0 + row) * ldb + chunk * 8);
  }
  auto stage = [&](int kt, int buf) {
    char* base = smem + buf * kStageBytes;
    const long long koff = (long long)kt * kBK * 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = wid * 4 + j;
      __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + koff), LDS_PTR(base + p * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(b_src[j] + koff), LDS_PTR(base + kTileBytes + p * 1024), 16, 0, 0);
    }
  };

  const int lr = lane & 15, lh = lane >> 4;
  const int sw = lh ^ (lr >> 1);
  const int off0 = lr * 128 + (sw << 4);
  const int off1 = lr * 128 + ((sw ^ 4) << 4);
  const int a_base = (wm * 128) * 128;
  const int b_base = kTileBytes + (wn * 64) * 128;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 a0[8], b0[4], a1[8], b1[4];
  auto read_frags = [&](const char* sbuf, int off, bf16x8(&af)[8], bf16x8(&bf)[4]) {
#pragma unroll
    for (int n = 0; n < 4; ++n) bf[n] = *reinterpret_cast<const bf16x8*>(sbuf + b_base + n * 2048 + off);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sbuf + a_base + i * 2048 + off);
  };
  // SCHED: no s_setprio inside the cluster (it is a scheduling-region boundary that would keep
  // sched_group_barrier from interleaving the loads into the MFMA stream); one static raise.
  if (SCHED) __builtin_amdgcn_s_setprio(1);
  auto mfmas = [&](bf16x8(&af)[8], bf16x8(&bf)[4]) {
    if (!SCHED) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[n], af[i], acc[i][n], 0, 0, 0);
    if (!SCHED) __builtin_amdgcn_s_setprio(0);
  };

  const int nk = K / kBK;
  stage(0, 0);
  if (nk > 1) {
    stage(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  COMPILER_FENCE();
  __builtin_amdgcn_s_barrier();
  COMPILER_FENCE();
  read_frags(smem, off0, a0, b0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): nothing pending at the loop head

  // One K-tile of the steady state. STAGE: issue the LDS-DMA of tile kt+2; NEXT: read F0(kt+1).
  // sched_barrier(0) pins the s_barrier section so hipcc cannot hoist an MFMA cluster across it.
  auto body = [&](int kt, auto do_stage, auto do_next) {
    constexpr bool kStage = decltype(do_stage)::value;
    constexpr bool kNext = decltype(do_next)::value;
    const char* cur = smem + (kt & 1) * kStageBytes;
    const char* nxt = smem + ((kt + 1) & 1) * kStageBytes;
    read_frags(cur, off1, a1, b1);
    mfmas(a0, b0);
    if (SCHED) {
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 ds_read
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    // vmcnt(0) (tile kt+1 landed) + lgkmcnt(0) (F1 in registers, cur fully read). The builtin
    // form is visible to hipcc's waitcnt pass, so it will not re-wait for F1 behind F0(kt+1).
    __builtin_amdgcn_s_waitcnt(0x0070);
    COMPILER_FENCE();
    __builtin_amdgcn_s_barrier();
    COMPILER_FENCE();
    __builtin_amdgcn_sched_barrier(0);
    if (kStage) stage(kt + 2, kt & 1);
    if (kNext) read_frags(nxt, off0, a0, b0);
    mfmas(a1, b1);
    if (SCHED) {
      if (kStage) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 1);  // 1 glds (VMEM read)
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // 1 MFMA
        }
      }
      if (kNext) {
#pragma unroll
        for (int q = 0; q < 12; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // retire F0(kt+1) here (it had the whole F1 MFMA cluster to land) so the waitcnt pass does
    // not emit lgkmcnt(0) at the loop head, behind the freshly issued F1 reads
    if (kNext) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt/expcnt untouched
  };
  using T = std::integral_constant<bool, true>;
  using F = std::integral_constant<bool, false>;
  int kt = 0;
  for (; kt + 2 < nk; ++kt) body(kt, T{}, T{});
  if (kt + 1 < nk) {
    body(kt, F{}, T{});
    ++kt;
  }
  if (kt < nk) body(kt, F{}, F{});

#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + lr;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = n0 + wn * 64 + n * 16 + lh * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][n][r] * alpha;
      if (HAS_BIAS) {
        const bf16x4 bb = *reinterpret_cast<const bf16x4*>(bias + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)bb[r];
      }
      if (ACT != KFAMD_ACT_NONE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], ACT);
      }
      if (HAS_RES) {
        const bf16x4 rr = *reinterpret_cast<const bf16x4*>(R + (long long)m * ldr + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)rr[r];
      }
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (__bf16)v[r];
      *reinterpret_cast<bf16x4*>(C + (long long)m * ldc + col) = o;
    }
  }
}

// -------------------------------------------------------------------------------------------
// Generic path: 128 x 128 x 32, 4 waves (2x2, 64x64 each), register staging, full bounds checks.
// -------------------------------------------------------------------------------------------
constexpr int gBM = 128, gBN = 128, gBK = 32, gThreads = 256;
constexpr int gRowBytes = gBK * 2 + 16;  // 64 B of data + 16 B pad (breaks the 64-B row stride)

__device__ __forceinline__ bf16x8 load8(const __bf16* p, long long row, int rows, long long ld,
                                        int k, int K, bool vec_ok) {
  bf16x8 v;
  if (row < rows && vec_ok && k + 8 <= K) {
    v = *reinterpret_cast<const bf16x8*>(p + row * ld + k);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = (row < rows && k + e < K) ? p[row * ld + k + e] : (__bf16)0.f;
  }
  return v;
}

template <int ACT, bool HAS_BIAS, bool HAS_RES>
__global__ __launch_bounds__(gThreads, 2) void gemm_nt_128(
    const __bf16* __restrict__ A, const __bf16* __restrict__ B, __bf16* __restrict__ C,
    const __bf16* __restrict__ bias, const __bf16* __restrict__ R, int M, int N, int K,
    long long lda, long long ldb, long long ldc, long long ldr, long long sa, long long sb,
    long long sc, long long sr, float alpha, int vec_a, int vec_b) {
  __shared__ __attribute__((aligned(16))) char smem[(gBM + gBN) * gRowBytes];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.x * gBM, n0 = blockIdx.z * gBN;
  const long long bz = blockIdx.y;
  A += bz * sa;
  B += bz * sb;
  C += bz * sc;
  if (HAS_RES) R += bz * sr;

  const int lr = lane & 15, lh = lane >> 4;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // each thread stages 2 chunks of A and 2 of B (128 rows x 4 chunks of 8 elements each)
  bf16x8 ra[2], rb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + j * gThreads, row = c >> 2, kc = (c & 3) * 8;
      ra[j] = load8(A, (long long)(m0 + row), M, lda, k0 + kc, K, vec_a);
      rb[j] = load8(B, (long long)(n0 + row), N, ldb, k0 + kc, K, vec_b);
    }
  };
  auto swrite = [&]() {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + j * gThreads, row = c >> 2, kc = (c & 3);
      *reinterpret_cast<bf16x8*>(smem + row * gRowBytes + kc * 16) = ra[j];
      *reinterpret_cast<bf16x8*>(smem + (gBM + row) * gRowBytes + kc * 16) = rb[j];
    }
  };

  gload(0);
  for (int k0 = 0; k0 < K; k0 += gBK) {
    __syncthreads();
    swrite();
    __syncthreads();
    if (k0 + gBK < K) gload(k0 + gBK);  // next tile's loads in flight under this tile's MFMAs
    bf16x8 af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(smem + (wm * 64 + i * 16 + lr) * gRowBytes + lh * 16);
#pragma unroll
    for (int n = 0; n < 4; ++n)
      bf[n] = *reinterpret_cast<const bf16x8*>(smem + (gBM + wn * 64 + n * 16 + lr) * gRowBytes + lh * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[n], af[i], acc[i][n], 0, 0, 0);
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + lr;
    if (m >= M) continue;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = n0 + wn * 64 + n * 16 + lh * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cc = col + r;
        if (cc >= N) continue;
        float v = acc[i][n][r] * alpha;
        if (HAS_BIAS) v += (float)bias[cc];
        v = apply_act(v, ACT);
        if (HAS_RES) v += (float)R[(long long)m * ldr + cc];
        C[(long long)m * ldc + cc] = (__bf16)v;
      }
    }
  }
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }


#define KFAMD_COMMA ,
#define KFAMD_DISPATCH_EPI(KERNEL, EXTRA, GRID, BLOCK, STREAM, ...)                                      \
  do {                                                                                           \
    const bool hb = bias != nullptr, hr = R != nullptr;                                          \
    switch (act) {                                                                               \
      case KFAMD_ACT_NONE:                                                                       \
        if (hb && hr) hipLaunchKernelGGL((KERNEL<KFAMD_ACT_NONE, true, true EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);  \
        else if (hb) hipLaunchKernelGGL((KERNEL<KFAMD_ACT_NONE, true, false EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);  \
        else if (hr) hipLaunchKernelGGL((KERNEL<KFAMD_ACT_NONE, false, true EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);  \
        else hipLaunchKernelGGL((KERNEL<KFAMD_ACT_NONE, false, false EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);         \
        break;                                                                                   \
      case KFAMD_ACT_RELU:                                                                       \
        if (hb) hipLaunchKernelGGL((KERNEL<KFAMD_ACT_RELU, true, false EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);       \
        else hipLaunchKernelGGL((KERNEL<KFAMD_ACT_RELU, false, false EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);         \
        break;                                                                                   \
      case KFAMD_ACT_GELU_TANH:                                                                  \
        if (hb) hipLaunchKernelGGL((KERNEL<KFAMD_ACT_GELU_TANH, true, false EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);  \
        else hipLaunchKernelGGL((KERNEL<KFAMD_ACT_GELU_TANH, false, false EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);    \
        break;                                                                                   \
      case KFAMD_ACT_SILU:                                                                       \
        if (hb) hipLaunchKernelGGL((KERNEL<KFAMD_ACT_SILU, true, false EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);       \
        else hipLaunchKernelGGL((KERNEL<KFAMD_ACT_SILU, false, false EXTRA>), GRID, BLOCK, 0, STREAM, __VA_ARGS__);         \
        break;                                                                                   \
    }                                                                                            \
  } while (0)

}  // namespace

extern "C" int kfamd_w4_launch_nt(int bm, const void* A, const void* B, void* C, const void* bias, const void* R,
                                  void* Aux, int M, int N, int K, int batch, long long lda, long long ldb, long long ldc,
                                  long long ldr, long long sa, long long sb, long long sc, long long sr, float alpha,
                                  int act, void* stream);
extern "C" int kfamd_w4_launch_t(int la, int lb, int bm, const void* A, const void* B, void* C, const void* R, int M,
                                 int N, int K, int batch, long long lda, long long ldb, long long ldc, long long ldr,
                                 long long sa, long long sb, long long sc, long long sr, float alpha, void* stream);

namespace {
// w4 tile choice: the 128x128 tile (two blocks per CU) when the problem has at most half as many
// 256x256 tiles as MI355X has CUs, or a dimension below 256 (profiles/r1_gemm_w4s: 1024^3 92 -> 206
// TF, 2048^3 430 -> 848; at 3072^3, 144 tiles, the 256 tile still wins 980 : 904).
// 256-tile count up to which the 128 tile runs instead (2 blocks per CU); KFAMD_W4_TILE128_MAX
// overrides it for A/B runs (read once)
long long w4_tile128_max() {
  static const long long v = [] {
    const char* e = std::getenv("KFAMD_W4_TILE128_MAX");
    return e && *e ? std::atoll(e) : 128LL;
  }();
  return v;
}

int w4_tile(int M, int N, int batch) {
  const long long t256 = (long long)((M + 255) / 256) * ((N + 255) / 256) * batch;
  return (t256 <= w4_tile128_max() || M < 256 || N < 256) ? 128 : 256;
}
}  // namespace

extern "C" int kfamd_gemm_nt_bf16_variant(int variant, const void* A, const void* B, void* C,
                                          const void* bias, const void* R, int M, int N, int K,
                                          int batch, long long lda, long long ldb, long long ldc,
                                          long long ldr, long long stride_a, long long stride_b,
                                          long long stride_c, long long stride_r, float alpha,
                                          int act, void* stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0) return KFAMD_EINVAL;
  // variants: 0 auto, 1 fast (8-wave 256^2), 2 generic, 3 pipe, 4 pipe_sched, 6 w4, 9 w4s
  if (variant < 0 || variant > 9 || variant == 5 || variant == 7 || variant == 8) return KFAMD_EINVAL;
  if (lda < K || ldb < K || ldc < N || (R && ldr < N)) return KFAMD_EINVAL;
  if (act < KFAMD_ACT_NONE || act > KFAMD_ACT_SILU) return KFAMD_EINVAL;
  // activation + residual together is only compiled for act == NONE (residual = "add & norm"
  // style), keep the contract explicit.
  if (R && act != KFAMD_ACT_NONE) return KFAMD_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);

  // w4 / w4s (gemm_bf16_w4.hip): edge tiles in-kernel, so auto takes them for any M, N >= 128 with
  // K % 8 and 16-byte aligned operand rows (any N / output alignment: the epilogue's odd path);
  // anything else falls through to the r1 kernels below.
  if (variant == 6 || variant == 9)
    return kfamd_w4_launch_nt(variant == 6 ? 256 : 128, A, B, C, bias, R, nullptr, M, N, K, batch, lda, ldb, ldc, ldr,
                              stride_a, stride_b, stride_c, stride_r, alpha, act, stream);
  if (variant == 0) {
    const int rc = kfamd_w4_launch_nt(w4_tile(M, N, batch), A, B, C, bias, R, nullptr, M, N, K, batch, lda, ldb, ldc,
                                      ldr, stride_a, stride_b, stride_c, stride_r, alpha, act, stream);
    if (rc >= 0) return rc;  // launched (or a HIP launch error)
  }
  const bool shapes_ok = (M % kBM == 0) && (N % kBN == 0) && (K % kBK == 0);
  const bool align_ok = aligned16(A) && aligned16(B) && aligned16(C) && (lda % 8 == 0) &&
                        (ldb % 8 == 0) && (ldc % 4 == 0) && (stride_a % 8 == 0) &&
                        (stride_b % 8 == 0) && (stride_c % 4 == 0) &&
                        (!bias || (reinterpret_cast<uintptr_t>(bias) & 7) == 0) &&
                        (!R || ((reinterpret_cast<uintptr_t>(R) & 7) == 0 && ldr % 4 == 0 && stride_r % 4 == 0));
  bool fast = shapes_ok && align_ok;
  if (variant == 1 || variant >= 3) {
    if (!shapes_ok) return KFAMD_EINVAL;
    if (!align_ok) return KFAMD_EALIGN;
    fast = true;
  } else if (variant == 2) {
    fast = false;
  }

  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
  __bf16* c = static_cast<__bf16*>(C);
  const __bf16* bs = static_cast<const __bf16*>(bias);
  const __bf16* r = static_cast<const __bf16*>(R);
  if (fast) {
    dim3 grid((M / kBM) * (N / kBN), batch), block(kThreads);
    if (variant == 0 || variant == 4) {  // 8 waves: pipelined + pinned interleave
      KFAMD_DISPATCH_EPI(gemm_nt_256p, KFAMD_COMMA 1, grid, block, s, a, b, c, bs, r, M, N, K, lda, ldb, ldc,
                         ldr, stride_a, stride_b, stride_c, stride_r, alpha);
    } else if (variant == 3) {
      KFAMD_DISPATCH_EPI(gemm_nt_256p, KFAMD_COMMA 0, grid, block, s, a, b, c, bs, r, M, N, K, lda, ldb, ldc,
                         ldr, stride_a, stride_b, stride_c, stride_r, alpha);
    } else {
      KFAMD_DISPATCH_EPI(gemm_nt_256, , grid, block, s, a, b, c, bs, r, M, N, K, lda, ldb, ldc, ldr,
                         stride_a, stride_b, stride_c, stride_r, alpha);
    }
  } else {
    const int vec_a = aligned16(A) && (lda % 8 == 0) && (stride_a % 8 == 0);
    const int vec_b = aligned16(B) && (ldb % 8 == 0) && (stride_b % 8 == 0);
    dim3 grid((M + gBM - 1) / gBM, batch, (N + gBN - 1) / gBN), block(gThreads);
    KFAMD_DISPATCH_EPI(gemm_nt_128, , grid, block, s, a, b, c, bs, r, M, N, K, lda, ldb, ldc, ldr,
                       stride_a, stride_b, stride_c, stride_r, alpha, vec_a, vec_b);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

extern "C" int kfamd_gemm_nt_bf16(const void* A, const void* B, void* C, const void* bias,
                                  const void* R, int M, int N, int K, int batch, long long lda,
                                  long long ldb, long long ldc, long long ldr, long long stride_a,
                                  long long stride_b, long long stride_c, long long stride_r,
                                  float alpha, int act, void* stream) {
  return kfamd_gemm_nt_bf16_variant(0, A, B, C, bias, R, M, N, K, batch, lda, ldb, ldc, ldr,
                                    stride_a, stride_b, stride_c, stride_r, alpha, act, stream);
}

// Layout-general entry (kfamd_kernels.h): la/lb select K-contiguous (0) or k-major (1) operands;
// Aux = pre-activation second output (NT only). Only the w4 template serves the transposed layouts:
// an unsupported shape returns KFAMD_EINVAL / KFAMD_EALIGN (callers fall back, never silently).
extern "C" int kfamd_gemm_bf16_ex(int la, int lb, const void* A, const void* B, void* C, const void* bias,
                                  const void* R, void* Aux, int M, int N, int K, int batch, long long lda,
                                  long long ldb, long long ldc, long long ldr, long long stride_a, long long stride_b,
                                  long long stride_c, long long stride_r, float alpha, int act, void* stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0) return KFAMD_EINVAL;
  if (la < 0 || la > 1 || lb < 0 || lb > 1 || act < KFAMD_ACT_NONE || act > KFAMD_ACT_SILU) return KFAMD_EINVAL;
  if (la == 0 && lb == 0) {
    if (!Aux)
      return kfamd_gemm_nt_bf16_variant(0, A, B, C, bias, R, M, N, K, batch, lda, ldb, ldc, ldr, stride_a, stride_b,
                                        stride_c, stride_r, alpha, act, stream);
    return kfamd_w4_launch_nt(w4_tile(M, N, batch), A, B, C, bias, R, Aux, M, N, K, batch, lda, ldb, ldc, ldr,
                              stride_a, stride_b, stride_c, stride_r, alpha, act, stream);
  }
  if (bias || Aux || act != KFAMD_ACT_NONE) return KFAMD_EINVAL;
  return kfamd_w4_launch_t(la, lb, w4_tile(M, N, batch), A, B, C, R, M, N, K, batch, lda, ldb, ldc, ldr, stride_a,
                           stride_b, stride_c, stride_r, alpha, stream);
}
