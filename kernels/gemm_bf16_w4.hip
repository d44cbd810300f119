// gemm_bf16_w4.hip — K1 variant "w4": 256x256x64 tile on FOUR waves (2x2), 128x128 per wave,
// one wave per SIMD with the full 512-register file (256 accumulators in AGPRs).
//
// Why (MI355X_MICROARCH.md 'DVFS give-back' + cdna_hip_programming.md §5.4 rule 28): on random
// data a bf16 GEMM runs clock-limited (~1.9 GHz), and what raises the held clock for the same
// MFMAs is less energy per MFMA — fewer LDS read bytes and fewer VALU. LDS fragment reads per
// K-tile scale with sum over waves of (wave_M + wave_N): 8 waves of 128x64 read 192 KiB per
// CU per K-tile, 4 waves of 128x128 read 128 KiB (-33 %), with the same MFMA count
// (128 x v_mfma_f32_16x16x32_bf16 per wave per K-tile) and the same DMA bytes.
//
// Register placement (the first version of this kernel lost 30 % to it — profiles/r1_gemm_w4):
//  * accumulators: the MFMA is issued from inline asm with a tied "+a" accumulator, so each of
//    the 64 f32x4 accumulators lives in ONE fixed AGPR quad for the whole K loop (the builtin
//    form let the allocator pick dst != srcC and rotate the loop-carried values through 300
//    v_accvgpr moves per K-tile);
//  * operand staging: buffer_load_dwordx4 ... lds (LDS-DMA) from a wave-uniform buffer resource
//    with the per-piece row offset in an SGPR, so the 32 staging addresses cost 4 VGPRs instead
//    of 32 (64-bit global pointers), keeping the VGPR side (128 fragment registers) unspilled.
// Pipeline: two LDS stages (128 KiB), DMA of tile kt+2 issued right after the single per-K-tile
// barrier, fragments of the next k-substep read while the current substep's MFMAs run (two
// register sets), and the ds_read / DMA : MFMA interleave written out in source order, pinned
// with sched_barrier (an asm MFMA is invisible to sched_group_barrier's classes).
// Negative results kept out of this file (profiles/r1_gemm_w4/README.md): BK = 32 in a 5-stage
// ring (deeper DMA lookahead) fetches half 128-B lines per row and lost 10-35 %.
// Same operand swap / epilogue / swizzle / XCD-remap conventions as gemm_bf16.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "kfamd_kernels.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))
#define COMPILER_FENCE() asm volatile("" ::: "memory")
#define PIN() __builtin_amdgcn_sched_barrier(0)

namespace {

constexpr int kBM = 256, kBN = 256, kBK = 64, kThreads = 256;
constexpr int kTileBytes = kBM * kBK * 2;    // 32 KiB per operand tile
constexpr int kStageBytes = 2 * kTileBytes;  // A + B
constexpr int kLdsBytes = 2 * kStageBytes;   // 128 KiB
constexpr int kRsrcWord3 = 0x00020000;       // gfx9 raw buffer: 32-bit dword format, no swizzle

__device__ __forceinline__ float act_fn(float v, int act) {
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

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ void mfma(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

template <int ACT, bool HAS_BIAS, bool HAS_RES>
__global__ __attribute__((amdgpu_flat_work_group_size(kThreads, kThreads), amdgpu_waves_per_eu(1, 1)))
void gemm_nt_256w4(const __bf16* __restrict__ A, const __bf16* __restrict__ B, __bf16* __restrict__ C,
                   const __bf16* __restrict__ bias, const __bf16* __restrict__ R, int M, int N, int K,
                   long long lda, long long ldb, long long ldc, long long ldr, long long sa, long long sb,
                   long long sc, long long sr, float alpha) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;

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
  A += bz * sa + (long long)m0 * lda;
  B += bz * sb + (long long)n0 * ldb;
  C += bz * sc;
  if (HAS_RES) R += bz * sr;
  // wave-uniform buffer resources over this block's 256-row panels (launcher checks < 2 GiB)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7fffffff, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7fffffff, kRsrcWord3);

  // 32 one-KiB pieces (8 rows each) per operand tile, 8 per wave: piece p = wid*8 + j covers rows
  // 8p..8p+7; lane i lands at LDS p*1024 + 16*i (row 8p + (i>>3), swizzled chunk (i&7)) and must
  // fetch global chunk (i&7) ^ ((row>>1)&7) = (i&7) ^ ((4*(j&1) + (i>>4)) & 7): two lane offsets
  // per operand (j even / odd); the row offset 8j*ld is wave-uniform (SGPR soffset).
  const int lrow = wid * 64 + (lane >> 3);
  int va[2], vb[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int chunk = (lane & 7) ^ ((4 * par + (lane >> 4)) & 7);
    va[par] = (int)(((long long)lrow * lda + chunk * 8) * 2);
    vb[par] = (int)(((long long)lrow * ldb + chunk * 8) * 2);
  }
  const int rowstep_a = (int)(8 * lda * 2), rowstep_b = (int)(8 * ldb * 2);
  auto stage_piece = [&](int kt, int buf, int j) {
    char* base = smem + buf * kStageBytes + (wid * 8 + j) * 1024;
    const int koff = kt * kBK * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, LDS_PTR(base), 16, va[j & 1], j * rowstep_a + koff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, LDS_PTR(base + kTileBytes), 16, vb[j & 1], j * rowstep_b + koff, 0, 0);
  };

  const int lr = lane & 15, lh = lane >> 4;
  const int sw = lh ^ (lr >> 1);
  const int off0 = lr * 128 + (sw << 4);
  const int off1 = lr * 128 + ((sw ^ 4) << 4);
  const int a_base = (wm * 128) * 128;
  const int b_base = kTileBytes + (wn * 128) * 128;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 a0[8], b0[8], a1[8], b1[8];
  // fragment q of a set: q < 8 -> B fragment q, q >= 8 -> A fragment q-8
  auto read_frag = [&](const char* sbuf, int off, bf16x8(&af)[8], bf16x8(&bf)[8], int q) {
    if (q < 8) bf[q] = *reinterpret_cast<const bf16x8*>(sbuf + b_base + q * 2048 + off);
    else af[q - 8] = *reinterpret_cast<const bf16x8*>(sbuf + a_base + (q - 8) * 2048 + off);
  };

  const int nk = K / kBK;
#pragma unroll
  for (int j = 0; j < 8; ++j) stage_piece(0, 0, j);
  if (nk > 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) stage_piece(1, 1, j);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  COMPILER_FENCE();
  __builtin_amdgcn_s_barrier();
  COMPILER_FENCE();
#pragma unroll
  for (int q = 0; q < 16; ++q) read_frag(smem, off0, a0, b0, q);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  PIN();
  __builtin_amdgcn_s_setprio(1);

  // The reads (and DMA) of a substep go out in its FIRST half, 1 ds_read (+1 DMA) per 2 MFMAs, so
  // the lgkmcnt(0) / vmcnt(0) at the substep's end finds them landed: with one wave per SIMD no
  // other wave's MFMAs cover a read still in flight there (issuing them evenly over the substep
  // left the last read ~4 MFMAs before its wait).
  auto body = [&](int kt, auto do_stage, auto do_next) {
    constexpr bool kStage = decltype(do_stage)::value;
    constexpr bool kNext = decltype(do_next)::value;
    const char* cur = smem + (kt & 1) * kStageBytes;
    const char* nxt = smem + ((kt + 1) & 1) * kStageBytes;
    // substep 0: MFMAs on F0 while F1 (substep 1 of this tile) streams in
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      if (q < 16) read_frag(cur, off1, a1, b1, q);
      PIN();
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int idx = q * 2 + t, i = idx >> 3, n = idx & 7;
        mfma(acc[i][n], b0[n], a0[i]);
      }
      PIN();
    }
    // tile kt+1 landed (vmcnt(0)) and F1 / this buffer fully read (lgkmcnt(0)), then one barrier
    __builtin_amdgcn_s_waitcnt(0x0070);
    COMPILER_FENCE();
    __builtin_amdgcn_s_barrier();
    COMPILER_FENCE();
    PIN();
    // substep 1: MFMAs on F1; beside them the DMA of tile kt+2 into the buffer just released and
    // the reads of F0(kt+1)
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      if (kStage && q < 16) {
        char* base = smem + (kt & 1) * kStageBytes + (wid * 8 + (q >> 1)) * 1024;
        const int j = q >> 1, koff = (kt + 2) * kBK * 2;
        if (q & 1)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, LDS_PTR(base + kTileBytes), 16, vb[j & 1], j * rowstep_b + koff, 0, 0);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, LDS_PTR(base), 16, va[j & 1], j * rowstep_a + koff, 0, 0);
      }
      if (kNext && q < 16) read_frag(nxt, off0, a0, b0, q);
      PIN();
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int idx = q * 2 + t, i = idx >> 3, n = idx & 7;
        mfma(acc[i][n], b1[n], a1[i]);
      }
      PIN();
    }
    if (kNext) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): F0(kt+1) in registers
    PIN();
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
  __builtin_amdgcn_s_setprio(0);
  // the asm MFMAs are opaque to the hazard recognizer: cover the MFMA -> v_accvgpr_read latency
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + lr;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int col = n0 + wn * 128 + n * 16 + lh * 4;
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
        for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], ACT);
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

}  // namespace

// Caller (kfamd_gemm_nt_bf16_variant) has validated shapes (M,N % 256, K % 64) and alignment;
// the buffer offsets are 32-bit, so a block's 256-row panel must span < 2 GiB.
extern "C" int kfamd_gemm_nt_bf16_w4_launch(const void* A, const void* B, void* C, const void* bias, const void* R,
                                            int M, int N, int K, int batch, long long lda, long long ldb, long long ldc,
                                            long long ldr, long long sa, long long sb, long long sc, long long sr,
                                            float alpha, int act, void* stream) {
  if ((long long)kBM * lda * 2 >= (1LL << 31) || (long long)kBN * ldb * 2 >= (1LL << 31)) return KFAMD_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((M / kBM) * (N / kBN), batch), block(kThreads);
  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
  __bf16* c = static_cast<__bf16*>(C);
  const __bf16* bs = static_cast<const __bf16*>(bias);
  const __bf16* r = static_cast<const __bf16*>(R);
  const bool hb = bias != nullptr, hr = R != nullptr;
#define W4_LAUNCH(ACTV, HB, HR) \
  hipLaunchKernelGGL((gemm_nt_256w4<ACTV, HB, HR>), grid, block, 0, s, a, b, c, bs, r, M, N, K, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha)
  switch (act) {
    case KFAMD_ACT_NONE:
      if (hb && hr) W4_LAUNCH(KFAMD_ACT_NONE, true, true);
      else if (hb) W4_LAUNCH(KFAMD_ACT_NONE, true, false);
      else if (hr) W4_LAUNCH(KFAMD_ACT_NONE, false, true);
      else W4_LAUNCH(KFAMD_ACT_NONE, false, false);
      break;
    case KFAMD_ACT_RELU:
      if (hb) W4_LAUNCH(KFAMD_ACT_RELU, true, false);
      else W4_LAUNCH(KFAMD_ACT_RELU, false, false);
      break;
    case KFAMD_ACT_GELU_TANH:
      if (hb) W4_LAUNCH(KFAMD_ACT_GELU_TANH, true, false);
      else W4_LAUNCH(KFAMD_ACT_GELU_TANH, false, false);
      break;
    case KFAMD_ACT_SILU:
      if (hb) W4_LAUNCH(KFAMD_ACT_SILU, true, false);
      else W4_LAUNCH(KFAMD_ACT_SILU, false, false);
      break;
    default:
      return KFAMD_EINVAL;
  }
#undef W4_LAUNCH
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
