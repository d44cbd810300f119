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
constexpr int kSlots = 5;                    // operand-tile slots (A or B each)
constexpr int kLdsBytes = kSlots * kTileBytes;  // 160 KiB: all of the CU's LDS
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

// BM = 256: the 256x256 tile above (one 160 KiB block per CU). BM = 128 ("w4s"): the same
// pipeline on a 128x128 tile, 64x64 per wave, 80 KiB of LDS -> two blocks per CU; chosen when a
// problem has fewer 256-tiles than CUs (2048^2: 64 tiles of 256^2 vs 256 of 128^2).
template <int ACT, bool HAS_BIAS, bool HAS_RES, bool DIAG = false, int RG = 2, int ABL = 0, int BM = 256>
__global__ __attribute__((amdgpu_flat_work_group_size(kThreads, kThreads),
                          amdgpu_waves_per_eu(BM == 256 ? 1 : 2, BM == 256 ? 1 : 2)))
void gemm_nt_256w4(const __bf16* __restrict__ A, const __bf16* __restrict__ B, __bf16* __restrict__ C,
                   const __bf16* __restrict__ bias, const __bf16* __restrict__ R, int M, int N, int K,
                   long long lda, long long ldb, long long ldc, long long ldr, long long sa, long long sb,
                   long long sc, long long sr, float alpha, unsigned long long* __restrict__ diag = nullptr) {
  constexpr int BN = BM, WT = BM / 2, NR = WT / 16;    // wave tile WT x WT = NR x NR MFMA blocks
  constexpr int TILE = BM * kBK * 2;                   // bytes per operand tile
  constexpr int PIECES = BM / 32;                      // 1 KiB DMA pieces per wave per operand tile
  constexpr int MF = NR * NR;                            // MFMAs per wave per k32 substep
  constexpr int DMA_EVERY = MF / PIECES;               // one DMA per DMA_EVERY MFMAs
  static_assert(BM == 256 || BM == 128, "tile");
  __shared__ __attribute__((aligned(16))) char smem[kSlots * TILE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  unsigned long long t_start = 0, rt_start = 0;
  if (DIAG) {
    t_start = __builtin_amdgcn_s_memtime();
    rt_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock: in-kernel clock + gaps
  }

  const int tiles_m = M / BM, tiles_n = N / BN, nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  constexpr int kGroupM = 4;
  const int per_group = kGroupM * tiles_n;
  const int g = wg / per_group, first_m = g * kGroupM;
  const int gm = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (wg % per_group) % gm;
  const int tn = (wg % per_group) / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const long long bz = blockIdx.y;
  A += bz * sa + (long long)m0 * lda;
  B += bz * sb + (long long)n0 * ldb;
  C += bz * sc;
  if (HAS_RES) R += bz * sr;
  // wave-uniform buffer resources over this block's 256-row panels (launcher checks < 2 GiB)
  // ABL (timing-only ablation builds, w4_diag): 1 = zero-record descriptors (every DMA dropped in
  // the address unit, instruction stream kept), 2 = no K-loop ds_reads.
  const int nrec = (DIAG && ABL == 1) ? 0 : 0x7fffffff;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, nrec, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, nrec, kRsrcWord3);

  // 32 one-KiB pieces (8 rows each) per operand tile, 8 per wave: piece p = wid*8 + j covers rows
  // 8p..8p+7; lane i lands at LDS p*1024 + 16*i (row 8p + (i>>3), swizzled chunk (i&7)) and must
  // fetch global chunk (i&7) ^ ((row>>1)&7) = (i&7) ^ ((4*(j&1) + (i>>4)) & 7): two lane offsets
  // per operand (j even / odd); the row offset 8j*ld is wave-uniform (SGPR soffset).
  const int lrow = wid * (BM / 4) + (lane >> 3);
  int va[2], vb[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int chunk = (lane & 7) ^ ((4 * par + (lane >> 4)) & 7);
    va[par] = (int)(((long long)lrow * lda + chunk * 8) * 2);
    vb[par] = (int)(((long long)lrow * ldb + chunk * 8) * 2);
  }
  const int rowstep_a = (int)(8 * lda * 2), rowstep_b = (int)(8 * ldb * 2);
  // LDS = 5 slots of 32 KiB, each holding ONE operand tile (A_t or B_t). With 4 slots live
  // (tile t being read, tile t+1 landing) the fifth lets A_{t+2} stream in during substep 0 of
  // iteration t, B_{t+2} during substep 1 (into A_t's slot, free after the mid barrier); B_t's
  // slot becomes the next free one. So the DMA is spread over the whole K-tile (1 per 8 MFMAs:
  // concentrated DMA issue stalled the single MFMA wave per SIMD — w4_diag: +30..80 cycles per
  // DMA) and A gets 3, B 2 substeps of lookahead instead of 1.5.
  auto dma_a = [&](int kt, int slot, int j) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, LDS_PTR(smem + slot * TILE + (wid * PIECES + j) * 1024), 16,
                                             va[j & 1], j * rowstep_a + kt * kBK * 2, 0, 0);
  };
  auto dma_b = [&](int kt, int slot, int j) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, LDS_PTR(smem + slot * TILE + (wid * PIECES + j) * 1024), 16,
                                             vb[j & 1], j * rowstep_b + kt * kBK * 2, 0, 0);
  };

  const int lr = lane & 15, lh = lane >> 4;
  const int sw = lh ^ (lr >> 1);
  const int off0 = lr * 128 + (sw << 4);
  const int off1 = lr * 128 + ((sw ^ 4) << 4);
  const int a_base = (wm * WT) * 128;
  const int b_base = (wn * WT) * 128;

  f32x4 acc[NR][NR];
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 a0[NR], b0[NR], a1[NR], b1[NR];
  // fragment q of a set: q < R -> B fragment q, q >= R -> A fragment q-R
  auto read_frag = [&](int sa_slot, int sb_slot, int off, bf16x8(&af)[NR], bf16x8(&bf)[NR], int q) {
    if (q < NR) bf[q] = *reinterpret_cast<const bf16x8*>(smem + sb_slot * TILE + b_base + q * 2048 + off);
    else af[q - NR] = *reinterpret_cast<const bf16x8*>(smem + sa_slot * TILE + a_base + (q - NR) * 2048 + off);
  };

  const int nk = K / kBK;
  // slot state (wave-uniform): tile t in (sa0, sb0), tile t+1 in (sa1, sb1), free slot sf
  int sa0 = 0, sb0 = 1, sa1 = 2, sb1 = 3, sf = 4;
#pragma unroll
  for (int j = 0; j < PIECES; ++j) {
    dma_a(0, sa0, j);
    dma_b(0, sb0, j);
  }
  if (nk > 1) {
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      dma_a(1, sa1, j);
      dma_b(1, sb1, j);
    }
    if constexpr (BM == 256) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  COMPILER_FENCE();
  __builtin_amdgcn_s_barrier();
  COMPILER_FENCE();
#pragma unroll
  for (int q = 0; q < 2 * NR; ++q) read_frag(sa0, sb0, off0, a0, b0, q);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  PIN();
  __builtin_amdgcn_s_setprio(1);

  // ds_reads of a substep go out 1 per RG MFMAs from its start (RG = 2: all in the first half, so
  // the waits at its end find them landed); DMA 1 per 8 MFMAs across the substep.
  // DIAG build only (cdna_hip_programming.md §7 'In-kernel stamps'): per-wave shader-clock sums of
  // the K-loop segments, read as SHARES (the stamps' lgkmcnt(0) forbids some overlap).
  unsigned long long seg[4] = {0, 0, 0, 0};
  unsigned long long t_loop0 = 0, t_loop1 = 0;
  auto stamp = [&]() -> unsigned long long {
    unsigned long long t = 0;
    if (DIAG) {
      PIN();
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      PIN();
    }
    return t;
  };
  auto body = [&](int kt, auto do_stage, auto do_next) {
    constexpr bool kStage = decltype(do_stage)::value;  // tile kt+2 exists
    constexpr bool kNext = decltype(do_next)::value;    // tile kt+1 exists
    const unsigned long long t0 = stamp();
    // substep 0: MFMAs on F0(kt); read F1(kt); DMA A_{kt+2} -> free slot
#pragma unroll
    for (int m = 0; m < MF; ++m) {
      if (!(DIAG && ABL == 2) && m % RG == 0 && m / RG < 2 * NR) read_frag(sa0, sb0, off1, a1, b1, m / RG);
      if (kStage && m % DMA_EVERY == 2) dma_a(kt + 2, sf, m / DMA_EVERY);
      PIN();
      mfma(acc[m / NR][m % NR], b0[m % NR], a0[m / NR]);
      PIN();
    }
    const unsigned long long t1 = stamp();
    // tile kt+1 landed (only A_{kt+2} may still be in flight), F1(kt) in registers, then barrier:
    // after it tile kt's slots are free
    if (kStage) {
      if constexpr (BM == 256) __builtin_amdgcn_s_waitcnt(0x0078);  // vmcnt(8) expcnt(7) lgkmcnt(0)
      else __builtin_amdgcn_s_waitcnt(0x0074);                      // vmcnt(4) expcnt(7) lgkmcnt(0)
    } else {
      __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
    }
    COMPILER_FENCE();
    __builtin_amdgcn_s_barrier();
    COMPILER_FENCE();
    PIN();
    const unsigned long long t2 = stamp();
    // substep 1: MFMAs on F1(kt); read F0(kt+1); DMA B_{kt+2} -> A_kt's slot
#pragma unroll
    for (int m = 0; m < MF; ++m) {
      if (!(DIAG && ABL == 2) && kNext && m % RG == 0 && m / RG < 2 * NR) read_frag(sa1, sb1, off0, a0, b0, m / RG);
      if (kStage && m % DMA_EVERY == 2) dma_b(kt + 2, sa0, m / DMA_EVERY);
      PIN();
      mfma(acc[m / NR][m % NR], b1[m % NR], a1[m / NR]);
      PIN();
    }
    const unsigned long long t3 = stamp();
    if (kNext) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): F0(kt+1) in registers
    PIN();
    // rotate: tile kt+1 -> current, tile kt+2 in (sf, sa0), B_kt's slot becomes free
    const int na = sf, nb = sa0;
    sf = sb0;
    sa0 = sa1;
    sb0 = sb1;
    sa1 = na;
    sb1 = nb;
    if (DIAG) {
      const unsigned long long t4 = stamp();
      seg[0] += t1 - t0;
      seg[1] += t2 - t1;
      seg[2] += t3 - t2;
      seg[3] += t4 - t3;
    }
  };
  using T = std::integral_constant<bool, true>;
  using F = std::integral_constant<bool, false>;
  if (DIAG) t_loop0 = stamp();
  int kt = 0;
  for (; kt + 2 < nk; ++kt) body(kt, T{}, T{});
  if (kt + 1 < nk) {
    body(kt, F{}, T{});
    ++kt;
  }
  if (kt < nk) body(kt, F{}, F{});
  __builtin_amdgcn_s_setprio(0);
  if (DIAG) t_loop1 = stamp();
  // the asm MFMAs are opaque to the hazard recognizer: cover the MFMA -> v_accvgpr_read latency
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  // pin every accumulator behind the padding: the MFMAs are asm, so the compiler treats their AGPR
  // results as ready at issue and would otherwise hoist v_accvgpr_read of the last writes above the
  // s_nops (it did in the bias build of w4d: stale sums). The empty asm "redefines" each one here.
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int n = 0; n < NR; ++n) asm volatile("" : "+a"(acc[i][n]));

  // Epilogue. Lane (lr, lh) holds row lr, columns 4lh..4lh+3 of every 16x16 block n. For each pair
  // of blocks (n, n+1) one v_permlane16_swap per dword trades rows 1<->0 and 3<->2 of the lane
  // groups (cdna_hip_programming.md T21, 16-lane form), after which every lane holds 8 contiguous
  // columns: lh 0 -> block n cols 0-7, lh 1 -> block n+1 cols 0-7, lh 2 -> block n cols 8-15,
  // lh 3 -> block n+1 cols 8-15. Half the store instructions (dwordx4 instead of dwordx2), every
  // row segment 64 contiguous bytes; the tail is ~5 % of a block at 8192^3 (w4_diag epilogue stamps).
  // lane id re-derived here (v_mbcnt) so no lane-derived VGPR has to survive the K loop (with every
  // VGPR taken by fragments such a survivor was spilled to scratch: profiles/r2_gemm_knobs)
  const int elane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int elr = elane & 15, elh = elane >> 4;
  auto finish = [&](int i, int n, int m) -> uint2 {
    const int col = n0 + wn * WT + n * 16 + elh * 4;
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
    return __builtin_bit_cast(uint2, o);
  };
  const int swap_col = 16 * (elh & 1) + 8 * (elh >> 1);
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int m = m0 + wm * WT + i * 16 + elr;
    __bf16* crow = C + (long long)m * ldc + n0 + wn * WT + swap_col;
#pragma unroll
    for (int n = 0; n < NR; n += 2) {
      uint2 p = finish(i, n, m), q = finish(i, n + 1, m);
      const auto sx = __builtin_amdgcn_permlane16_swap(p.x, q.x, false, false);
      const auto sy = __builtin_amdgcn_permlane16_swap(p.y, q.y, false, false);
      *reinterpret_cast<uint4*>(crow + n * 16) = uint4{sx[0], sy[0], sx[1], sy[1]};
    }
  }
  if (DIAG) {
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stores retired: the block's real end
    const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
    unsigned hw_id, xcc_id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_id));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_id));
    if (lane == 0) {
      unsigned long long* d = diag + ((long long)blockIdx.x * 4 + wid) * 16;
      for (int j = 0; j < 4; ++j) d[j] = seg[j];
      d[4] = t_loop0 - t_start;  // prologue (address setup, first two tiles, F0(0))
      d[5] = t_end - t_loop1;    // epilogue (stores issued)
      d[6] = t_loop1 - t_loop0;  // K loop
      d[7] = t_end - t_start;    // shader clocks, whole block (to the last store issue)
      d[8] = rt_start;           // 100 MHz realtime at block start / end (stores retired)
      d[9] = rt_end;
      d[10] = ((unsigned long long)(xcc_id & 0xf) << 32) | hw_id;  // which CU ran the block
    }
  }
}

}  // namespace

namespace {
template <int BM>
int launch_w4(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int batch,
              long long lda, long long ldb, long long ldc, long long ldr, long long sa, long long sb, long long sc,
              long long sr, float alpha, int act, void* stream) {
  if ((long long)BM * lda * 2 >= (1LL << 31) || (long long)BM * ldb * 2 >= (1LL << 31)) return KFAMD_EINVAL;
  if (M % BM || N % BM || K % kBK) return KFAMD_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((M / BM) * (N / BM), batch), block(kThreads);
  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
  __bf16* c = static_cast<__bf16*>(C);
  const __bf16* bs = static_cast<const __bf16*>(bias);
  const __bf16* r = static_cast<const __bf16*>(R);
  const bool hb = bias != nullptr, hr = R != nullptr;
#define W4_LAUNCH(ACTV, HB, HR)                                                                                  \
  hipLaunchKernelGGL((gemm_nt_256w4<ACTV, HB, HR, false, 2, 0, BM>), grid, block, 0, s, a, b, c, bs, r, M, N, K, lda, \
                     ldb, ldc, ldr, sa, sb, sc, sr, alpha)
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
}  // namespace

// Caller (kfamd_gemm_nt_bf16_variant) has validated alignment; shapes are re-checked per tile
// size. The buffer offsets are 32-bit, so a block's BM-row panel must span < 2 GiB.
extern "C" int kfamd_gemm_nt_bf16_w4_launch(const void* A, const void* B, void* C, const void* bias, const void* R,
                                            int M, int N, int K, int batch, long long lda, long long ldb, long long ldc,
                                            long long ldr, long long sa, long long sb, long long sc, long long sr,
                                            float alpha, int act, void* stream) {
  return launch_w4<256>(A, B, C, bias, R, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, act, stream);
}

// 128x128 tiles (two blocks per CU) for problems with fewer 256-tiles than CUs.
extern "C" int kfamd_gemm_nt_bf16_w4s_launch(const void* A, const void* B, void* C, const void* bias, const void* R,
                                             int M, int N, int K, int batch, long long lda, long long ldb,
                                             long long ldc, long long ldr, long long sa, long long sb, long long sc,
                                             long long sr, float alpha, int act, void* stream) {
  return launch_w4<128>(A, B, C, bias, R, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, act, stream);
}

#ifdef KFAMD_DIAG
// Diagnostic build only (libkfamd_kernels_diag.so, kubeflow_rm_amd._build.build_diag_kernels; never
// in the production library): per-wave K-loop segment cycle sums into diag
// [(M/256)*(N/256) blocks][4 waves][4 segments] (tools/kbench.py --diag-w4).
extern "C" int kfamd_gemm_nt_bf16_w4_diag(const void* A, const void* B, void* C, int M, int N, int K,
                                          unsigned long long* diag, int abl, void* stream) {
  if (M % kBM || N % kBN || K % kBK || !diag) return KFAMD_EINVAL;
  dim3 grid((M / kBM) * (N / kBN), 1), block(kThreads);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
  __bf16* c = static_cast<__bf16*>(C);
#define W4_DIAG(AB)                                                                                              \
  hipLaunchKernelGGL((gemm_nt_256w4<KFAMD_ACT_NONE, false, false, true, 2, AB>), grid, block, 0, s, a, b, c, nullptr, \
                     nullptr, M, N, K, (long long)K, (long long)K, (long long)N, 0LL, 0LL, 0LL, 0LL, 0LL, 1.0f, diag)
  if (abl == 0) W4_DIAG(0);
  else if (abl == 1) W4_DIAG(1);
  else if (abl == 2) W4_DIAG(2);
  else return KFAMD_EINVAL;
#undef W4_DIAG
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
#endif  // KFAMD_DIAG
