// gemm_w4.h — the K1 "w4" MFMA GEMM template: 4 waves (2x2) per block, one wave per SIMD with the
// full register file (accumulators pinned in AGPRs), LDS-DMA staging through a 5-slot ring.
// Instantiated by gemm_bf16_w4.hip (forward "NT" layout) and gemm_bf16_w4_t.hip (the backward
// layouts), so each translation unit compiles only the variants it launches
// (cdna_hip_programming.md §5.4 rule 19: co-compiled template variants perturb each other).
//
// Why this shape (MI355X_MICROARCH.md 'DVFS give-back' + cdna_hip_programming.md §5.4 rule 28):
// on random data a bf16 GEMM runs clock-limited (~1.9 GHz), and what raises the held clock for the
// same MFMAs is less energy per MFMA — fewer LDS read bytes and fewer VALU. LDS fragment reads per
// K-tile scale with sum over waves of (wave_M + wave_N): 4 waves of 128x128 read 128 KiB per CU per
// K-tile against 192 KiB for 8 waves of 128x64, with the same MFMA count and DMA bytes.
//
// Operand layouts (template LA / LB), C[m][n] = sum_k Aop[m][k] * Bop[n][k]:
//   LA = 0: A stored [M][K], K contiguous (row-major activations: the forward and dgrad A)
//   LA = 1: A stored [K][M], M contiguous (dY read as dY^T by the wgrad GEMM)
//   LB = 0: B stored [N][K] (F.linear weight);  LB = 1: B stored [K][N] (W in dgrad, X in wgrad)
// A K-contiguous operand is staged as [rows][64 k] 128-B rows (XOR swizzle on the 16-B chunk, read
// with ds_read_b128); a row-contiguous ("k-major") operand as [64 k][BM] rows of BM*2 bytes, read
// with ds_read_b64_tr_b16 (cdna_hip_programming.md T10), which hands each lane 4 consecutive k of one
// column: two reads make the 8-k MFMA fragment. The k-major image is XOR-swizzled on chunk bits 1-3
// by f(row) = 2*((row&3) | ((row>>3)&1)<<2): the 8 rows one 32-lane half reads (q = 0..3, two lane
// groups 8 rows apart) then land on 8 distinct 32-B bank slots — conflict-free. The swizzle goes on
// the DMA SOURCE address (LDS stays lane-linear, §5.4 rule 21) and on the read address.
//
// Edges (no padding copies):
//   * M / N: the last tile row/column is SHIFTED to end at M / N (m0 = min(tm*BM, M-BM)); it
//     overlaps its neighbour, recomputes those outputs from the same data and does not store them
//     (store mask m >= tm*BM, n >= tn*BN). Needs M, N >= BM.
//   * K: the K tiling is shifted so the partial tile is the FIRST one (tile t covers k from
//     koff + 64t, koff = K - 64*ceil(K/64) <= 0; the buffer base moves by koff). Only the prologue's
//     tile 0 has out-of-range 16-B pieces (k < 0): they get a voffset past the buffer's num_records,
//     so the LDS-DMA writes zeros (raw-buffer range check; valid pieces keep voffset + soffset inside
//     the record, so this holds whether or not the check includes soffset). The K loop itself carries
//     no edge code.
// Pipeline (unchanged from r2): two LDS tiles live + one free slot, DMA of tile kt+2 spread over
// the K-tile (1 per 8 MFMAs), fragments of the next k-substep read under the current substep's
// MFMAs (two register sets), interleave pinned with sched_barrier.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "kfamd_kernels.h"

namespace kfw4 {
namespace {  // internal linkage: each translation unit instantiates its own kernels

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define KFW4_LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))
#define KFW4_FENCE() asm volatile("" ::: "memory")
#define KFW4_PIN() __builtin_amdgcn_sched_barrier(0)

constexpr int kBK = 64, kThreads = 256;
constexpr int kSlots = 5;                         // operand-tile slots (A or B each)
constexpr int kRsrcWord3 = 0x00020000;            // gfx9 raw buffer: 32-bit dword format, no swizzle
constexpr unsigned kOOB = 0x80000000u;            // voffset of a zero-filled (out-of-range) piece
constexpr int kNumRecords = 0x7fffffff;
constexpr unsigned long long kSkTimeoutTicks = 5000000;  // stream-K partial wait: 50 ms of s_memrealtime

__device__ __forceinline__ float act_fn(float v, int act) {
  switch (act) {
    case KFAMD_ACT_RELU: return v > 0.f ? v : 0.f;
    case KFAMD_ACT_GELU_TANH: {
      // 0.5 v (1 + tanh(u)) == v * sigmoid(2u): one v_exp + one v_rcp instead of libm tanhf (the
      // tanhf epilogue cost ~25 % of an 8192x4096x4096 GEMM, profiles/r3_linear)
      const float u2 = 1.5957691216057308f * (v + 0.044715f * v * v * v);
      return v * __builtin_amdgcn_rcpf(1.f + __expf(-u2));
    }
    case KFAMD_ACT_SILU: return v * __builtin_amdgcn_rcpf(1.f + __expf(-v));
    default: return v;
  }
}

// act'(z) on a pair of values: the polynomial parts as packed f32 ops (v_pk_mul / v_pk_fma: two
// lanes' worth per instruction), the exp / rcp per value. gelu_tanh with 2u = z (A + B z^2):
// act' = s (1 + z (1 - s) (A + 3 B z^2)), s = sigmoid(2u), log2(e) folded into exp's argument.
typedef float kf32x2 __attribute__((ext_vector_type(2)));
template <int ACT>
__device__ __forceinline__ kf32x2 dact2(kf32x2 z) {
  if constexpr (ACT == KFAMD_ACT_RELU) {
    return kf32x2{z.x > 0.f ? 1.f : 0.f, z.y > 0.f ? 1.f : 0.f};
  } else if constexpr (ACT == KFAMD_ACT_GELU_TANH) {
    constexpr float A = 1.5957691216057308f, B = 1.5957691216057308f * 0.044715f, L2E = 1.4426950408889634f;
    const kf32x2 z2 = z * z;
    const kf32x2 q = z * __builtin_elementwise_fma(z2, kf32x2{-B * L2E, -B * L2E}, kf32x2{-A * L2E, -A * L2E});
    const kf32x2 s{__builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(q.x)),
                   __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(q.y))};
    const kf32x2 r = __builtin_elementwise_fma(z2, kf32x2{3.f * B, 3.f * B}, kf32x2{A, A});
    const kf32x2 w = __builtin_elementwise_fma((kf32x2{1.f, 1.f} - s) * z, r, kf32x2{1.f, 1.f});
    return s * w;
  } else if constexpr (ACT == KFAMD_ACT_SILU) {
    constexpr float L2E = 1.4426950408889634f;
    const kf32x2 q = z * kf32x2{-L2E, -L2E};
    const kf32x2 s{__builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(q.x)),
                   __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(q.y))};
    return s * __builtin_elementwise_fma((kf32x2{1.f, 1.f} - s), z, kf32x2{1.f, 1.f});
  } else {
    return kf32x2{1.f, 1.f};
  }
}

// act(z) on a pair (the forward epilogue, KFW4_ACT_PK): gelu_tanh / silu as z * sigmoid(.), the
// polynomial parts packed as in dact2
#ifndef KFW4_ACT_PK
#define KFW4_ACT_PK 1
#endif
template <int ACT>
__device__ __forceinline__ kf32x2 act2(kf32x2 z) {
  constexpr float L2E = 1.4426950408889634f;
  kf32x2 q;
  if constexpr (ACT == KFAMD_ACT_GELU_TANH) {
    constexpr float A = 1.5957691216057308f, B = 1.5957691216057308f * 0.044715f;
    q = z * __builtin_elementwise_fma(z * z, kf32x2{-B * L2E, -B * L2E}, kf32x2{-A * L2E, -A * L2E});
  } else {
    q = z * kf32x2{-L2E, -L2E};
  }
  const kf32x2 e{__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  const kf32x2 d = e + kf32x2{1.f, 1.f};
  return z * kf32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ void mfma(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
// The same, opaque to CSE: the epilogue re-derives it after the K loop instead of the compiler
// keeping a prologue copy (lane >> 4) alive - or spilled - across the loop.
__device__ __forceinline__ int lane_id_fresh() {
  int v;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
  return v;
}

// Per-operand staging geometry. One operand tile = 64 k x BM rows/cols = BM*128 bytes, DMA'd as
// BM/32 one-KiB pieces per wave (4 waves).
template <int L, int BM>
struct Stage {
  static constexpr int TILE = BM * kBK * 2;
  static constexpr int PIECES = BM / 32;
  // number of distinct per-lane voffsets over the wave's pieces (depends on the swizzle)
  static constexpr int NV = L == 0 ? 2 : (BM == 256 ? 4 : 2);
  static constexpr int RPP = 512 / BM;            // k-major: k rows per 1-KiB piece (2 or 4)
  static constexpr int LPR = BM / 8;              // k-major: lanes per k row (32 or 16)

  unsigned voff[NV];
  int rowstep;   // bytes between consecutive pieces of a wave (wave-uniform)
  int ktstep;    // bytes per K tile (wave-uniform)

  __device__ __forceinline__ void init(int wid, int lane, long long ld) {
    if constexpr (L == 0) {
      // piece p = wid*PIECES + j covers rows 8p..8p+7; lane i lands at LDS p*1024 + 16*i (row
      // 8p + (i>>3), swizzled chunk (i&7)) and fetches global chunk (i&7) ^ ((row>>1)&7)
      const int lrow = wid * (BM / 4) + (lane >> 3);
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        const int chunk = (lane & 7) ^ ((4 * par + (lane >> 4)) & 7);
        voff[par] = (unsigned)(((long long)lrow * ld + chunk * 8) * 2);
      }
      rowstep = (int)(8 * ld * 2);
      ktstep = kBK * 2;
    } else {
      // piece j of wave w covers k rows 16w + RPP*j + rip (rip = lane / LPR), phys chunk lane % LPR;
      // global chunk = phys ^ f(row), f = lane part (2*rip) ^ wave part (depends on j only)
      const int rip = lane / LPR, phys = lane % LPR;
      const unsigned v16 = (unsigned)((phys ^ (2 * (rip & 3))) * 16);
      const unsigned vrow = (unsigned)((long long)(16 * wid + rip) * ld * 2);
#pragma unroll
      for (int v = 0; v < NV; ++v) voff[v] = (v16 ^ (unsigned)(wave_f16_of_variant(v))) + vrow;
      rowstep = (int)(RPP * ld * 2);
      ktstep = (int)(kBK * ld * 2);
    }
  }
  // k-major: XOR (in bytes) the wave part of f adds to the chunk offset, per voffset variant
  static __device__ __forceinline__ int wave_f16_of_variant(int v) {
    if constexpr (BM == 256) return ((v & 1) * 4 + ((v >> 1) & 1) * 8) * 16;
    else return (v & 1) * 8 * 16;
  }
  static __device__ __forceinline__ constexpr int variant_of_piece(int j) {
    if constexpr (L == 0) return j & 1;
    else if constexpr (BM == 256) return (j & 1) | (((j >> 2) & 1) << 1);
    else return (j >> 1) & 1;
  }
  // validity of this lane's 16-B piece j of the first (partial) K tile, koff = K - 64*nk <= 0
  static __device__ __forceinline__ bool valid0(int j, int wid, int lane, int koff) {
    if constexpr (L == 0) {
      const int chunk = (lane & 7) ^ ((4 * (j & 1) + (lane >> 4)) & 7);
      return koff + chunk * 8 >= 0;
    } else {
      return koff + 16 * wid + RPP * j + lane / LPR >= 0;
    }
  }
};

// LDS fragment reader for one operand: fragment q (16 rows/cols of the wave tile) of k-substep s.
template <int L, int BM>
struct Reader {
  static constexpr int TILE = BM * kBK * 2;
  static constexpr int ROWB = BM * 2;    // k-major LDS row bytes
  int wbase;       // L=0: byte offset of the wave's first row; L=1: unused
  int off[2];      // L=0: per-lane byte offset within a 2 KiB fragment block, per substep
  unsigned vfw;    // L=1: (32*F) ^ (2*wave column base), F = (q4 | (g&1)<<2)
  unsigned vl;     // L=1: lane part (8g+q4)*ROWB + 8p

  __device__ __forceinline__ void init(int lane, int wpos) {
    const int WT = BM / 2;
    if constexpr (L == 0) {
      const int lr = lane & 15, lh = lane >> 4;
      const int sw = lh ^ (lr >> 1);
      off[0] = lr * 128 + (sw << 4);
      off[1] = lr * 128 + ((sw ^ 4) << 4);
      wbase = (wpos * WT) * 128;
    } else {
      const int g = lane >> 4, i = lane & 15, q4 = i >> 2, p = i & 3;
      const int F = q4 | ((g & 1) << 2);
      vfw = (unsigned)((32 * F) ^ (2 * wpos * WT));
      vl = (unsigned)((8 * g + q4) * ROWB + 8 * p);
      wbase = 0;
    }
  }
  template <int S>
  __device__ __forceinline__ bf16x8 read(const char* smem, int slot, int q) const {
    if constexpr (L == 0) {
      return *reinterpret_cast<const bf16x8*>(smem + slot * TILE + wbase + q * 2048 + off[S]);
    } else {
      // inline asm, not __builtin_amdgcn_ds_read_tr16_b64: hipcc 7.2 puts an s_waitcnt vmcnt(0)
      // before every builtin tr read that follows an LDS-DMA (draining the staging pipeline each
      // substep). Ordering against the DMA comes from the K loop's counted vmcnt + barrier, and
      // the results are covered by the loop's explicit lgkmcnt(0) before their MFMAs (as for the
      // plain ds_read_b128 of the K-contiguous operand).
      typedef short s16x4 __attribute__((ext_vector_type(4)));
      const unsigned a = (vfw ^ (unsigned)(32 * q)) + vl + (unsigned)(slot * TILE) +
                         (unsigned)(uintptr_t)KFW4_LDS_PTR(smem);
      s16x4 lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(a), "i"((32 * S) * ROWB));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a), "i"((32 * S + 4) * ROWB));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

// BM = 256: 256x256 tile (one 160 KiB block per CU). BM = 128 ("w4s"): the same pipeline on a 128x128
// tile, 64x64 per wave, 80 KiB of LDS -> two blocks per CU (problems with fewer 256-tiles than CUs).
// AUX (ACT != NONE only): also store the pre-activation act^-1 input, for the activation's backward.
// SPLIT (split-K, for problems with too few output tiles to fill 256 CUs): blockIdx.z takes the K
// range [z*kper, (z+1)*kper) and the block stores its raw fp32 partial tile to W[z][M][N]; the
// epilogue (alpha, bias, activation, Aux, residual) runs in splitk_reduce (gemm_bf16.hip).
// SPLIT == 2 (split-K with the fixup in the kernel, 256 tile, for tile counts well under the CU
// count): the same K ranges, but every split block stores its fp32 partial in accumulator-fragment
// order - wave w's f32x4 (i, n) for its 64 lanes is 1 KiB contiguous, so each store and load covers 8
// whole 128-B lines - written through to the agent's coherence point (sc1), then counts itself in on
// the tile's arrival counter (sk_flags[tile]). The block that arrives last adds the other splits'
// partials to its accumulators, rearms the counter (0) and runs the full epilogue. Nobody waits on
// anybody, so the grid needs no co-residency.
// SK (stream-K, for grids that leave part of the last wave of 256 CUs idle): a persistent grid of
// G = gridDim.x blocks (one per CU) first runs the whole data-parallel waves (tiles [0, T - T % G)),
// then the remaining tiles in kper K-splits each, spread round-robin over all G blocks. The block
// running a tile's last split owns it: it adds the other splits' fp32 partials (W[unit][BM][BN],
// released with an agent-scope flag = epoch) and runs the epilogue; a partial that does not arrive
// within the deadline is recomputed by the owner itself, so a non-co-resident grid is slow, never
// hung or wrong.
// GRP: a second problem in the same launch (W4Grp: its own A, B, C, M, N and leading dimensions; the
// same K, layouts and epilogue): blocks [0, tiles of problem 1) take problem 1, the rest problem 2,
// after the XCD remap over both. For two GEMMs that under-fill the chip alone, e.g. a transformer
// block's QKV and output-projection weight gradients (192 + 64 tiles of 256 x 256 at gpt-1b:
// one full wave of 256 CUs together; kfamd_w4_wgrad_pair, gemm_bf16_w4_t.hip).
struct W4Grp {
  const __bf16* A;
  const __bf16* B;
  __bf16* C;
  int M, N;
  long long lda, ldb, ldc;
};

// DACT (a linear layer's backward through its activation, gemm_bf16_w4_t.hip kfamd_w4_dgrad_act):
// C = (A·B) * act'(R), R = the pre-activation the forward stored, and when W is given the column
// sums of C per wave-row slab (W[M / (BM / 2)][N], the next layer's bias-gradient partials):
// the elementwise act-grad pass (act_grad_bf16.hip) folded into the dgrad GEMM's epilogue, which
// reads R where that pass read both dY and R and wrote G. Whole interior tiles only (the host
// requires M and N multiples of 256 and 16-B rows), on the full-line residual epilogue.
template <int ACT, bool HAS_BIAS, bool HAS_RES, bool HAS_AUX, int LA, int LB, int BM, int SPLIT = 0,
          bool DIAG = false, int ABL = 0, bool SK = false, bool PO = false, bool DACT = false, bool GRP = false>
__global__ __attribute__((amdgpu_flat_work_group_size(kThreads, kThreads),
                          amdgpu_waves_per_eu(BM == 256 ? 1 : 2, BM == 256 ? 1 : 2)))
void gemm_w4(const __bf16* __restrict__ A, const __bf16* __restrict__ B, __bf16* __restrict__ C,
             const __bf16* __restrict__ bias, const __bf16* __restrict__ R, __bf16* __restrict__ Aux, int M, int N,
             int K, long long lda, long long ldb, long long ldc, long long ldr, long long sa, long long sb,
             long long sc, long long sr, float alpha, unsigned long long* __restrict__ diag,
             float* __restrict__ W = nullptr, int kper = 0, unsigned* __restrict__ sk_flags = nullptr,
             unsigned sk_epoch = 0, W4Grp g2 = W4Grp{}) {
  constexpr int BN = BM, WT = BM / 2, NR = WT / 16;    // wave tile WT x WT = NR x NR MFMA blocks
  constexpr int TILE = BM * kBK * 2;                   // bytes per operand tile
  constexpr int PIECES = BM / 32;                      // 1 KiB DMA pieces per wave per operand tile
  constexpr int MF = NR * NR;                          // MFMAs per wave per k32 substep
  // Schedule knobs (tools/w4_ab.py A/B builds; the defaults are the production schedule):
  //   KFW4_RG: one fragment read per RG MFMAs; KFW4_DMA_EVERY / KFW4_DMA_PHASE: DMA piece j at
  //   MFMA j * DMA_EVERY + DMA_PHASE of its substep; KFW4_PIN_MFMA: sched_barrier around every MFMA.
#ifndef KFW4_DMA_EVERY
#define KFW4_DMA_EVERY 0
#endif
#ifndef KFW4_DMA_PHASE
#define KFW4_DMA_PHASE 2
#endif
#ifndef KFW4_RG
#define KFW4_RG 2
#endif
#ifndef KFW4_PIN_MFMA
#define KFW4_PIN_MFMA 1
#endif
#ifndef KFW4_PRIO
#define KFW4_PRIO 1
#endif
  constexpr int DMA_EVERY = KFW4_DMA_EVERY > 0 ? KFW4_DMA_EVERY : MF / PIECES;  // one DMA per DMA_EVERY MFMAs
  constexpr int DMA_PHASE = KFW4_DMA_PHASE;
  static_assert(DMA_EVERY * (PIECES - 1) + DMA_PHASE < MF, "every DMA piece inside its substep");
  constexpr int RG = KFW4_RG < MF / (2 * NR) ? KFW4_RG : MF / (2 * NR);  // 128 tile: at most 2
  static_assert(RG * (2 * NR - 1) < MF, "every fragment read inside its substep");
  static_assert(BM == 256 || BM == 128, "tile");
  static_assert(!HAS_AUX || ACT != KFAMD_ACT_NONE, "aux = pre-activation");
  static_assert(SPLIT != 1 || (ACT == KFAMD_ACT_NONE && !HAS_BIAS && !HAS_RES && !HAS_AUX), "split-K: epilogue in the reduce");
  static_assert(SPLIT != 2 || BM == 256, "split-K fixup: 256 tile");
  static_assert(!SK || (!HAS_AUX && BM == 256 && !SPLIT), "stream-K: 256 tile, no pre-activation output");
  static_assert(!PO || (BM == 256 && !SPLIT && !SK && !DIAG), "persistent overlapped: 256 tile, whole K");
  static_assert(!GRP || (SPLIT != 1 && !SK && !PO && !DACT && !HAS_BIAS && !HAS_RES && !HAS_AUX && !DIAG),
                "grouped pair: plain epilogue, whole K or the in-kernel split-K fixup");
  static_assert(!DACT || (HAS_RES && !HAS_BIAS && !HAS_AUX && ACT != KFAMD_ACT_NONE && !SPLIT && !SK && !PO),
                "act-grad epilogue: the pre-activation as R, 256 tile, whole K");
  // PO: the epilogue's LDS staging lives in the ring's fifth slot, which the next tile's prologue
  // (tiles 0 and 1 into slots 0-3) leaves alone, so that prologue can be issued before the epilogue
  constexpr int kEpiBase = PO ? (kSlots - 1) * TILE : 0;
  __shared__ __attribute__((aligned(16))) char smem[kSlots * TILE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  unsigned long long t_start = 0, rt_start = 0;
  if (DIAG) {
    t_start = __builtin_amdgcn_s_memtime();
    rt_start = __builtin_amdgcn_s_memrealtime();
  }

  int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN, nwg = tiles_m * tiles_n;
  int wg;
  int grp_base = 0, nwg_all = nwg;  // GRP: this problem's first tile / both problems' tiles (split-K slots)
  if constexpr (GRP) {
    const int t1 = nwg, t2 = ((g2.M + BM - 1) / BM) * ((g2.N + BN - 1) / BN);
    nwg_all = t1 + t2;
    wg = xcd_remap(blockIdx.x, t1 + t2);
    if (wg >= t1) {  // problem 2 (uniform per block)
      grp_base = t1;
      wg -= t1;
      A = g2.A;
      B = g2.B;
      C = g2.C;
      M = g2.M;
      N = g2.N;
      lda = g2.lda;
      ldb = g2.ldb;
      ldc = g2.ldc;
      tiles_m = (M + BM - 1) / BM;
      tiles_n = (N + BN - 1) / BN;
      nwg = t2;
    }
  } else {
    wg = xcd_remap(blockIdx.x, nwg);
  }
#ifndef KFW4_SK_AB
#define KFW4_SK_AB 0  // stream-K timing ablations (tools/sk_ab.py builds): 1 no partial traffic, 2 no owner wait
#endif
#ifndef KFW4_GROUP_M
#define KFW4_GROUP_M 4  // tile-row group of the grouped raster (A/B runs build other values)
#endif
  constexpr int kGroupM = KFW4_GROUP_M;
  const int per_group = kGroupM * tiles_n;
  const int g = wg / per_group, first_m = g * kGroupM;
  const int gm = min(tiles_m - first_m, kGroupM);
  int tm = first_m + (wg % per_group) % gm;
  int tn = (wg % per_group) / gm;
#ifndef KFW4_SUPER
#define KFW4_SUPER 1  // 16 x 16-tile superblocks across the 8 XCDs for operands past the MALL (below)
#endif
  if constexpr (KFW4_SUPER && !GRP && BM == 256) {
    // the chip's 256 resident tiles (one per CU) as ONE 16 x 16 block of the output: XCD x (block b
    // runs on XCD b % 8) takes its 4 x 8 sub-block, rows 4 (x & 3), columns 8 (x >> 2); the waves walk
    // the superblocks column-major. 16 A + 16 B panels are live at once instead of 32 A + 8 B with the
    // per-XCD row groups (at 16384^3 a panel is 8 MiB: 256 vs 320 MiB against the 256 MiB MALL):
    // 16384^3 0.987 -> 1.012 of hipBLASLt, 4096^3 / 8192^3 level (profiles/r6zm_super). Only where A
    // and B together exceed the MALL; smaller problems keep the row groups.
    if ((tiles_m & 15) == 0 && (tiles_n & 15) == 0 && gridDim.x == (unsigned)nwg &&  // (not the persistent grid)
        (long long)(M + N) * K * 2 > (256LL << 20)) {
      const int b = blockIdx.x, x = b & 7, i = b >> 3, wave = i >> 5, j = i & 31;
      const int sbm = tiles_m >> 4, sr = wave % sbm, sc = wave / sbm;
      tm = 16 * sr + 4 * (x & 3) + (j & 3);
      tn = 16 * sc + 8 * (x >> 2) + (j >> 2);
    }
  }
  int m_lo = tm * BM, n_lo = tn * BN;                  // first output row / column this block stores
  int m0 = min(m_lo, M - BM), n0 = min(n_lo, N - BN);  // edge tiles shifted inside

  long long kbeg = 0;
  if (SPLIT) {  // this block's K range; only the last split can be partial (kper % 64 == 0)
    kbeg = (long long)blockIdx.z * kper;
    K = min((long long)kper, (long long)K - kbeg);
  }
  int nk = (K + kBK - 1) / kBK;
  int koff = K - nk * kBK;                             // first K tile starts at k = koff (<= 0)
  const long long bz = blockIdx.y;
  const long long ka = kbeg + koff;
  const __bf16* const A_in = A;
  const __bf16* const B_in = B;
  A += bz * sa + (LA == 0 ? (long long)m0 * lda + ka : (long long)m0 + ka * lda);
  B += bz * sb + (LB == 0 ? (long long)n0 * ldb + ka : (long long)n0 + ka * ldb);
  C += bz * sc;
  if (HAS_AUX) Aux += bz * sc;
  if (HAS_RES) R += bz * sr;
  // ABL (timing-only ablation builds, w4_diag): 1 = zero-record descriptors (every DMA dropped in
  // the address unit, instruction stream kept), 2 = no K-loop ds_reads.
  const int nrec = (DIAG && ABL == 1) ? 0 : kNumRecords;
  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, nrec, kRsrcWord3);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, nrec, kRsrcWord3);

  Stage<LA, BM> sta;
  Stage<LB, BM> stb;
  sta.init(wid, lane, lda);
  stb.init(wid, lane, ldb);
  // LDS = 5 slots, each holding ONE operand tile. With 4 slots live (tile t being read, tile t+1
  // landing) the fifth lets A_{t+2} stream in during substep 0 of iteration t, B_{t+2} during
  // substep 1 (into A_t's slot, free after the mid barrier); B_t's slot becomes the next free one.
  // the soffset operands as plain locals: naming a struct member inside the builtin's soffset made
  // hipcc 7.2's host pass drop the kernel's launch stub (and with it the whole device bundle of the
  // translation unit) without a diagnostic; _build.check_object_kernels guards against a recurrence
  const int rs_a = sta.rowstep, kts_a = sta.ktstep, rs_b = stb.rowstep, kts_b = stb.ktstep;
  auto dma_a = [&](int kt, int slot, int j, bool first) {
    unsigned v = sta.voff[Stage<LA, BM>::variant_of_piece(j)];
    if (first && !Stage<LA, BM>::valid0(j, wid, lane_id(), koff)) v = kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, KFW4_LDS_PTR(smem + slot * TILE + (wid * PIECES + j) * 1024), 16,
                                             v, j * rs_a + kt * kts_a, 0, 0);
  };
  auto dma_b = [&](int kt, int slot, int j, bool first) {
    unsigned v = stb.voff[Stage<LB, BM>::variant_of_piece(j)];
    if (first && !Stage<LB, BM>::valid0(j, wid, lane_id(), koff)) v = kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, KFW4_LDS_PTR(smem + slot * TILE + (wid * PIECES + j) * 1024), 16,
                                             v, j * rs_b + kt * kts_b, 0, 0);
  };

#ifndef KFW4_FASTK
#define KFW4_FASTK 2  // 2: steady-state DMAs with a voffset register per piece and one soffset per K-tile
#endif
  // (a per-K-tile descriptor rebuild, tried as mode 1, made hipcc 7.2's host pass drop the launch stubs)
#ifndef KFW4_UNROLL5
#define KFW4_UNROLL5 1  // K loop unrolled over the 5-slot ring's period: every slot index a constant
#endif
#ifndef KFW4_ASM_DMA
#define KFW4_ASM_DMA 1
#endif
  static_assert(!KFW4_ASM_DMA || (KFW4_FASTK == 2 && KFW4_DMA_PHASE >= 1), "asm DMA: voffset regs, M0 set one MFMA ahead");
  // stream-K keeps the round-3 steady state: its persistent schedule's live state plus these
  // registers (voffsets, descriptors, the unrolled loop's constants) spill
  constexpr int kFastK = SK ? 0 : KFW4_FASTK;
  constexpr bool kAsmDma = !SK && KFW4_ASM_DMA;
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  // raw buffer descriptors as SGPR quads for the asm pieces (gfx9: base, base_hi | stride 0, records, word 3)
  auto make_desc = [&](const void* p) __attribute__((always_inline)) -> i32x4 {
    const unsigned long long a = reinterpret_cast<unsigned long long>(p);
    return i32x4{__builtin_amdgcn_readfirstlane((int)(unsigned)a), __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff)),
                 nrec, kRsrcWord3};
  };
  i32x4 dra = make_desc(A), drb = make_desc(B);
  const unsigned lds_w = (unsigned)(uintptr_t)KFW4_LDS_PTR(smem) + (unsigned)(wid * PIECES * 1024);  // wave's pieces
  // KFW4_FASTK == 2: piece j's full voffset (chunk swizzle + j rows) in a register of its own
  unsigned vpa[PIECES], vpb[PIECES];
  if (kFastK == 2) {
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      vpa[j] = sta.voff[Stage<LA, BM>::variant_of_piece(j)] + (unsigned)(j * rs_a);
      vpb[j] = stb.voff[Stage<LB, BM>::variant_of_piece(j)] + (unsigned)(j * rs_b);
    }
  }

  Reader<LA, BM> rda;
  Reader<LB, BM> rdb;
  rda.init(lane, wm);
  rdb.init(lane, wn);

  f32x4 acc[NR][NR];
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 a0[NR], b0[NR], a1[NR], b1[NR];
  // fragment q of a set: q < NR -> B fragment q, q >= NR -> A fragment q-NR
  auto read_frag0 = [&](int sa_slot, int sb_slot, bf16x8(&af)[NR], bf16x8(&bf)[NR], int q) {
    if (q < NR) bf[q] = rdb.template read<0>(smem, sb_slot, q);
    else af[q - NR] = rda.template read<0>(smem, sa_slot, q - NR);
  };
  auto read_frag1 = [&](int sa_slot, int sb_slot, bf16x8(&af)[NR], bf16x8(&bf)[NR], int q) {
    if (q < NR) bf[q] = rdb.template read<1>(smem, sb_slot, q);
    else af[q - NR] = rda.template read<1>(smem, sa_slot, q - NR);
  };

  // DIAG build only (cdna_hip_programming.md §7 'In-kernel stamps'): per-wave shader-clock sums of
  // the K-loop segments, read as SHARES (the stamps' lgkmcnt(0) forbids some overlap).
  unsigned long long seg[4] = {0, 0, 0, 0};
  unsigned long long t_loop0 = 0, t_loop1 = 0;
#ifndef KFW4_CHEAP_STAMPS
#define KFW4_CHEAP_STAMPS 0  // 1: s_memtime with no wait of its own; read after the loop's own lgkmcnt(0)
#endif
  auto stamp = [&]() -> unsigned long long {
    unsigned long long t = 0;
    if (DIAG) {
      KFW4_PIN();
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      KFW4_PIN();
    }
    return t;
  };
  // K-loop stamps: with KFW4_CHEAP_STAMPS no wait of their own (valid after the loop's lgkmcnt(0))
  auto stamp_k = [&]() -> unsigned long long {
    unsigned long long t = 0;
    if (DIAG && KFW4_CHEAP_STAMPS) {
      KFW4_PIN();
      asm volatile("s_memtime %0" : "=s"(t)::"memory");
      KFW4_PIN();
    } else if (DIAG) {
      t = stamp();
    }
    return t;
  };
  unsigned long long prev_t3 = 0;  // cheap stamps: the previous iteration's end-of-MFMA stamp
  using T = std::integral_constant<bool, true>;
  using F = std::integral_constant<bool, false>;
  unsigned long long sk_mask = 0;  // stream-K owner: which producer splits' partials the epilogue adds
  int sk_base = 0, sk_stride = 0;  // ... split j's partial is slot sk_base + j * sk_stride
  // prologue + K loop over the current (ra, rb, nk, koff): adds into acc
  // the first two K tiles into slots 0-3 (PO issues them for the next tile before this one's epilogue)
  auto issue_prologue = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      dma_a(0, 0, j, true);
      dma_b(0, 1, j, true);
    }
    if (nk > 1) {
#pragma unroll
      for (int j = 0; j < PIECES; ++j) {
        dma_a(1, 2, j, false);
        dma_b(1, 3, j, false);
      }
    }
  };
  auto run_k = [&](auto pro_issued) __attribute__((always_inline)) {
  // slot state (wave-uniform): tile t in (sa0, sb0), tile t+1 in (sa1, sb1), free slot sf
  int sa0 = 0, sb0 = 1, sa1 = 2, sb1 = 3, sf = 4;
  if constexpr (!decltype(pro_issued)::value) issue_prologue();
  if (nk > 1) {
    // (PO: the epilogue's stores were issued after these DMAs; counting them in too only waits
    // longer, and the epilogue has covered the DMAs' latency)
    if constexpr (BM == 256) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  KFW4_FENCE();
  __builtin_amdgcn_s_barrier();
  KFW4_FENCE();
#pragma unroll
  for (int q = 0; q < 2 * NR; ++q) read_frag0(sa0, sb0, a0, b0, q);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  KFW4_PIN();
  if (KFW4_PRIO) __builtin_amdgcn_s_setprio(1);

  // one K-tile; the slots come in as ints (rotating at run time) or integral constants (unrolled)
  auto body_g = [&](int kt, auto do_stage, auto do_next, auto sa0, auto sb0, auto sa1, auto sb1, auto sf)
      __attribute__((always_inline)) {
    constexpr bool kStage = decltype(do_stage)::value;  // tile kt+2 exists
    constexpr bool kNext = decltype(do_next)::value;    // tile kt+1 exists
    // KFW4_ASM_DMA: the steady-state pieces as inline asm, M0 written one MFMA ahead (no s_nop for
    // the M0 -> LDS-DMA hazard, no per-piece M0 copy); waits stay the loop's explicit ones
    const unsigned lw = lds_w;  // (named here: a nested generic lambda does not capture it otherwise)
    auto m0_set = [&](int slot, int j) __attribute__((always_inline)) {
      const unsigned m0v = lw + (unsigned)(slot * TILE + j * 1024);
      asm volatile("s_mov_b32 m0, %0" ::"s"(m0v) : "memory", "m0");
    };
    auto asm_dma = [&](const i32x4& r, unsigned v, int so) __attribute__((always_inline)) {
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(v), "s"(r), "s"(so) : "memory");
    };
    auto stage_a = [&](int j) __attribute__((always_inline)) {
      if (kAsmDma) {
        asm_dma(dra, vpa[j], (kt + 2) * kts_a);
      } else if (kFastK == 2) {  // per-piece voffset registers, one soffset per K-tile
        // plain locals as the builtin's operands (see the soffset note above dma_a)
        const unsigned v = vpa[j];
        const int so = (kt + 2) * kts_a;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, KFW4_LDS_PTR(smem + sf * TILE + (wid * PIECES + j) * 1024), 16,
                                                 v, so, 0, 0);
      }
      else dma_a(kt + 2, sf, j, false);
    };
    auto stage_b = [&](int j) __attribute__((always_inline)) {
      if (kAsmDma) {
        asm_dma(drb, vpb[j], (kt + 2) * kts_b);
      } else if (kFastK == 2) {
        const unsigned v = vpb[j];
        const int so = (kt + 2) * kts_b;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, KFW4_LDS_PTR(smem + sa0 * TILE + (wid * PIECES + j) * 1024), 16,
                                                 v, so, 0, 0);
      }
      else dma_b(kt + 2, sa0, j, false);
    };
    const unsigned long long t0 = stamp_k();
    // substep 0: MFMAs on F0(kt); read F1(kt); DMA A_{kt+2} -> free slot
#pragma unroll
    for (int m = 0; m < MF; ++m) {
      if (!(DIAG && ABL == 2) && m % RG == 0 && m / RG < 2 * NR) read_frag1(sa0, sb0, a1, b1, m / RG);
      if (kAsmDma && kStage && (m + 1) % DMA_EVERY == DMA_PHASE && (m + 1) / DMA_EVERY < PIECES)
        m0_set(sf, (m + 1) / DMA_EVERY);
      if (kStage && m % DMA_EVERY == DMA_PHASE && m / DMA_EVERY < PIECES) stage_a(m / DMA_EVERY);
      if (KFW4_PIN_MFMA) KFW4_PIN();
      mfma(acc[m / NR][m % NR], b0[m % NR], a0[m / NR]);
      if (KFW4_PIN_MFMA) KFW4_PIN();
    }
    const unsigned long long t1 = stamp_k();
    // tile kt+1 landed (only A_{kt+2} may still be in flight), F1(kt) in registers, then barrier:
    // after it tile kt's slots are free
    if (kStage) {
      if constexpr (BM == 256) __builtin_amdgcn_s_waitcnt(0x0078);  // vmcnt(8) expcnt(7) lgkmcnt(0)
      else __builtin_amdgcn_s_waitcnt(0x0074);                      // vmcnt(4) expcnt(7) lgkmcnt(0)
    } else {
      __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
    }
    // KFW4_PREBAR: the first substep-1 MFMAs (registers only) issue between the wait and the barrier,
    // so the matrix pipe has work while the waves meet; the reads of tile kt+1 start after it
#ifndef KFW4_PREBAR
#define KFW4_PREBAR 1
#endif
    constexpr int PB = KFW4_PREBAR;
    static_assert(PB + RG * (2 * NR - 1) < MF && PB <= DMA_PHASE, "pre-barrier MFMAs");
#pragma unroll
    for (int m = 0; m < PB; ++m) {
      KFW4_PIN();
      mfma(acc[m / NR][m % NR], b1[m % NR], a1[m / NR]);
      KFW4_PIN();
    }
    KFW4_FENCE();
    __builtin_amdgcn_s_barrier();
    KFW4_FENCE();
    KFW4_PIN();
    const unsigned long long t2 = stamp_k();
    // substep 1: MFMAs on F1(kt); read F0(kt+1); DMA B_{kt+2} -> A_kt's slot
#pragma unroll
    for (int m = PB; m < MF; ++m) {
      if (!(DIAG && ABL == 2) && kNext && (m - PB) % RG == 0 && (m - PB) / RG < 2 * NR)
        read_frag0(sa1, sb1, a0, b0, (m - PB) / RG);
      if (kAsmDma && kStage && (m + 1) % DMA_EVERY == DMA_PHASE && (m + 1) / DMA_EVERY < PIECES)
        m0_set(sa0, (m + 1) / DMA_EVERY);
      if (kStage && m % DMA_EVERY == DMA_PHASE && m / DMA_EVERY < PIECES) stage_b(m / DMA_EVERY);
      if (KFW4_PIN_MFMA) KFW4_PIN();
      mfma(acc[m / NR][m % NR], b1[m % NR], a1[m / NR]);
      if (KFW4_PIN_MFMA) KFW4_PIN();
    }
    const unsigned long long t3 = stamp_k();
    if (kNext) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): F0(kt+1) in registers
    KFW4_PIN();
    if (DIAG && KFW4_CHEAP_STAMPS) {
      // the stamps landed by this lgkmcnt(0) (the loop's own, except after the last tile); the empty
      // asm re-defines them after it so no arithmetic on them is hoisted above the wait
      if (!kNext) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      unsigned long long u0 = t0, u1 = t1, u2 = t2, u3 = t3;
      asm volatile("" : "+s"(u0), "+s"(u1), "+s"(u2), "+s"(u3)::"memory");
      seg[0] += u1 - u0;  // substep 0: MFMA issue + F1 reads + A DMAs
      seg[1] += u2 - u1;  // mid wait (vmcnt / lgkmcnt) + barrier
      seg[2] += u3 - u2;  // substep 1
      if (prev_t3) seg[3] += u0 - prev_t3;  // end lgkmcnt(0) + slot rotation to the next tile
      prev_t3 = u3;
    } else if (DIAG) {
      const unsigned long long t4 = stamp();
      seg[0] += t1 - t0;
      seg[1] += t2 - t1;
      seg[2] += t3 - t2;
      seg[3] += t4 - t3;
    }
  };
  // rotate after each tile: tile kt+1 -> current, tile kt+2 in (sf, sa0), B_kt's slot becomes free
  auto body = [&](int kt, auto do_stage, auto do_next) __attribute__((always_inline)) {
    body_g(kt, do_stage, do_next, sa0, sb0, sa1, sb1, sf);
    const int na = sf, nb = sa0;
    sf = sb0;
    sa0 = sa1;
    sb0 = sb1;
    sa1 = na;
    sb1 = nb;
  };
  if (DIAG) t_loop0 = stamp();
  int kt = 0;
  if (KFW4_UNROLL5 && !SK) {  // (stream-K: the unrolled loop spills beside the persistent schedule's state)
    // the ring's period is 5 tiles: (sa0, sb0, sa1, sb1, sf) = (0,1,2,3,4) -> (2,3,4,0,1) -> (4,0,1,2,3)
    // -> (1,2,3,4,0) -> (3,4,0,1,2) -> (0,1,2,3,4); state 0 again after each group of five
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using C2 = std::integral_constant<int, 2>;
    using C3 = std::integral_constant<int, 3>;
    using C4 = std::integral_constant<int, 4>;
    for (; kt + 6 < nk; kt += 5) {
      body_g(kt, T{}, T{}, C0{}, C1{}, C2{}, C3{}, C4{});
      body_g(kt + 1, T{}, T{}, C2{}, C3{}, C4{}, C0{}, C1{});
      body_g(kt + 2, T{}, T{}, C4{}, C0{}, C1{}, C2{}, C3{});
      body_g(kt + 3, T{}, T{}, C1{}, C2{}, C3{}, C4{}, C0{});
      body_g(kt + 4, T{}, T{}, C3{}, C4{}, C0{}, C1{}, C2{});
    }
  }
  for (; kt + 2 < nk; ++kt) body(kt, T{}, T{});
  if (kt + 1 < nk) {
    body(kt, F{}, T{});
    ++kt;
  }
  if (kt < nk) body(kt, F{}, F{});
  if (KFW4_PRIO) __builtin_amdgcn_s_setprio(0);
  if (DIAG) t_loop1 = stamp();
  // the asm MFMAs are opaque to the hazard recognizer: cover the MFMA -> v_accvgpr_read latency
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  // pin every accumulator behind the padding: the MFMAs are asm, so the compiler treats their AGPR
  // results as ready at issue and would otherwise hoist v_accvgpr_read of the last writes above the
  // s_nops (it did in the bias build of r2's w4d: stale sums). The empty asm "redefines" each one.
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int n = 0; n < NR; ++n) asm volatile("" : "+a"(acc[i][n]));
  };  // run_k

  // Epilogue. Lane (lr, lh) holds row lr, columns 4lh..4lh+3 of every 16x16 block n. For each pair
  // of blocks (n, n+1) one v_permlane16_swap per dword trades rows 1<->0 and 3<->2 of the lane
  // groups (cdna_hip_programming.md T21, 16-lane form), after which every lane holds 8 contiguous
  // columns: lh 0 -> block n cols 0-7, lh 1 -> block n+1 cols 0-7, lh 2 -> block n cols 8-15,
  // lh 3 -> block n+1 cols 8-15: one dwordx4 store per lane per pair. The lane id is re-derived
  // here (v_mbcnt) so no lane-derived VGPR has to survive the K loop.
  auto epilogue = [&]() __attribute__((always_inline)) {
  const int elane = lane_id_fresh();
  const int elr = elane & 15, elh = elane >> 4;
  // Output granularity og (elements, uniform): the widest store every lane's 8-column run allows,
  // from the alignment of C / Aux, ldc, the batch stride and N (n0 = min(n_lo, N - BN) is then a
  // multiple of og too, so the per-og-group edge mask is exact). og = 8 is the 16-B fast path; an odd
  // output (e.g. a 1500-wide C, or a column slice of a wider buffer) stores 8, 4 or 2 bytes.
  const unsigned gbits = (unsigned)(reinterpret_cast<uintptr_t>(C) | reinterpret_cast<uintptr_t>(HAS_AUX ? Aux : C)) |
                         (unsigned)(2 * (ldc | sc | N)) | 16u;
  const int og = (gbits & -gbits) / 2;  // 1, 2, 4 or 8
  // bias / residual fragments (4 columns at col = ... + 4 lh) as 8-B vectors when aligned for it
  const bool vec_in = og >= 4 && !((reinterpret_cast<uintptr_t>(HAS_BIAS ? bias : nullptr) |
                                   reinterpret_cast<uintptr_t>(HAS_RES ? R : nullptr)) & 7) &&
                      !(HAS_RES && ((ldr | sr) & 3));
  // the bias fragments of this lane's columns (n0 + wn*WT + 16n + 4lh; the same for every fragment
  // row i), loaded once up front: eight loads in flight instead of one load and wait per fragment
  bf16x4 bpre[NR];
  if (HAS_BIAS && vec_in) {
#pragma unroll
    for (int n = 0; n < NR; ++n) bpre[n] = *reinterpret_cast<const bf16x4*>(bias + n0 + wn * WT + n * 16 + elh * 4);
  }
  // VEC (compile time): bias / residual as 8-B vector loads (the fast path) or element loads
  // UNIT (compile time): alpha == 1, the scale is skipped (128 v_pk_mul_f32 per wave)
  auto finish = [&](auto VEC, auto UNIT, int i, int n, int m, uint2& pre_out) -> uint2 {
    constexpr bool vec = decltype(VEC)::value;
    const int col = n0 + wn * WT + n * 16 + elh * 4;
    float v[4];
    // the accumulator reads as volatile asm, so each path streams them next to their use instead of
    // the compiler hoisting all 256 reads above the path branch (256 extra live VGPRs + moves)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a;
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(a) : "a"(acc[i][n][r]));
      v[r] = a;
    }
    if constexpr (SK) {
      // stream-K owner: add the producers' fp32 partials (same fragment layout as acc)
      for (unsigned long long mk = (KFW4_SK_AB & 1) ? 0ull : sk_mask; mk; mk &= mk - 1) {
        const int slot = sk_base + __builtin_ctzll(mk) * sk_stride;
        // agent-coherent (sc1) loads: a producer on another XCD wrote them through its L2
        unsigned long long* pp = reinterpret_cast<unsigned long long*>(
            W + (long long)slot * BM * BN + (long long)(wm * WT + i * 16 + elr) * BN + wn * WT + n * 16 + elh * 4);
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const f32x2 lo = __builtin_bit_cast(f32x2, __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const f32x2 hi = __builtin_bit_cast(f32x2, __hip_atomic_load(pp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        v[0] += lo[0];
        v[1] += lo[1];
        v[2] += hi[0];
        v[3] += hi[1];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if constexpr (!decltype(UNIT)::value) v[r] *= alpha;
    if (HAS_BIAS) {
      if constexpr (vec) {
        const bf16x4 bb = bpre[n];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)bb[r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)bias[col + r];
      }
    }
    if (HAS_AUX) {
      bf16x4 p;
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = (__bf16)v[r];
      pre_out = __builtin_bit_cast(uint2, p);
    }
    if constexpr (KFW4_ACT_PK && (ACT == KFAMD_ACT_GELU_TANH || ACT == KFAMD_ACT_SILU)) {
      const kf32x2 lo = act2<ACT>(kf32x2{v[0], v[1]}), hi = act2<ACT>(kf32x2{v[2], v[3]});
      v[0] = lo.x;
      v[1] = lo.y;
      v[2] = hi.x;
      v[3] = hi.y;
    } else if (ACT != KFAMD_ACT_NONE) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], ACT);
    }
    if (HAS_RES) {
      const __bf16* rp = R + (long long)m * ldr + col;
      if constexpr (vec) {
        const bf16x4 rr = *reinterpret_cast<const bf16x4*>(rp);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)rr[r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)rp[r];
      }
    }
    // two v_cvt_pk_bf16_f32 (RNE), no per-element insert / perm shuffling
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 lo = __builtin_convertvector((f32x2{v[0], v[1]}), bf16x2);
    const bf16x2 hi = __builtin_convertvector((f32x2{v[2], v[3]}), bf16x2);
    return uint2{__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi)};
  };
  if constexpr (SPLIT == 1) {
    // raw fp32 partials, 4 consecutive columns per lane per block: W[z][m][n], ld N
    float* Wz = W + ((long long)blockIdx.z * gridDim.y + blockIdx.y) * (long long)M * N;
#ifndef KFW4_FULLLINE
#define KFW4_FULLLINE 1
#endif
    if (KFW4_FULLLINE && m0 == m_lo && n0 == n_lo) {
      // interior tile: whole 128-B lines per store, as the bf16 epilogue below. A block pair (n, n+1)
      // is 16 rows x 32 fp32; lane (lh, lr) holds row lr, 16 B at slot (n & 1) * 4 + lh; staged in the
      // wave's 2 KiB of the idle ring (slot c of row r at r * 128 + 16 * (c ^ ((r >> 1) & 7))) and read
      // back by rows (8 lanes per row)
      char* stage = smem + kEpiBase + wid * 2048;
      const int wsw = (elr >> 1) & 7;
      const int w0 = elr * 128 + 16 * (elh ^ wsw), w1 = elr * 128 + 16 * ((4 + elh) ^ wsw);
      const int rr = elane >> 3, rc = elane & 7;
      const int r0 = rr * 128 + 16 * (rc ^ ((rr >> 1) & 7)), r1 = (rr + 8) * 128 + 16 * (rc ^ (((rr + 8) >> 1) & 7));
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        float* wrow = Wz + (long long)(m0 + wm * WT + i * 16 + rr) * N + n0 + wn * WT + rc * 4;
#pragma unroll
        for (int n = 0; n < NR; n += 2) {
          *reinterpret_cast<f32x4*>(stage + w0) = acc[i][n];
          *reinterpret_cast<f32x4*>(stage + w1) = acc[i][n + 1];
          const f32x4 X = *reinterpret_cast<const f32x4*>(stage + r0);
          const f32x4 Y = *reinterpret_cast<const f32x4*>(stage + r1);
          *reinterpret_cast<f32x4*>(wrow + n * 16) = X;
          *reinterpret_cast<f32x4*>(wrow + 8LL * N + n * 16) = Y;
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int m = m0 + wm * WT + i * 16 + elr;
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        const int col = n0 + wn * WT + n * 16 + elh * 4;
        if (m >= m_lo && col >= n_lo)
          *reinterpret_cast<f32x4*>(Wz + (long long)m * N + col) = acc[i][n];
      }
    }
    return;
  }
  // 8 contiguous bf16 (4 dwords after the swap) at element offset o, column c0: one 16-B store (the
  // fast path), or og-groups for an odd output
  auto store16 = [&](__bf16* base, long long o, int c0, bool row_ok, uint4 d) {
    if (row_ok && c0 >= n_lo) *reinterpret_cast<uint4*>(base + o) = d;
  };
  // interior tile (not shifted at an M or N edge): every lane stores, no mask
  auto store_all = [&](__bf16* base, long long o, int, bool, uint4 d) { *reinterpret_cast<uint4*>(base + o) = d; };
  auto store_og = [&](__bf16* base, long long o, int c0, bool row_ok, uint4 d) {
    if (og == 8) {
      if (row_ok && c0 >= n_lo) *reinterpret_cast<uint4*>(base + o) = d;
    } else if (og == 4) {
      if (row_ok && c0 >= n_lo) *reinterpret_cast<uint2*>(base + o) = uint2{d.x, d.y};
      if (row_ok && c0 + 4 >= n_lo) *reinterpret_cast<uint2*>(base + o + 4) = uint2{d.z, d.w};
    } else if (og == 2) {
      const unsigned w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (row_ok && c0 + 2 * q >= n_lo) *reinterpret_cast<unsigned*>(base + o + 2 * q) = w[q];
    } else {
      const bf16x8 e = __builtin_bit_cast(bf16x8, d);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (row_ok && c0 + q >= n_lo) base[o + q] = e[q];
    }
  };
  const int swap_col = 16 * (elh & 1) + 8 * (elh >> 1);
  auto emit = [&](auto VEC, auto store, auto UNIT) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int m = m0 + wm * WT + i * 16 + elr;
      const bool row_ok = m >= m_lo;
      // one row pointer per i; the n blocks are immediate offsets from it
      __bf16* crow = C + ((long long)m * ldc + n0 + wn * WT + swap_col);
      __bf16* xrow = HAS_AUX ? Aux + ((long long)m * ldc + n0 + wn * WT + swap_col) : nullptr;
#pragma unroll
      for (int n = 0; n < NR; n += 2) {
        uint2 pp{0, 0}, pq{0, 0};
        uint2 p = finish(VEC, UNIT, i, n, m, pp), q = finish(VEC, UNIT, i, n + 1, m, pq);
        const auto sx = __builtin_amdgcn_permlane16_swap(p.x, q.x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(p.y, q.y, false, false);
        const int c0 = n0 + wn * WT + n * 16 + swap_col;
        store(crow, n * 16, c0, row_ok, uint4{sx[0], sy[0], sx[1], sy[1]});
        if (HAS_AUX) {
          const auto ax = __builtin_amdgcn_permlane16_swap(pp.x, pq.x, false, false);
          const auto ay = __builtin_amdgcn_permlane16_swap(pp.y, pq.y, false, false);
          store(xrow, n * 16, c0, row_ok, uint4{ax[0], ay[0], ax[1], ay[1]});
        }
      }
    }
  };
  // Interior tiles (C and the pre-activation output alike): every 16-B store covers 8 WHOLE 128-B lines (8 rows x
  // 64 columns, consecutive lanes on consecutive 16-B chunks of a row) instead of 16 half lines: the
  // CU's store path takes those in ~72 % of the time (epilogue 8.2 k -> 5.9 k cycles with the store
  // layout alone, profiles/r4_gemm_isa). After the permlane16 swap lane (lh, lr) holds row lr, 16 B at
  // column swap_col(lh) of its block pair's 32-column span; the pairs (n, n+1) and (n+2, n+3) of one
  // fragment row make a 16 x 64 span, which each wave stages in its own 2 KiB of the idle LDS ring
  // (no wave reads the ring after the last tile's mid barrier) and reads back row-major. Row r's 16-B
  // slot c sits at r * 128 + 16 * (c ^ ((r >> 1) & 7)): the writes (16 rows, one slot each per 16
  // lanes) and the reads (two rows of 8 slots per 16 lanes) both cover 16 distinct bank quads.
  auto emit_fullline = [&](auto UNIT) {
    static_assert(NR % 4 == 0, "full-line stores: two block pairs per span");
    char* stage = smem + kEpiBase + wid * 2048;
    // write side: this lane's row lr, slots ch(lh) (pair n) and 4 + ch(lh) (pair n+2); ch = 2*(lh&1) + (lh>>1)
    const int ch = 2 * (elh & 1) + (elh >> 1);
    const int wsw = (elr >> 1) & 7;
    const int w0 = elr * 128 + 16 * (ch ^ wsw), w1 = elr * 128 + 16 * ((4 + ch) ^ wsw);
    // read side: rows t/8 (X) and 8 + t/8 (Y), slot t % 8
    const int rr = elane >> 3, rc = elane & 7;
    const int r0 = rr * 128 + 16 * (rc ^ ((rr >> 1) & 7)), r1 = (rr + 8) * 128 + 16 * (rc ^ (((rr + 8) >> 1) & 7));
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int m = m0 + wm * WT + i * 16 + elr;
      __bf16* xrow = C + ((long long)(m0 + wm * WT + i * 16 + rr) * ldc + n0 + wn * WT + rc * 8);
#pragma unroll
      for (int n = 0; n < NR; n += 4) {
        uint4 d[2], x[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint2 pp{0, 0}, pq{0, 0};
          const uint2 p = finish(T{}, UNIT, i, n + 2 * h, m, pp), q = finish(T{}, UNIT, i, n + 2 * h + 1, m, pq);
          const auto sx = __builtin_amdgcn_permlane16_swap(p.x, q.x, false, false);
          const auto sy = __builtin_amdgcn_permlane16_swap(p.y, q.y, false, false);
          d[h] = uint4{sx[0], sy[0], sx[1], sy[1]};
          if (HAS_AUX) {
            const auto ax = __builtin_amdgcn_permlane16_swap(pp.x, pq.x, false, false);
            const auto ay = __builtin_amdgcn_permlane16_swap(pp.y, pq.y, false, false);
            x[h] = uint4{ax[0], ay[0], ax[1], ay[1]};
          }
        }
        *reinterpret_cast<uint4*>(stage + w0) = d[0];
        *reinterpret_cast<uint4*>(stage + w1) = d[1];
        if (HAS_AUX) {  // the pre-activation output, through its own 2 KiB
          *reinterpret_cast<uint4*>(stage + 8192 + w0) = x[0];
          *reinterpret_cast<uint4*>(stage + 8192 + w1) = x[1];
        }
        const uint4 X = *reinterpret_cast<const uint4*>(stage + r0);
        const uint4 Y = *reinterpret_cast<const uint4*>(stage + r1);
        *reinterpret_cast<uint4*>(xrow + n * 16) = X;
        *reinterpret_cast<uint4*>(xrow + 8 * ldc + n * 16) = Y;
        if (HAS_AUX) {
          const long long ao = (long long)(xrow - C);
          const uint4 XA = *reinterpret_cast<const uint4*>(stage + 8192 + r0);
          const uint4 YA = *reinterpret_cast<const uint4*>(stage + 8192 + r1);
          *reinterpret_cast<uint4*>(Aux + ao + n * 16) = XA;
          *reinterpret_cast<uint4*>(Aux + ao + 8 * ldc + n * 16) = YA;
        }
      }
    }
  };
  // Interior tiles with a residual: the residual is read as whole lines too. The scattered 8-B
  // fragment-order loads finish() makes touch 16 half-filled lines per instruction, and the load
  // path is charged per line like the store path (an out-projection forward, K = 2048, spent ~40 k
  // cycles outside its K loop, profiles/r4_train_trace). Here each wave stages alpha / bias /
  // activation results as fp32 (a 16 x 64 span is 4 KiB: row r's 16-B chunk c at r * 256 +
  // 16 * (c ^ r), so writes and reads both spread over all banks), reads them back row-major (8
  // columns per lane), adds the residual loaded row-major (8 lanes per 128-B line; the loads are
  // issued before the LDS round trip) in fp32 as finish() does, and stores whole lines.
  auto pre_res = [&](auto UNIT, int i, int n) __attribute__((always_inline)) -> f32x4 {
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a;
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(a) : "a"(acc[i][n][r]));
      v[r] = a;
    }
    if constexpr (!decltype(UNIT)::value) v *= alpha;
    if (HAS_BIAS) {
      const bf16x4 bb = bpre[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += (float)bb[r];
    }
    if (ACT != KFAMD_ACT_NONE && !DACT) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], ACT);
    }
    return v;
  };
  auto emit_fullline_res = [&](auto UNIT) {
    static_assert(NR % 4 == 0, "full-line stores: four blocks per span");
    char* stage = smem + kEpiBase + wid * 4096;
    const int rr = elane >> 3, rc = elane & 7;
    const int ra0 = rr * 256 + 16 * ((2 * rc) ^ rr), ra1 = rr * 256 + 16 * ((2 * rc + 1) ^ rr);
    const int rb0 = (rr + 8) * 256 + 16 * ((2 * rc) ^ (rr + 8)), rb1 = (rr + 8) * 256 + 16 * ((2 * rc + 1) ^ (rr + 8));
    // DACT: this lane's column sums (rows rr and rr + 8 of every fragment row), 8 columns per span
    float csum[DACT ? NR / 4 : 1][8];
#pragma unroll
    for (int h = 0; h < (DACT ? NR / 4 : 1); ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) csum[h][e] = 0.f;
    // R (residual / pre-activation) rows of span sp = (fragment row i, 64-column half n / 4), issued
    // KFW4_RES_PD spans ahead of their use: one span's loads per use left the HBM latency exposed
    // once per span, 16 times per wave and tile (profiles/r5zg_dact2)
#ifndef KFW4_RES_PD
#define KFW4_RES_PD 2
#endif
    constexpr int SPW = NR / 4, NS = NR * SPW, PD = KFW4_RES_PD;
    bf16x8 rbuf[PD + 1][2];
    auto rload = [&](int sp) __attribute__((always_inline)) {
      const int i = sp / SPW, n = (sp % SPW) * 4;
      const __bf16* rrow = R + ((long long)(m0 + wm * WT + i * 16 + rr) * ldr + n0 + wn * WT + rc * 8);
      rbuf[sp % (PD + 1)][0] = *reinterpret_cast<const bf16x8*>(rrow + n * 16);
      rbuf[sp % (PD + 1)][1] = *reinterpret_cast<const bf16x8*>(rrow + 8 * ldr + n * 16);
    };
#pragma unroll
    for (int sp = 0; sp < PD && sp < NS; ++sp) rload(sp);
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const long long row = m0 + wm * WT + i * 16 + rr;
      __bf16* xrow = C + (row * ldc + n0 + wn * WT + rc * 8);
#pragma unroll
      for (int n = 0; n < NR; n += 4) {
        const int sp = i * SPW + n / 4;
        if (sp + PD < NS) rload(sp + PD);
        const bf16x8 RX = rbuf[sp % (PD + 1)][0];
        const bf16x8 RY = rbuf[sp % (PD + 1)][1];
#pragma unroll
        for (int nn = 0; nn < 4; ++nn)
          *reinterpret_cast<f32x4*>(stage + elr * 256 + 16 * ((4 * nn + elh) ^ elr)) = pre_res(UNIT, i, n + nn);
        const f32x4 xa = *reinterpret_cast<const f32x4*>(stage + ra0), xb = *reinterpret_cast<const f32x4*>(stage + ra1);
        const f32x4 ya = *reinterpret_cast<const f32x4*>(stage + rb0), yb = *reinterpret_cast<const f32x4*>(stage + rb1);
        bf16x8 X, Y;
        if constexpr (DACT) {
          // pairs: the packed-f32 act' (dact2), the product, one v_cvt_pk_bf16_f32 per pair; the
          // column sums add the fp32 products (the act-grad pass summed the bf16-rounded ones)
          typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
          float* cs = csum[n / 4];
          auto pair = [&](int e, float x0, float x1, float y0, float y1) __attribute__((always_inline)) {
            const kf32x2 gx = kf32x2{x0, x1} * dact2<ACT>(kf32x2{(float)RX[e], (float)RX[e + 1]});
            const kf32x2 gy = kf32x2{y0, y1} * dact2<ACT>(kf32x2{(float)RY[e], (float)RY[e + 1]});
            const bf16x2_t bx = __builtin_convertvector(gx, bf16x2_t), by = __builtin_convertvector(gy, bf16x2_t);
            X[e] = bx[0];
            X[e + 1] = bx[1];
            Y[e] = by[0];
            Y[e + 1] = by[1];
            const kf32x2 c2 = kf32x2{cs[e], cs[e + 1]} + gx + gy;
            cs[e] = c2.x;
            cs[e + 1] = c2.y;
          };
          pair(0, xa[0], xa[1], ya[0], ya[1]);
          pair(2, xa[2], xa[3], ya[2], ya[3]);
          pair(4, xb[0], xb[1], yb[0], yb[1]);
          pair(6, xb[2], xb[3], yb[2], yb[3]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            X[r] = (__bf16)(xa[r] + (float)RX[r]);
            X[4 + r] = (__bf16)(xb[r] + (float)RX[4 + r]);
            Y[r] = (__bf16)(ya[r] + (float)RY[r]);
            Y[4 + r] = (__bf16)(yb[r] + (float)RY[4 + r]);
          }
        }
        *reinterpret_cast<bf16x8*>(xrow + n * 16) = X;
        *reinterpret_cast<bf16x8*>(xrow + 8 * ldc + n * 16) = Y;
      }
    }
    if constexpr (DACT) {
      if (W != nullptr) {
        // sum over the 8 lanes of one column run (lane bits 3-5: row_ror:8 within a row, then the
        // row pairs and halves by v_permlane16 / 32 swaps); lanes 0-7 store the slab's partials
#pragma unroll
        for (int h = 0; h < NR / 4; ++h) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float v = csum[h][e];
            v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));
            auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
            v = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
            auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
            csum[h][e] = __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
          }
        }
        if (rr == 0) {
          float* wrow = W + ((long long)(m0 / WT) + wm) * N + n0 + wn * WT + rc * 8;
#pragma unroll
          for (int h = 0; h < NR / 4; ++h) {
            *reinterpret_cast<f32x4*>(wrow + 64 * h) = f32x4{csum[h][0], csum[h][1], csum[h][2], csum[h][3]};
            *reinterpret_cast<f32x4*>(wrow + 64 * h + 4) = f32x4{csum[h][4], csum[h][5], csum[h][6], csum[h][7]};
          }
        }
      }
    }
  };
  // the residual as 16-B rows (its own alignment; vec_in only asks for 8 B)
  const bool res16 = HAS_RES && !(reinterpret_cast<uintptr_t>(HAS_RES ? R : nullptr) & 15) && !((ldr | sr) & 7);
#ifndef KFW4_FULLLINE
#define KFW4_FULLLINE 1
#endif
  // uniform branches: interior tiles store unmasked straight-line 16-B stores, shifted edge tiles
  // mask per lane, an odd output takes the og path; only the path that runs is fetched
  if constexpr (DACT) {  // interior tiles only (host contract): one path
    if (alpha == 1.f) emit_fullline_res(T{});
    else emit_fullline_res(F{});
  } else if (og == 8 && vec_in) {
    if (m0 == m_lo && n0 == n_lo) {
      if constexpr (KFW4_FULLLINE && HAS_RES && !HAS_AUX && !SK) {  // (the stream-K owner adds partials in finish())
        if (res16) {
          if (alpha == 1.f) emit_fullline_res(T{});
          else emit_fullline_res(F{});
        } else {
          emit(T{}, store_all, F{});
        }
      } else if constexpr (KFW4_FULLLINE) {
        if (alpha == 1.f) emit_fullline(T{});
        else emit_fullline(F{});
      } else {
        if (alpha == 1.f) emit(T{}, store_all, T{});
        else emit(T{}, store_all, F{});
      }
    } else {
      emit(T{}, store16, F{});
    }
  } else {
    emit(F{}, store_og, F{});
  }
  };  // epilogue

  if constexpr (SK) {
    // ---- stream-K persistent schedule (batch 1) -------------------------------------------------
    const int G = gridDim.x, KT = nk, koff_full = koff;
    const int T_dp = nwg - nwg % G;
    auto set_tile = [&](int w) __attribute__((always_inline)) {
      const int gg = w / per_group, fm = gg * kGroupM;
      const int gmm = min(tiles_m - fm, kGroupM);
      const int tm_ = fm + (w % per_group) % gmm, tn_ = (w % per_group) / gmm;
      m_lo = tm_ * BM;
      n_lo = tn_ * BN;
      m0 = min(m_lo, M - BM);
      n0 = min(n_lo, N - BN);
    };
    auto set_k = [&](int k0, int k1) __attribute__((always_inline)) {  // K-tiles [k0, k1) of the current tile
      const long long kofs = koff_full + (long long)kBK * k0;
      const __bf16* a = A_in + (LA == 0 ? (long long)m0 * lda + kofs : (long long)m0 + kofs * lda);
      const __bf16* b = B_in + (LB == 0 ? (long long)n0 * ldb + kofs : (long long)n0 + kofs * ldb);
      ra = __builtin_amdgcn_make_buffer_rsrc((void*)a, (short)0, nrec, kRsrcWord3);
      rb = __builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, nrec, kRsrcWord3);
      if (kAsmDma) {
        dra = make_desc(a);
        drb = make_desc(b);
      }
      nk = k1 - k0;
      koff = k0 == 0 ? koff_full : 0;  // only the tile's first K tile is partial
    };
    // zero the accumulators when `zero` is set, in place: an MFMA of zero fragments with C = 0 writes
    // the AGPRs. The branch sits inside the asm, so every accumulator has one unconditional def per
    // work item: a def under a branch gives the accumulators a phi at the join, which the allocator
    // resolves through VGPR copies of all 256 (and spills). Each asm pads its MFMAs' write latency
    // itself: the hazard recognizer cannot see into it, and a compiler copy of an accumulator
    // placed right after it read the previous tile's value (stale r = 0 elements, r3 sk_diag).
    static_assert(NR % 4 == 0, "zero_acc_if: 4 accumulators per asm");
    auto zero_acc_if = [&](int zero) __attribute__((always_inline)) {
      const bf16x8 z = {};
#pragma unroll
      for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int n = 0; n < NR; n += 4)
          asm volatile(
              "s_cmp_eq_u32 %4, 0\n\ts_cbranch_scc1 1f\n\t"
              "v_mfma_f32_16x16x32_bf16 %0, %5, %5, 0\n\tv_mfma_f32_16x16x32_bf16 %1, %5, %5, 0\n\t"
              "v_mfma_f32_16x16x32_bf16 %2, %5, %5, 0\n\tv_mfma_f32_16x16x32_bf16 %3, %5, %5, 0\n\t"
              "s_nop 7\n\ts_nop 7\n\ts_nop 7\n1:"
              : "+a"(acc[i][n]), "+a"(acc[i][n + 1]), "+a"(acc[i][n + 2]), "+a"(acc[i][n + 3])
              : "s"(zero), "v"(z)
              : "scc");
    };
    // one fp32 partial tile per producer unit, lane layout = the accumulator fragments
    auto partial_at = [&](int slot, int i, int n) __attribute__((always_inline)) -> float* {
      const int el = lane_id_fresh();
      return W + (long long)slot * BM * BN + (long long)(wm * WT + i * 16 + (el & 15)) * BN + wn * WT + n * 16 +
             (el >> 4) * 4;
    };
    // Schedule. The rem = T % G tiles past the whole waves are cut into S = kper K-splits each; in a
    // partition (below) unit u = j * n + t (split j of its t-th tile, split-major) goes to the
    // partition's block u % Gx, round u / Gx. Split-major keeps a round's blocks on the same K range
    // of their tiles, so they share A / B panels in L2 like the data-parallel waves. The last split's
    // block owns the tile; splits 0..S-2 store fp32 partials (slot u) and raise
    // flag[u]. An owner waits only for smaller units (same or earlier rounds, whose producers never
    // wait), so a co-resident grid cannot deadlock; a partial that misses the deadline is recomputed
    // by the owner on top of its accumulators.
    // One work loop, one unconditional run_k per item (the K loop and the epilogue are inlined once).
    // kper < 0: test mode, producers publish a flag value no owner accepts (every owner takes the
    // deadline path and recomputes the producers' splits)
    const int rem = nwg - T_dp, S = kper < 0 ? -kper : kper;
    const unsigned pub = kper < 0 ? ~sk_epoch : sk_epoch;
    // XCD-aware: the leftover tiles are cut into P = 8 contiguous ranges (neighbours in the grouped
    // raster share A / B panels) and range x is run by the blocks b % 8 == x, which the dispatcher
    // places on one XCD (one L2). Round-robin over all blocks spread a tile's panel-sharing
    // neighbours over all 8 L2s and ran HBM-bound. Only locality rests on the placement: every unit
    // still runs exactly once, on whichever CU its block lands.
    const int P = (G % 8 == 0 && rem >= 8) ? 8 : 1;
    const int part = blockIdx.x % P, Gx = G / P;
    const int t_begin = (int)((long long)part * rem / P);
    const int nx = (int)((long long)(part + 1) * rem / P) - t_begin;
    const int units = nx * S;
    int dp_j = blockIdx.x, u = blockIdx.x / P;
    int coll_j = S, coll_t = 0;  // an owner's next producer split to collect
    int fb_j = -1;               // a producer split to recompute (deadline missed)
    int cur_u = 0;
    auto split_k = [&](int j) __attribute__((always_inline)) { set_k((int)((long long)j * KT / S), (int)((long long)(j + 1) * KT / S)); };
    sk_stride = rem;
    while (true) {
      int role;  // 0: epilogue now, 1: producer, 2: owner (collect, then epilogue)
      int zero = 1;
      if (fb_j >= 0) {
        split_k(fb_j);
        fb_j = -1;
        zero = 0;
        role = 2;
      } else if (dp_j < T_dp) {  // whole waves: plain tiles
        sk_mask = 0;
        set_tile(xcd_remap(dp_j, T_dp));
        set_k(0, KT);
        role = 0;
        dp_j += G;
      } else if (u < units) {
        const int jj = u / nx, t = t_begin + (u - jj * nx);
        sk_mask = 0;
        set_tile(T_dp + t);
        split_k(jj);
        cur_u = jj * rem + t;  // partial slot / flag word
        if (S == 1) {
          role = 0;
        } else if (jj < S - 1) {
          role = 1;
        } else {
          role = 2;
          coll_j = 0;
          coll_t = t;
          sk_base = t;
        }
        u += Gx;
      } else {
        break;
      }
      zero_acc_if(zero);
      __syncthreads();  // the previous item's fragment reads are done before the ring refills
      run_k(std::false_type{});
      if (role == 1) {
#pragma unroll
        for (int i = 0; i < NR; ++i)
#pragma unroll
          for (int n = 0; n < NR; ++n) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[r]) : "a"(acc[i][n][r]));
            typedef float f32x2 __attribute__((ext_vector_type(2)));
            unsigned long long* pp = reinterpret_cast<unsigned long long*>(partial_at(cur_u, i, n));
            if (!(KFW4_SK_AB & 1)) {
              __hip_atomic_store(pp, __builtin_bit_cast(unsigned long long, (f32x2{v[0], v[1]})), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
              __hip_atomic_store(pp + 1, __builtin_bit_cast(unsigned long long, (f32x2{v[2], v[3]})), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
            }
          }
        // The partials and flags move as agent-scope relaxed atomics (sc1: written through / read past
        // the XCD's L2), so no agent-scope fence is needed: a release / acquire fence writes back /
        // invalidates the whole L2 of the XCD, evicting the A / B panels every other block on it is
        // streaming (that made each split cost about a whole tile). Completion of this wave's stores,
        // then the barrier, orders them before the flag.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(sk_flags + cur_u, pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      if (role == 2) {
        while (coll_j < S - 1) {
          const int ob = coll_j * rem + coll_t;
          __syncthreads();
          if (tid == 0) {
            int ok = 0;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (true) {
              if ((KFW4_SK_AB & 2) ||
                  __hip_atomic_load(sk_flags + ob, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == sk_epoch) {
                ok = 1;
                break;
              }
              if (__builtin_amdgcn_s_memrealtime() - t0 > kSkTimeoutTicks) break;
              __builtin_amdgcn_s_sleep(4);
            }
            *reinterpret_cast<volatile __attribute__((address_space(3))) int*>(KFW4_LDS_PTR(smem)) = ok;  // ring idle
          }
          __syncthreads();
          const int ok = __builtin_amdgcn_readfirstlane(
              *reinterpret_cast<volatile __attribute__((address_space(3))) int*>(KFW4_LDS_PTR(smem)));
          if (!ok) {  // producer not (yet) resident: its split becomes this block's next item
            fb_j = coll_j++;
            break;
          }
          sk_mask |= 1ull << coll_j;
          ++coll_j;
        }
        if (fb_j >= 0) continue;
      }
      epilogue();
    }
    return;
  }
  if constexpr (PO) {
    // ---- persistent, overlapped (batch 1, whole K): block b runs tiles b, b + G, b + 2G, ... of the
    // XCD-remapped order (G % 8 == 0 keeps every tile of a block on its XCD's contiguous chunk). The
    // next tile's first two K tiles are DMA'd before this tile's epilogue, so their latency and the
    // ring refill hide under its stores; no block boundary between tiles.
    const int G = gridDim.x;
    auto set_tile = [&](int w) __attribute__((always_inline)) {
      const int gg = w / per_group, fm = gg * kGroupM;
      const int gmm = min(tiles_m - fm, kGroupM);
      const int tm_ = fm + (w % per_group) % gmm, tn_ = (w % per_group) / gmm;
      m_lo = tm_ * BM;
      n_lo = tn_ * BN;
      m0 = min(m_lo, M - BM);
      n0 = min(n_lo, N - BN);
    };
    auto set_operands = [&]() __attribute__((always_inline)) {
      const __bf16* a = A_in + (LA == 0 ? (long long)m0 * lda + ka : (long long)m0 + ka * lda);
      const __bf16* b = B_in + (LB == 0 ? (long long)n0 * ldb + ka : (long long)n0 + ka * ldb);
      ra = __builtin_amdgcn_make_buffer_rsrc((void*)a, (short)0, nrec, kRsrcWord3);
      rb = __builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, nrec, kRsrcWord3);
      if (kAsmDma) {
        dra = make_desc(a);
        drb = make_desc(b);
      }
    };
    static_assert(NR % 4 == 0, "zero_acc: 4 accumulators per asm");
    auto zero_acc = [&]() __attribute__((always_inline)) {
      // an MFMA of zero fragments with C = 0 writes each AGPR (one unconditional def per tile, so the
      // loop-carried accumulators stay in AGPRs); the asm pads the VALU -> MFMA operand hazard of the
      // zero fragment's v_mov (invisible to the hazard recognizer) and its own write latency
      const bf16x8 z = {};
#pragma unroll
      for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int n = 0; n < NR; n += 4)
          asm volatile(
              "s_nop 4\n\tv_mfma_f32_16x16x32_bf16 %0, %4, %4, 0\n\tv_mfma_f32_16x16x32_bf16 %1, %4, %4, 0\n\t"
              "v_mfma_f32_16x16x32_bf16 %2, %4, %4, 0\n\tv_mfma_f32_16x16x32_bf16 %3, %4, %4, 0\n\t"
              "s_nop 7\n\ts_nop 7\n\ts_nop 7"
              : "=a"(acc[i][n]), "=a"(acc[i][n + 1]), "=a"(acc[i][n + 2]), "=a"(acc[i][n + 3])
              : "v"(z));
    };
    int j = blockIdx.x;  // the kernel prologue set this block's first tile (wg = xcd_remap(j, nwg))
    issue_prologue();
    while (true) {
      run_k(std::true_type{});
      const int jn = j + G;
      const bool more = jn < nwg;
      const int cm0 = m0, cn0 = n0, cmlo = m_lo, cnlo = n_lo;
      int nm0 = 0, nn0 = 0, nmlo = 0, nnlo = 0;
      if (more) {
        set_tile(xcd_remap(jn, nwg));
        set_operands();
        nm0 = m0, nn0 = n0, nmlo = m_lo, nnlo = n_lo;
        m0 = cm0, n0 = cn0, m_lo = cmlo, n_lo = cnlo;
        __syncthreads();  // every wave's last fragment reads of this tile are done before the ring refills
        issue_prologue();
      }
      epilogue();
      if (!more) break;
      m0 = nm0, n0 = nn0, m_lo = nmlo, n_lo = nnlo;
      j = jn;
      zero_acc();
    }
    return;
  }
  run_k(std::false_type{});
  if constexpr (SPLIT == 2) {
    // ---- split-K fixup: publish this split's partial, the last split to arrive finishes the tile ----
#ifndef KFW4_FIX_AB
#define KFW4_FIX_AB 0  // timing ablations (tools/fix_ab.py builds): 1 no partial stores, 2 no partial reads, 4 no sc1
#endif
    constexpr int kFixPol = (KFW4_FIX_AB & 4) ? 0 : 16;  // sc1
    const int el = lane_id_fresh();
    const long long tile_id = (long long)blockIdx.y * nwg_all + grp_base + wg;
    constexpr long long kPerTile = (long long)BM * BN;  // floats
    const long long zstride = (long long)gridDim.y * nwg_all * kPerTile;
    const unsigned lane_off = (unsigned)(wid * (NR * NR * 1024) + el * 16);
    {
      __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(W + (long long)blockIdx.z * zstride + tile_id * kPerTile), (short)0, kNumRecords, kRsrcWord3);
#pragma unroll
      for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int n = 0; n < NR; ++n) {
          i32x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float a;
            asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(a) : "a"(acc[i][n][r]));
            v[r] = __builtin_bit_cast(int, a);
          }
          // sc1: written through to the agent's coherence point, visible to a reader on another XCD
          if (!(KFW4_FIX_AB & 1)) __builtin_amdgcn_raw_buffer_store_b128(v, rw, lane_off, (i * NR + n) * 1024, kFixPol);
        }
    }
    // this block's partial is complete at agent scope before it counts itself in
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    volatile __attribute__((address_space(3))) int* bc =
        reinterpret_cast<volatile __attribute__((address_space(3))) int*>(KFW4_LDS_PTR(smem + kSlots * TILE - 16));
    if (tid == 0) *bc = (int)__hip_atomic_fetch_add(sk_flags + tile_id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int arrived = __builtin_amdgcn_readfirstlane(*bc);
    if (arrived != (int)gridDim.z - 1) return;
    // last split: every other partial is in; rearm the counter for the next launch on this stream
    if (tid == 0) __hip_atomic_store(sk_flags + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // one split at a time, two fragment rows of loads in flight (row i + 1 is requested before row i
    // is added); the scheduling barriers keep the compiler from hoisting every row's loads at once,
    // which spilled them to scratch behind vmcnt(0) waits
    for (int z = 0; z < ((KFW4_FIX_AB & 2) ? 0 : (int)gridDim.z); ++z) {
      if (z == (int)blockIdx.z) continue;
      __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(W + (long long)z * zstride + tile_id * kPerTile), (short)0, kNumRecords, kRsrcWord3);
      i32x4 t[2][NR];
#pragma unroll
      for (int n = 0; n < NR; ++n) t[0][n] = __builtin_amdgcn_raw_buffer_load_b128(rz, lane_off, n * 1024, kFixPol);
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        if (i + 1 < NR) {
#pragma unroll
          for (int n = 0; n < NR; ++n)
            t[(i + 1) & 1][n] = __builtin_amdgcn_raw_buffer_load_b128(rz, lane_off, ((i + 1) * NR + n) * 1024, kFixPol);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int n = 0; n < NR; ++n) acc[i][n] += __builtin_bit_cast(f32x4, t[i & 1][n]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
      for (int n = 0; n < NR; ++n) asm volatile("" : "+a"(acc[i][n]));
  }
  epilogue();
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

// Shape/alignment contract shared by the launchers (returns KFAMD_OK or an error code):
//  A/B: 16-B aligned bases, leading dims / batch strides in multiples of 8 elements; a K-contiguous
//  operand needs K % 8, a k-major A needs M % 8, a k-major B needs N % 8; M, N >= BM; the 32-bit
//  buffer offsets must cover a block's operand span. C/Aux/bias/R: bf16-aligned, any N and ldc (the
//  epilogue takes its element-wise path when they are off the 16-B grid).
inline int check_shape(int la, int lb, int BM, const void* A, const void* B, const void* C, const void* bias,
                       const void* R, const void* Aux, int M, int N, int K, long long lda, long long ldb,
                       long long ldc, long long ldr, long long sa, long long sb, long long sc, long long sr) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (M < BM || N < BM || K <= 0) return KFAMD_EINVAL;
  if (lb == 1 && N % 8) return KFAMD_EINVAL;
  if ((la == 0 || lb == 0) && K % 8) return KFAMD_EINVAL;
  if (la == 1 && M % 8) return KFAMD_EINVAL;
  if (la == 0 ? lda < K : lda < M) return KFAMD_EINVAL;
  if (lb == 0 ? ldb < K : ldb < N) return KFAMD_EINVAL;
  if (ldc < N || (R && ldr < N)) return KFAMD_EINVAL;
  auto al2 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 1) == 0; };
  if (!al16(A) || !al16(B) || !al2(C) || (Aux && !al2(Aux))) return KFAMD_EALIGN;
  if (lda % 8 || ldb % 8 || sa % 8 || sb % 8) return KFAMD_EALIGN;
  if ((bias && !al2(bias)) || (R && !al2(R))) return KFAMD_EALIGN;
  // buffer offsets: L=0 spans BM rows of ld; L=1 spans K rows of ld (voffset + soffset < 2^31)
  const long long span_a = la == 0 ? ((long long)BM * lda + kBK) * 2 : ((long long)K + kBK) * lda * 2;
  const long long span_b = lb == 0 ? ((long long)BM * ldb + kBK) * 2 : ((long long)K + kBK) * ldb * 2;
  if (span_a >= (1LL << 31) || span_b >= (1LL << 31)) return KFAMD_EINVAL;
  return KFAMD_OK;
}

}  // namespace
}  // namespace kfw4
