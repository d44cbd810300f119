// attention_bf16.hip — flash attention forward + backward for gfx950 (bf16 I/O, fp32 softmax).
//
// The in-notebook model's attention (models/gpt.py) without the N x N score matrix and without
// torch's aotriton (Triton-generated) kernels: every product runs on v_mfma_f32_32x32x16_bf16,
// the online softmax in fp32 registers, K/V tiles staged through a swizzled LDS image.
//
// Layout and lane maps (cdna_hip_programming.md §3, "An accumulator tile as the next MFMA's
// operand"): a 32x32 accumulator has its column on the lane (lane & 31) and its rows in the 16
// registers, row(reg, half) = (reg & 3) + 8 * (reg >> 2) + 4 * half. Every product is oriented
// so that the NEXT product sums over the accumulator's row index, which lets the accumulator
// (converted to bf16 pairwise) be that product's operand with no lane movement:
//
//   forward, per wave = 32 query rows, per 64-key tile:
//     S^T[key][q]  = K . Q^T          A = K rows (LDS, ds_read_b128), B = Q (registers)
//     O^T[d][q]   += V^T . P^T        A = V columns (LDS, ds_read_b64_tr_b16), B = P^T = the S^T
//                                     accumulator in bf16 (query on the lane: the online-softmax
//                                     max / sum / rescale of a row stay in its lane pair)
//   backward, per wave = 32 keys, per 32-query tile (keys on the lane):
//     S[q][key]   = Q . K^T - lse/scale    (the row constant preloaded into the accumulator)
//     dP[q][key]  = dO . V^T - delta       (delta = rowsum(dO * O), preloaded the same way)
//     dV^T[d][key] += dO^T . P             A = dO columns (tr reads), B = P accumulator
//     dK^T[d][key] += Q^T . dS             A = Q columns (tr reads),  B = dS accumulator
//     dQ[q][d]    += dS . K                dS crosses LDS once as a [key][q] image (tr reads for
//                                          the A operand), K columns by tr reads; one wave per
//                                          32-column d slice, f32 atomics into a workspace
//
// LDS images: one swizzle per head dim serves both the row reads (ds_read_b128 of a 16-B chunk
// by 32 different rows) and the transposed reads (ds_read_b64_tr_b16 of 4 consecutive rows by 32
// columns) without bank conflicts (T2 / T10): 16-B chunk ch of row r sits at chunk
//   D = 128 (256-B rows): ch ^ (((r & 3) << 2) | ((r >> 2) & 3))
//   D =  64 (128-B rows): ch ^ g((r >> 1) & 7),  g(x) = ((x & 1) << 2) | (x >> 1)
//
// Tensors are [B][H][T][D] views with element strides (b, h, t) and a contiguous head dim, so the
// fused QKV projection output [B][T][3][H][D] is read in place and the output / gradients are
// written straight into [B][T][H][D] / [B][T][3][H][D] (no transposes around the kernel).
// Causal masking is key <= query. The forward's workgroups run heaviest query block first; the
// backward's key blocks are heaviest first already (block 0 sees every query).
//
// Counterpart in the reference: none (its notebook images ship the framework's own attention);
// SURVEY §7.1C rules out Triton on the hot path.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kfamd_kernels.h"
#include "wave_ops.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr float kLog2e = 1.4426950408889634f;

struct AttnShape {
  int B, H, T;
  float scale;
  // element strides (b, h, t) of q, k, v, o, do, dq, dk, dv
  long long s[8][3];
};

enum { TQ = 0, TK = 1, TV = 2, TO = 3, TDO = 4, TDQ = 5, TDK = 6, TDV = 7 };

__device__ __forceinline__ long long base_off(const AttnShape& a, int t, int b, int h) {
  return b * a.s[t][0] + h * a.s[t][1];
}

// bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"): the
// blocks dealt to one XCD (bid % 8 equal) get consecutive logical ids, so a head's blocks share L2
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Work order (KFATT_LPT). A causal pass's blocks differ in work: query block i of the forward sees
// i + 1 key tiles, key block i of the backward sees the queries from i on. The hardware deals
// workgroups to the 8 XCDs round-robin (bid % 8) and each XCD starts its share in bid order, so a
// head-major order left the heaviest blocks of an XCD's last heads to start when the rest was done
// (makespan 1.5x the mean at 8 heads x 16 blocks on an XCD's 64 slots). Here XCD x owns heads
// [x BH/8, (x+1) BH/8) and walks them in groups of G heads, the fewest whose blocks fill its slots:
// the heaviest rank of every head of the group first (longest-processing-time order), the group's
// K / V shared in the XCD's L2. rank 0 = the heaviest block. Other head counts: the plain order.
#ifndef KFATT_LPT
#define KFATT_LPT 1
#endif
struct BlockId {
  int bh, rank;
};
__device__ __forceinline__ BlockId block_order(int bid, int nblk, int BH, int slots) {
  if (KFATT_LPT && (BH & 7) == 0) {
    const int hpx = BH >> 3, xcd = bid & 7, i = bid >> 3;
    int G = 1;
    while (G < hpx && (G * nblk < slots || hpx % G != 0)) ++G;
    const int gs = G * nblk, g = i / gs, j = i - g * gs;
    return {xcd * hpx + g * G + j % G, j / G};
  }
  const int nwg = nblk * BH;
  const int lid = (nwg & 7) == 0 ? xcd_remap(bid, nwg) : bid;
  return {lid / nblk, lid % nblk};
}

template <int D>
__device__ __forceinline__ int swz(int row, int ch) {
  if constexpr (D == 128) {
    return ch ^ (((row & 3) << 2) | ((row >> 2) & 3));
  } else {
    const int x = (row >> 1) & 7;
    return ch ^ (((x & 1) << 2) | (x >> 1));
  }
}

// byte offset of 16-B chunk ch of row `row` in an image of D-element bf16 rows
template <int D>
__device__ __forceinline__ int img_off(int row, int ch) {
  return row * (D * 2) + (swz<D>(row, ch) << 4);
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// v_exp_f32 as is: the libm exp2f wraps it in a denormal range reduction (v_cmp, v_cndmask, v_ldexp
// per call) that softmax does not need — a result below 2^-126 is 0 for a probability
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ uint32_t pack2(float x, float y) {
  const bf16x2 v = __builtin_convertvector((f32x2){x, y}, bf16x2);
  return __builtin_bit_cast(uint32_t, v);
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ds_read_b64_tr_b16 at an LDS byte offset: 4 consecutive rows x 16 columns per 16-lane group,
// lane i of the group receives column i (row q in element q)
__device__ __forceinline__ s16x4 tr_read(const char* smem, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + byte_off));
}

__device__ __forceinline__ bf16x8 join(s16x4 lo, s16x4 hi) {
  const short __attribute__((ext_vector_type(8))) v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 lds_row(const char* smem, int byte_off) {
  return *reinterpret_cast<const bf16x8*>(smem + byte_off);
}

__device__ __forceinline__ u32x4 gload16(const __bf16* p) { return *reinterpret_cast<const u32x4*>(p); }

// KFATT_BUF: row-guarded loads and the dQ atomics as raw buffer operations over one (b, h) slice
// whose range ends at row T: a row past T reads as zero / is dropped by the address unit, so the
// inner loops carry no per-row branches (a divergent `if (row < T)` around each load / atomic split
// the loops into ~30 basic blocks and cost the scheduler and the register allocator). The host
// requires every slice's extent below 2^31 bytes (32-bit buffer offsets).
#ifndef KFATT_BUF
#define KFATT_BUF 1
#endif
#ifndef KFATT_ABL
#define KFATT_ABL 0  // timing ablations (tools/attn_ab.py builds): 1 = dQ atomics dropped
#endif
// Backward schedule (profiles/r5q_attn_split, tools/attn_ab.py variants, one box, 2 rounds each):
//   gpt-1b 4x16x2048x128 bwd: register-staged + dQ atomics 570 us; + LDS-DMA staging 557-568; the
//   atomics dropped (timing only) 525-545; the atomic-free dQ kernel 482 (-15 %); D = 64
//   (16x12x2048): 827-832 -> 557-559 (-33 %: at D = 64 the fp32 atomics are a third of the pass);
//   1x16x4096x128: 489-495 -> 417-419. The forward with LDS-DMA K / V was 2-7 % slower: kept off.
#ifndef KFATT_DQ_SPLIT
#define KFATT_DQ_SPLIT 1  // dQ by the atomic-free attn_bwd_dq_split kernel (recomputes S and dP)
#endif
#ifndef KFATT_DMA
#define KFATT_DMA 1  // backward Q / dO tiles by LDS-DMA (attn_bwd stage_dma)
#endif
#ifndef KFATT_DKDV8
#define KFATT_DKDV8 1  // D = 128 dK / dV with 8 waves (two per SIMD), attn_bwd_dkdv8 (profiles/r5w_attn_dkdv8)
#endif
#ifndef KFATT_DKDV8_64
#define KFATT_DKDV8_64 1  // D = 64 with the 8-wave dK / dV kernel too (16x12x2048x64: 516 -> 485 us)
#endif
#ifndef KFATT_DQ_DELTA
#define KFATT_DQ_DELTA 1  // the dQ kernel computes delta (runs first; no separate prologue kernel): gpt-1b bwd -5 %
#endif
#ifndef KFATT_FWD_OFFS
#define KFATT_FWD_OFFS 1  // forward: LDS read offsets precomputed per lane, buffers unrolled
#endif
#ifndef KFATT_FWD_PAIR
#define KFATT_FWD_PAIR 1  // causal forward: heavy + light query block per workgroup (attn_fwd PAIR, profiles/r5zm_fpair)
#endif
#ifndef KFATT_FWD_NW
#define KFATT_FWD_NW 4  // forward workgroup: 4 waves (two workgroups per CU) or 8 (one; A/B runs)
#endif
#ifndef KFATT_DKDV_ABL
#define KFATT_DKDV_ABL 0  // attn_bwd_dkdv8 timing ablations (tools/attn_ab.py builds; wrong results)
#endif
#ifndef KFATT_DQ_PAIR
#define KFATT_DQ_PAIR 0  // the same for the dQ kernel (attn_bwd_dq_split PAIR)
#endif
#ifndef KFATT_FWD_WIDE
#define KFATT_FWD_WIDE 1  // the forwards store O in whole 16-B rows per lane (store_rows16, T21)
#endif
#ifndef KFATT_FWD_DMA
#define KFATT_FWD_DMA 0  // forward K / V tiles by LDS-DMA (attn_fwd stage_dma)
#endif
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slice_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, int byte_off, int soff = 0) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, soff, 0));
}

// LDS-DMA as inline asm (KFATT_DMA): the compiler, seeing a buffer_load ... lds builtin, waits
// vmcnt(0) before later LDS reads it cannot prove disjoint (it did, mid-tile, before the dV / dK tr
// reads: the next tile's DMA latency exposed). The kernel's own waits cover the pieces instead.
// The descriptor is an SGPR quad (base, base_hi | stride 0, records, gfx9 raw-buffer word 3); M0 holds
// the wave's 1 KiB LDS destination (lane L writes +16 L); s_nop 1 covers the M0 -> LDS-DMA hazard.
// (No compiler-generated code in this file uses M0: LDS instructions do not on gfx9+, and every
// LDS-DMA here is this asm, so M0 is not listed as clobbered — hipcc treats it as reserved.)
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 slice_desc(const void* base, long long bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  return i32x4{__builtin_amdgcn_readfirstlane((int)(unsigned)a), __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff)),
               (int)bytes, 0x00020000};
}
__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// voff: the lane's byte offset (VGPR); soff: a wave-uniform byte offset (SGPR: the tile's row offset,
// so the per-lane part is computed once outside the loop)
__device__ __forceinline__ void dma16(const i32x4& desc, unsigned lds, int voff, int soff = 0) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 1\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(desc),
                  "s"(__builtin_amdgcn_readfirstlane(soff)) : "memory");
}
__device__ __forceinline__ void dma4(const i32x4& desc, unsigned lds, int voff, int soff = 0) {  // lane L -> +4 L
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 1\n\tbuffer_load_dword %1, %2, %3 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(desc),
                  "s"(__builtin_amdgcn_readfirstlane(soff)) : "memory");
}

// The A operand of a product whose k index is an accumulator's row (the permuted order of
// §3): element j of lane half hh is row kbase + 8 * (j >> 2) + 4 * hh + (j & 3) of the operand's
// k dimension, column `col` (this lane's row of the A operand). Read as two tr reads of 4 rows.
// Address of lane (group g, index i = 4 qq + p): row kbase + 4 hh + qq (+ 8), columns
// col0 + 4 p .. +3 with col0 = the 16-column half of the 32-column tile this group covers.
template <int D>
__device__ __forceinline__ bf16x8 tr_operand(const char* smem, int kbase, int colbase, int lane) {
  const int g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3, hh = lane >> 5;
  const int col = colbase + 16 * (g & 1) + 4 * p;
  const int r0 = kbase + 4 * hh + qq;
  const int off0 = img_off<D>(r0, col >> 3) + 8 * (p & 1);
  const int off1 = img_off<D>(r0 + 8, col >> 3) + 8 * (p & 1);
  return join(tr_read(smem, off0), tr_read(smem, off1));
}

// Whole 16-B row stores of an accumulator in the O^T layout (cdna_hip_programming.md T21): lane
// (r, hh) holds row r's columns 32 n + 8 g + 4 hh .. +3 as acc[n][4 g .. 4 g + 3], g = 0..3. For each
// column-group pair (2k, 2k + 1) the lanes r and r + 32 trade halves with v_permlane32_swap, after
// which lane hh holds the 8 contiguous columns 8 (2k + hh) .. +7: 2 ND dwordx4 stores per lane
// instead of 4 ND dwordx2. Every lane must execute it (the swap needs EXEC full): `ok` guards only
// the stores (rows past T).
template <int ND>
__device__ __forceinline__ void store_rows16(__bf16* row, const f32x16 (&acc)[ND], float sc, bool ok, int hh) {
#pragma unroll
  for (int n = 0; n < ND; ++n)
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const int g0 = 2 * k2, g1 = g0 + 1;
      uint32_t p[2], q[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const auto sw = __builtin_amdgcn_permlane32_swap(pack2(acc[n][4 * g0 + 2 * x] * sc, acc[n][4 * g0 + 2 * x + 1] * sc),
                                                         pack2(acc[n][4 * g1 + 2 * x] * sc, acc[n][4 * g1 + 2 * x + 1] * sc),
                                                         false, false);
        p[x] = sw[0];
        q[x] = sw[1];
      }
      if (ok) *reinterpret_cast<u32x4*>(row + 32 * n + 8 * (g0 + hh)) = (u32x4){p[0], p[1], q[0], q[1]};
    }
}

// ------------------------------------------------------------------------------------------------
// forward: one workgroup = 4 waves = 128 query rows of one (b, h); 64-key K/V tiles through a
// double-buffered LDS image, register-staged (issued before the tile's products, written after)
// ------------------------------------------------------------------------------------------------
constexpr int FQ = 128, FK = 64;

// PAIR (causal, an even number of query blocks, KFATT_FWD_PAIR): one workgroup runs query blocks
// nq - 1 - i and i one after the other, nq + 1 key tiles for every workgroup, half the grid
// The forwards' two MFMA phases with every LDS operand read RA MFMAs ahead of its use, the order
// pinned by sched groups (KFATT_FWD_RA, profiles/r6v_ra): the compiler's own order read each
// fragment one or two MFMAs early and waited on it there, so a wave paid an LDS round trip per
// k-step. S^T = K Q^T: MFMA i is k-step i / 2, key half t = i & 1.
template <int D, int RA>
__device__ __forceinline__ void qk_ra(const char* kimg, const int (&koff)[D / 16], const bf16x8 (&qf)[D / 16],
                                      f32x16 (&s)[2]) {
  constexpr int NM = D / 8;
  bf16x8 kf[NM];
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    if (i == 0)
#pragma unroll
      for (int u = 0; u < RA; ++u) kf[u] = lds_row(kimg + 32 * (u & 1) * D * 2, koff[u >> 1]);
    if (i + RA < NM) kf[i + RA] = lds_row(kimg + 32 * ((i + RA) & 1) * D * 2, koff[(i + RA) >> 1]);
    s[i & 1] = mfma32(kf[i], qf[i >> 1], s[i & 1]);
  }
  __builtin_amdgcn_sched_group_barrier(0x100, RA, 0);  // DS reads
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    if (i + RA < NM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
  }
}

// O += P V: MFMA i is d tile n = i / 4, key half t = (i / 2) & 1, 16-key step s2 = i & 1, its A
// operand two transposed V reads
template <int D, int RA>
__device__ __forceinline__ void pv_ra(const char* vimg, const int (&voff0)[D / 32], const int (&voff1)[D / 32],
                                      const uint32_t (&pf)[2][2][4], f32x16 (&oa)[D / 32]) {
  constexpr int NM = D / 8;
  auto rd = [&](int i) __attribute__((always_inline)) {
    const char* base = vimg + (32 * ((i >> 1) & 1) + 16 * (i & 1)) * D * 2;
    return join(tr_read(base, voff0[i >> 2]), tr_read(base, voff1[i >> 2]));
  };
  bf16x8 vf[NM];
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    if (i == 0)
#pragma unroll
      for (int u = 0; u < RA; ++u) vf[u] = rd(u);
    if (i + RA < NM) vf[i + RA] = rd(i + RA);
    const int t = (i >> 1) & 1, s2 = i & 1;
    const u32x4 pw = {pf[t][s2][0], pf[t][s2][1], pf[t][s2][2], pf[t][s2][3]};
    oa[i >> 2] = mfma32(vf[i], __builtin_bit_cast(bf16x8, pw), oa[i >> 2]);
  }
  __builtin_amdgcn_sched_group_barrier(0x100, 2 * RA, 0);
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    if (i + RA < NM) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  }
}

#ifndef KFATT_FWD4_RA
#define KFATT_FWD4_RA 2  // attn_fwd (4 waves; D = 64 and small grids): KFATT_FWD_RA's pinned reads
#endif

template <int D, bool CAUSAL, bool PAIR = false, int NW = 4>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void attn_fwd(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                   const __bf16* __restrict__ v, __bf16* __restrict__ o,
                                                   float* __restrict__ lse, AttnShape a) {
  constexpr int KS = D / 16;           // k-steps of the QK^T product
  constexpr int ND = D / 32;           // 32-wide d tiles of O
  constexpr int CH = D / 8;            // 16-B chunks per row
  constexpr int NT = 64 * NW, FQW = 32 * NW;  // threads, query rows per workgroup (NW waves x 32)
  constexpr int NCH = FK * CH / NT;    // chunks per thread per K (and per V) tile
  constexpr int TILE = FK * D * 2;     // bytes of one K (or V) tile image
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // [buf][K, V]

  const int nq = (a.T + FQW - 1) / FQW;
  const BlockId bo = block_order(blockIdx.x, PAIR ? nq / 2 : nq, a.H * a.B, NW == 4 ? 64 : 32);  // workgroups per XCD
  const int bh = bo.bh, h = bh % a.H, b = bh / a.H;
#pragma unroll 1
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  if (PAIR && pass) __syncthreads();  // the first block's last tile reads are done before the LDS is refilled
  const int qblk = pass ? bo.rank : nq - 1 - bo.rank;  // the heaviest (most keys) first

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int q0 = qblk * FQW, qw = q0 + 32 * w, qrow = qw + r;
  const int T = a.T;

  const __bf16* qb = q + base_off(a, TQ, b, h);
  const __bf16* kb = k + base_off(a, TK, b, h);
  const __bf16* vb = v + base_off(a, TV, b, h);
  const long long qt = a.s[TQ][2], kt = a.s[TK][2], vt = a.s[TV][2];

  bf16x8 qf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    u32x4 x = {0u, 0u, 0u, 0u};
    if (qrow < T) x = gload16(qb + qrow * qt + kk * 16 + 8 * hh);
    qf[kk] = __builtin_bit_cast(bf16x8, x);
  }

  const int ntiles = CAUSAL ? min((T + FK - 1) / FK, (q0 + FQW) / FK) : (T + FK - 1) / FK;

  constexpr bool kDma = KFATT_FWD_DMA && KFATT_BUF;
  u32x4 kreg[kDma ? 1 : NCH], vreg[kDma ? 1 : NCH];
  const auto rk = slice_rsrc(kb, 2LL * T * kt), rv = slice_rsrc(vb, 2LL * T * vt);
  const i32x4 dk_desc = slice_desc(kb, 2LL * T * kt), dv_desc = slice_desc(vb, 2LL * T * vt);
  // KFATT_DMA: K / V tiles by LDS-DMA (as the backward's stage_dma): no staging registers
  constexpr int NPC = TILE / 1024 / NW;
  // LDS-DMA pieces: the wave index as a uniform value, each piece's per-lane source offset computed
  // once (image chunk sc of row `row` holds source chunk sc ^ swz(row, 0))
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int dvo_k[NPC], dvo_v[NPC];
#pragma unroll
  for (int i = 0; i < NPC; ++i) {
    const int byte = (wu * NPC + i) * 1024 + lane * 16;
    const int row = byte / (D * 2), ch = ((byte % (D * 2)) >> 4) ^ swz<D>(row, 0);
    dvo_k[i] = 2 * (row * (int)kt + ch * 8);
    dvo_v[i] = 2 * (row * (int)vt + ch * 8);
  }
  auto stage_dma = [&](int tile, int buf) {
    const int k0 = tile * FK;
    char* kimg = smem + buf * 2 * TILE;
    char* vimg = kimg + TILE;
#pragma unroll
    for (int i = 0; i < NPC; ++i) {
      dma16(dk_desc, lds_addr(kimg + (wu * NPC + i) * 1024), dvo_k[i], 2 * k0 * (int)kt);
      dma16(dv_desc, lds_addr(vimg + (wu * NPC + i) * 1024), dvo_v[i], 2 * k0 * (int)vt);
    }
  };
  auto stage_load = [&](int tile) {
    const int k0 = tile * FK;
#pragma unroll
    for (int i = 0; i < (kDma ? 0 : NCH); ++i) {
      const int c = tid + NT * i, row = c / CH, ch = c % CH;
      const int key = k0 + row;
      if constexpr (KFATT_BUF) {
        // lane part in the voffset, the tile's row offset in the (scalar) soffset: no VALU per load
        kreg[i] = bload16(rk, 2 * (row * (int)kt + ch * 8), 2 * k0 * (int)kt);
        vreg[i] = bload16(rv, 2 * (row * (int)vt + ch * 8), 2 * k0 * (int)vt);
      } else {
        u32x4 xk = {0u, 0u, 0u, 0u}, xv = {0u, 0u, 0u, 0u};
        if (key < T) {
          xk = gload16(kb + key * kt + ch * 8);
          xv = gload16(vb + key * vt + ch * 8);
        }
        kreg[i] = xk;
        vreg[i] = xv;
      }
    }
  };
  auto stage_write = [&](int buf) {
    char* kimg = smem + buf * 2 * TILE;
    char* vimg = kimg + TILE;
#pragma unroll
    for (int i = 0; i < (kDma ? 0 : NCH); ++i) {
      const int c = tid + NT * i, row = c / CH, ch = c % CH;
      const int off = img_off<D>(row, ch);
      *reinterpret_cast<u32x4*>(kimg + off) = kreg[i];
      *reinterpret_cast<u32x4*>(vimg + off) = vreg[i];
    }
  };

  const float c = a.scale * kLog2e;
  float m = -INFINITY, l = 0.f;
  f32x16 oacc[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) oacc[n] = (f32x16){};

  if constexpr (kDma) {
    stage_dma(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  stage_load(0);
  stage_write(0);
  __syncthreads();

  // per-lane LDS offsets of every operand read, computed once (KFATT_FWD_OFFS): the row parts that
  // vary per read (t, k-step, buffer) are compile-time and ride in the ds_read immediate, so the loop
  // body carries no address arithmetic (it was ~80 VALU per 64-key tile, a third of the VALU stream)
  int koff[KS], voff0[ND], voff1[ND];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) koff[kk] = img_off<D>(r, 2 * kk + hh);  // + 32 t rows: swz bits unchanged
  {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
    const int r0 = 4 * hh + qq;  // + kbase (a multiple of 16): swz bits unchanged
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const int col = 32 * n + 16 * (g & 1) + 4 * pp;
      voff0[n] = img_off<D>(r0, col >> 3) + 8 * (pp & 1);
      voff1[n] = img_off<D>(r0 + 8, col >> 3) + 8 * (pp & 1);
    }
  }
  // the tile loop unrolled over the two buffers: the buffer offset is compile-time too
  auto tile_body = [&](int j, auto BUFC) __attribute__((always_inline)) {
    constexpr int BUF = decltype(BUFC)::value;
    const int k0 = j * FK;
    const bool more = j + 1 < ntiles;
    if (more) {
      if constexpr (kDma) stage_dma(j + 1, 1 - BUF);
      stage_load(j + 1);
    }
    const char* kimg = smem + BUF * 2 * TILE;
    const char* vimg = kimg + TILE;
    // a wave whose 32 rows all precede the tile's first key has nothing to do (causal)
    if (!(CAUSAL && k0 > qw + 31)) {
      f32x16 sacc[2] = {(f32x16){}, (f32x16){}};
      if constexpr (KFATT_FWD4_RA > 0 && KFATT_FWD_OFFS) qk_ra<D, KFATT_FWD4_RA>(kimg, koff, qf, sacc);
      else
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 kf = KFATT_FWD_OFFS ? lds_row(kimg + 32 * t * D * 2, koff[kk])
                                           : lds_row(kimg, img_off<D>(32 * t + r, 2 * kk + hh));
          sacc[t] = mfma32(kf, qf[kk], sacc[t]);
        }
      }
      // masks: causal (key > query) on tiles that reach the wave's diagonal, key >= T on the tail
      const bool causal_mask = CAUSAL && k0 + FK - 1 > qw;
      if (causal_mask || k0 + FK > T) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int key = k0 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * hh;
            if ((CAUSAL && key > qrow) || key >= T) sacc[t][e] = -INFINITY;
          }
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) mx = fmaxf(mx, sacc[t][e]);
      mx = kfw::max_halves(mx);  // the row's other 32 keys (v_permlane32_swap; no LDS round trip)
      const float mn = fmaxf(m, mx);  // finite: the first tile holds key 0 <= every query
      // O and l are rescaled only when some row's max grew (exact: alpha == 1 otherwise); late in a
      // row's sweep that is the rare case, and the 64-register multiply is skipped
      const bool grew = __builtin_amdgcn_ballot_w64(mx > m) != 0;
      const float alpha = grew ? fast_exp2((m - mn) * c) : 1.f;
      m = mn;
      const float mc = mn * c;
      float rs = 0.f;
      uint32_t pf[2][2][4];  // [t][s][pair]: P^T as the B operand of PV
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int e = 0; e < 16; e += 2) {
          const float p0 = fast_exp2(fmaf(sacc[t][e], c, -mc));
          const float p1 = fast_exp2(fmaf(sacc[t][e + 1], c, -mc));
          rs += p0 + p1;
          pf[t][e >> 3][(e & 7) >> 1] = pack2(p0, p1);
        }
      }
      if (grew) {
        l = l * alpha + rs;
#pragma unroll
        for (int n = 0; n < ND; ++n) oacc[n] *= alpha;
      } else {
        l += rs;
      }
      if constexpr (KFATT_FWD4_RA > 0 && KFATT_FWD_OFFS) pv_ra<D, KFATT_FWD4_RA>(vimg, voff0, voff1, pf, oacc);
      else
#pragma unroll
      for (int n = 0; n < ND; ++n) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const bf16x8 vf = KFATT_FWD_OFFS ? join(tr_read(vimg + (32 * t + 16 * s) * D * 2, voff0[n]),
                                                    tr_read(vimg + (32 * t + 16 * s) * D * 2, voff1[n]))
                                               : tr_operand<D>(vimg, 32 * t + 16 * s, 32 * n, lane);
            const u32x4 pw = {pf[t][s][0], pf[t][s][1], pf[t][s][2], pf[t][s][3]};
            oacc[n] = mfma32(vf, __builtin_bit_cast(bf16x8, pw), oacc[n]);
          }
        }
      }
    }
    if (more) {
      if constexpr (kDma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next tile's pieces
      stage_write(1 - BUF);
    }
    __syncthreads();
  };
  for (int j = 0; j < ntiles; j += 2) {
    tile_body(j, std::integral_constant<int, 0>{});
    if (j + 1 < ntiles) tile_body(j + 1, std::integral_constant<int, 1>{});
  }

  // epilogue: lane (r, hh) holds row qrow, d = 32 n + (e & 3) + 8 (e >> 2) + 4 hh
  const float lt = kfw::sum_halves(l);
  const float inv = 1.f / lt;
  __bf16* ob = o + base_off(a, TO, b, h) + qrow * a.s[TO][2];
  if constexpr (KFATT_FWD_WIDE) {
    store_rows16<ND>(ob, oacc, inv, qrow < T, hh);
  } else if (qrow < T) {
#pragma unroll
    for (int n = 0; n < ND; ++n) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u32x2 v2 = {pack2(oacc[n][4 * g] * inv, oacc[n][4 * g + 1] * inv),
                          pack2(oacc[n][4 * g + 2] * inv, oacc[n][4 * g + 3] * inv)};
        *reinterpret_cast<u32x2*>(ob + 32 * n + 8 * g + 4 * hh) = v2;
      }
    }
  }
  if (qrow < T && hh == 0) lse[((long long)b * a.H + h) * T + qrow] = m * a.scale + logf(lt);
  }  // pass
}

// ------------------------------------------------------------------------------------------------
// forward, 8 waves x 32 query rows = 256 rows per workgroup, one workgroup per CU (KFATT_FWD_PP,
// profiles/r6d_attn_pp): two waves per SIMD share its matrix pipe, one K / V image per CU per tile
// instead of two (half the LDS stores and global loads of attn_fwd's two 128-row workgroups), and the
// hardware interleaves one wave's softmax VALU with the other's MFMAs. One barrier per tile.
// The running max is a reference that moves only when a row's scores pass it by more than
// KFATT_FWD_THR (log2 units; cdna_hip_programming.md T13): probabilities stay <= 2^THR (exact in the
// fp32 l and O, bf16 keeps its relative precision), and the 64-register O rescale runs only on
// those tiles instead of on nearly every early one (the tests force both branches: rule 26).
// K / V are loaded two tiles ahead (KFATT_FWD_PF2: a four-slot ring, two staging register sets;
// without it one tile ahead through a three-slot ring).
// Measured and not taken (tools/attn_ab.py, profiles/r6d_attn_pp): staggering waves 4-7 half a tile
// behind waves 0-3 (MI355X_MICROARCH.md "Two waves per SIMD" item 9): +7 % time; the QK^T of tile
// j + 1 issued beside softmax(j), Q moved to LDS to pay for the second S tile (T15): +6 %.
// ------------------------------------------------------------------------------------------------
#ifndef KFATT_FWD_PP
#define KFATT_FWD_PP 1  // forward by attn_fwd_pp (profiles/r6d_attn_pp)
#endif
#ifndef KFATT_FWD_THR
#define KFATT_FWD_THR 8.0f
#endif
#ifndef KFATT_FWD_FENCE
#define KFATT_FWD_FENCE 1  // scheduling fences between the QK^T / softmax / PV phases of attn_fwd_pp
#endif
#define FENCE() \
  do {                                                   \
    if (KFATT_FWD_FENCE) __builtin_amdgcn_sched_barrier(0); \
  } while (0)
#ifndef KFATT_FWD_PF2
#define KFATT_FWD_PF2 1  // K / V loads two tiles ahead (four-tile ring)
#endif
#ifndef KFATT_BWD_WIDE
#define KFATT_BWD_WIDE 1  // dQ / dK / dV in whole 16-B rows per lane (store_rows16)
#endif
#ifndef KFATT_FWD_PRIO
#define KFATT_FWD_PRIO 0  // attn_fwd_pp: static priority 1 for waves 4-7 (A/B knob)
#endif
#ifndef KFATT_FWD_PXP
#define KFATT_FWD_PXP 1  // attn_fwd_pp pairs: the light block's prologue loads issued under the heavy block's epilogue
#endif
#ifndef KFATT_FWD_ABL
#define KFATT_FWD_ABL 0  // timing ablations of attn_fwd_pp (tools/attn_ab.py; wrong results)
#endif
#ifndef KFATT_FWD_RA
#define KFATT_FWD_RA 2  // attn_fwd_pp: LDS reads pinned this many MFMAs ahead of their use (0: compiler order)
#endif
#ifndef KFATT_DQ_RA
#define KFATT_DQ_RA 0  // attn_bwd_dq_split (D = 128): LDS reads pinned this many MFMAs ahead (0: compiler order)
#endif
#ifndef KFATT_BWD_RA
#define KFATT_BWD_RA 0  // attn_bwd_dkdv8: LDS reads pinned this many MFMAs ahead (0: compiler order)
#endif
#ifndef KFATT_FWD_SPLIT
#define KFATT_FWD_SPLIT 0  // attn_fwd_pp softmax: row max and row sum as 4 independent chains
#endif

template <int D, bool CAUSAL, bool PAIR>
__global__ __launch_bounds__(512, 1) void attn_fwd_pp(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                      const __bf16* __restrict__ v, __bf16* __restrict__ o,
                                                      float* __restrict__ lse, AttnShape a) {
  constexpr int KS = D / 16, ND = D / 32, CH = D / 8;
  constexpr int NT = 512, FQW = 256;
  constexpr int NCH = FK * CH / NT;  // 16-B chunks per thread per K (and per V) tile
  constexpr int TILE = FK * D * 2;
  // K ring [NS][TILE] then V ring [NS][TILE]; the V ring's base VBASE rides in the V read offsets,
  // so every slot / row offset of a read fits the 16-bit ds_read immediate
  constexpr int NS = KFATT_FWD_PF2 ? 4 : 3, VBASE = NS * TILE;
  __shared__ __attribute__((aligned(16))) char smem[2 * NS * TILE];

  const int T = a.T;
  const int nq = (T + FQW - 1) / FQW, nta = (T + FK - 1) / FK;
  const BlockId bo = block_order(blockIdx.x, PAIR ? nq / 2 : nq, a.H * a.B, 32);  // one workgroup per CU
  const int bh = bo.bh, h = bh % a.H, b = bh / a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // the wave index as a uniform (scalar) value
  // KFATT_FWD_PRIO: waves 4-7, the second-dispatched half that loses every VALU arbitration to its
  // SIMD partner, at priority 1 for the whole kernel (MI355X_MICROARCH.md "Two waves per SIMD" item 4)
  if (KFATT_FWD_PRIO && wu >= 4) __builtin_amdgcn_s_setprio(1);

  const __bf16* qb = q + base_off(a, TQ, b, h);
  const __bf16* kb = k + base_off(a, TK, b, h);
  const __bf16* vb = v + base_off(a, TV, b, h);
  const long long qt = a.s[TQ][2], kt = a.s[TK][2], vt = a.s[TV][2];
  const auto rk = slice_rsrc(kb, 2LL * T * kt), rv = slice_rsrc(vb, 2LL * T * vt);
  const float c = a.scale * kLog2e;
  constexpr float THR = KFATT_FWD_THR;

  // per-lane LDS offsets (as attn_fwd KFATT_FWD_OFFS): tile row parts ride in the ds_read immediates
  int koff[KS], voff0[ND], voff1[ND];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) koff[kk] = img_off<D>(r, 2 * kk + hh);
  {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
    const int r0 = 4 * hh + qq;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const int col = 32 * n + 16 * (g & 1) + 4 * pp;
      voff0[n] = VBASE + img_off<D>(r0, col >> 3) + 8 * (pp & 1);
      voff1[n] = VBASE + img_off<D>(r0 + 8, col >> 3) + 8 * (pp & 1);
    }
  }
  u32x4 kreg[NCH], vreg[NCH];
  auto stage_load = [&](int tile) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cc = tid + NT * i, row = cc / CH, ch = cc % CH;
      kreg[i] = bload16(rk, 2 * (row * (int)kt + ch * 8), 2 * tile * FK * (int)kt);
      vreg[i] = bload16(rv, 2 * (row * (int)vt + ch * 8), 2 * tile * FK * (int)vt);
    }
  };
  auto stage_write = [&](int slot) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cc = tid + NT * i;
      const int off = img_off<D>(cc / CH, cc % CH);
      *reinterpret_cast<u32x4*>(smem + slot * TILE + off) = kreg[i];
      *reinterpret_cast<u32x4*>(smem + VBASE + slot * TILE + off) = vreg[i];
    }
  };
  auto qk = [&](const char* kimg, const bf16x8 (&qf)[KS], f32x16 (&s)[2]) __attribute__((always_inline)) {
    s[0] = (f32x16){};
    s[1] = (f32x16){};
    if constexpr (KFATT_FWD_RA > 0) {
      qk_ra<D, KFATT_FWD_RA>(kimg, koff, qf, s);
    } else {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int t = 0; t < 2; ++t) s[t] = mfma32(lds_row(kimg + 32 * t * D * 2, koff[kk]), qf[kk], s[t]);
    }
  };
  auto pv = [&](const char* vimg, const uint32_t (&pf)[2][2][4], f32x16 (&oa)[ND]) __attribute__((always_inline)) {
    if constexpr (KFATT_FWD_RA > 0) {
      pv_ra<D, KFATT_FWD_RA>(vimg, voff0, voff1, pf, oa);
      return;
    }
#pragma unroll
    for (int n = 0; n < ND; ++n)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 vf = join(tr_read(vimg + (32 * t + 16 * s2) * D * 2, voff0[n]),
                                 tr_read(vimg + (32 * t + 16 * s2) * D * 2, voff1[n]));
          const u32x4 pw = {pf[t][s2][0], pf[t][s2][1], pf[t][s2][2], pf[t][s2][3]};
          oa[n] = mfma32(vf, __builtin_bit_cast(bf16x8, pw), oa[n]);
        }
  };
  // causal / tail mask of the wave's S^T tile (keys from k0, rows from qw); a uniform branch
  auto mask = [&](f32x16 (&s)[2], int k0, int qw) __attribute__((always_inline)) {
    if ((CAUSAL && k0 + FK - 1 > qw) || k0 + FK > T) {
      const int lim = (CAUSAL ? min(qw + r, T - 1) : T - 1) - k0 - 4 * hh;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          if (32 * t + (e & 3) + 8 * (e >> 2) > lim) s[t][e] = -INFINITY;
    }
  };
  // online softmax of one S^T tile into P (bf16 pairs: the PV B operand) and l; O is rescaled when
  // some lane's reference max moved
  auto softmax = [&](const f32x16 (&s)[2], float& m, float& l, uint32_t (&pf)[2][2][4], f32x16 (&oa)[ND])
                     __attribute__((always_inline)) {
    float mx = -INFINITY;
    if constexpr (KFATT_FWD_SPLIT) {
      float mp[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) mp[e & 3] = fmaxf(mp[e & 3], s[t][e]);
      mx = fmaxf(fmaxf(mp[0], mp[1]), fmaxf(mp[2], mp[3]));
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) mx = fmaxf(mx, s[t][e]);
    }
    mx = kfw::max_halves(mx);
    const bool move = (mx - m) * c > THR;  // m = -inf on the first tile: moves
    const float mn = move ? mx : m;
    const float alpha = move ? fast_exp2((m - mn) * c) : 1.f;
    m = mn;
    const float mc = mn * c;
    float rp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        const float p0 = fast_exp2(fmaf(s[t][e], c, -mc));
        const float p1 = fast_exp2(fmaf(s[t][e + 1], c, -mc));
        rp[KFATT_FWD_SPLIT ? (e >> 1) & 3 : 0] += p0 + p1;
        pf[t][e >> 3][(e & 7) >> 1] = pack2(p0, p1);
      }
    const float rs = KFATT_FWD_SPLIT ? (rp[0] + rp[1]) + (rp[2] + rp[3]) : rp[0];
    l = l * alpha + rs;
    if (__builtin_amdgcn_ballot_w64(move) != 0) {
#pragma unroll
      for (int n = 0; n < ND; ++n) oa[n] *= alpha;
    }
  };

  bf16x8 qf[KS];
  auto load_q = [&](int qr) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      u32x4 x = {0u, 0u, 0u, 0u};
      if (qr < T) x = gload16(qb + qr * qt + kk * 16 + 8 * hh);
      qf[kk] = __builtin_bit_cast(bf16x8, x);
    }
  };
  // KFATT_FWD_PF2 staging: two register sets, tile j + 2 issued at tile j (see the tile loop)
  u32x4 kr2[NCH], vr2[NCH];
  auto ld = [&](int tile, u32x4 (&kr)[NCH], u32x4 (&vr)[NCH]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cc = tid + NT * i, row = cc / CH, ch = cc % CH;
      kr[i] = bload16(rk, 2 * (row * (int)kt + ch * 8), 2 * tile * FK * (int)kt);
      vr[i] = bload16(rv, 2 * (row * (int)vt + ch * 8), 2 * tile * FK * (int)vt);
    }
  };
  auto st = [&](int slot, const u32x4 (&kr)[NCH], const u32x4 (&vr)[NCH]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cc = tid + NT * i;
      const int off = img_off<D>(cc / CH, cc % CH);
      *reinterpret_cast<u32x4*>(smem + slot * TILE + off) = kr[i];
      *reinterpret_cast<u32x4*>(smem + VBASE + slot * TILE + off) = vr[i];
    }
  };
  // KFATT_FWD_PXP (pairs): the light block's Q and first two K / V tiles are issued when the heavy
  // block's tile loop ends, so their latency hides under its epilogue instead of stalling a second
  // prologue
  constexpr bool PXP = KFATT_FWD_PXP && KFATT_FWD_PF2 && PAIR;

#pragma unroll 1
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
    if (PAIR && pass) __syncthreads();  // the first block's last reads are done before the LDS is refilled
    const int qblk = pass ? bo.rank : nq - 1 - bo.rank;  // the heaviest first
    const int q0 = qblk * FQW, qw = q0 + 32 * wu, qrow = qw + r;
    const int ntiles = CAUSAL ? min(nta, (q0 + FQW) / FK) : nta;
    const int jl = CAUSAL ? min(ntiles - 1, (qw + 31) / FK) : ntiles - 1;  // this wave's last tile
    const bool pre = PXP && pass == 1;  // Q and tiles 0 / 1 already in flight

    if (!pre) load_q(qrow);
    f32x16 oacc[ND], S[2][2];
#pragma unroll
    for (int n = 0; n < ND; ++n) oacc[n] = (f32x16){};
    float m = -INFINITY, l = 0.f;
    uint32_t pf[2][2][4];
    // tile j sits in ring slot j % 3, compile-time in the unrolled loop (pv reads through
    // smem + slot * TILE, the V ring base riding in voff)
    if constexpr (KFATT_FWD_PF2) {
      // K / V two tiles ahead: tile j + 2's loads are issued at tile j into the register set tile j
      // used (written at tile j - 1), and tile j + 1's set is written at the end of tile j into the
      // slot of tile j - 3 (a four-tile ring: slot and set compile-time in the 4x unrolled loop)
      if (!pre) ld(0, kreg, vreg);
      st(0, kreg, vreg);
      if (!pre && 1 < ntiles) ld(1, kr2, vr2);
      __syncthreads();
      auto tile = [&](int j, auto SLC) __attribute__((always_inline)) {
        constexpr int SL = decltype(SLC)::value;  // j % 4; register set j & 1
        auto& kc = (SL & 1) ? kr2 : kreg;
        auto& vc = (SL & 1) ? vr2 : vreg;
        auto& kn = (SL & 1) ? kreg : kr2;
        auto& vn = (SL & 1) ? vreg : vr2;
        if ((KFATT_FWD_ABL & 1) == 0 && j + 2 < ntiles) ld(j + 2, kc, vc);
        if (j <= jl) {
          qk(smem + SL * TILE, qf, S[0]);
          mask(S[0], j * FK, qw);
          FENCE();
          softmax(S[0], m, l, pf, oacc);
          FENCE();
          pv(smem + SL * TILE, pf, oacc);
        }
        if ((KFATT_FWD_ABL & 1) == 0 && j + 1 < ntiles) st((SL + 1) % 4, kn, vn);
        if ((KFATT_FWD_ABL & 2) == 0) __syncthreads();
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      using I2 = std::integral_constant<int, 2>;
      using I3 = std::integral_constant<int, 3>;
      int j = 0;
#pragma unroll 1
      for (; j + 3 < ntiles; j += 4) {
        tile(j, I0{});
        tile(j + 1, I1{});
        tile(j + 2, I2{});
        tile(j + 3, I3{});
      }
      if (j < ntiles) tile(j, I0{});
      if (j + 1 < ntiles) tile(j + 1, I1{});
      if (j + 2 < ntiles) tile(j + 2, I2{});
    } else {
      stage_load(0);
      stage_write(0);
      __syncthreads();
      auto tile = [&](int j, auto SLC) __attribute__((always_inline)) {
        constexpr int SL = decltype(SLC)::value;
        const bool more = (KFATT_FWD_ABL & 1) == 0 && j + 1 < ntiles;  // ABL 1: no staging (timing only)
        if (more) stage_load(j + 1);
        if (j <= jl) {
          qk(smem + SL * TILE, qf, S[0]);
          mask(S[0], j * FK, qw);
          FENCE();
          softmax(S[0], m, l, pf, oacc);
          FENCE();
          pv(smem + SL * TILE, pf, oacc);
        }
        if (more) stage_write((SL + 1) % 3);
        if ((KFATT_FWD_ABL & 2) == 0) __syncthreads();  // ABL 2: no barrier (timing only)
      };
      int j = 0;
#pragma unroll 1
      for (; j + 2 < ntiles; j += 3) {
        tile(j, std::integral_constant<int, 0>{});
        tile(j + 1, std::integral_constant<int, 1>{});
        tile(j + 2, std::integral_constant<int, 2>{});
      }
      if (j < ntiles) tile(j, std::integral_constant<int, 0>{});
      if (j + 1 < ntiles) tile(j + 1, std::integral_constant<int, 1>{});
    }

    if (PXP && pass == 0) {  // the light block's Q and first K / V tiles, under this epilogue
      const int q0n = bo.rank * FQW;
      load_q(q0n + 32 * wu + r);
      ld(0, kreg, vreg);
      if (1 < (CAUSAL ? min(nta, (q0n + FQW) / FK) : nta)) ld(1, kr2, vr2);
    }

    // epilogue: lane (r, hh) holds row qrow, d = 32 n + (e & 3) + 8 (e >> 2) + 4 hh
    const float lt = kfw::sum_halves(l);
    const float inv = 1.f / lt;
    __bf16* ob = o + base_off(a, TO, b, h) + qrow * a.s[TO][2];
    if constexpr (KFATT_FWD_WIDE) {
      store_rows16<ND>(ob, oacc, inv, qrow < T, hh);
    } else if (qrow < T) {
#pragma unroll
      for (int n = 0; n < ND; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const u32x2 v2 = {pack2(oacc[n][4 * g] * inv, oacc[n][4 * g + 1] * inv),
                            pack2(oacc[n][4 * g + 2] * inv, oacc[n][4 * g + 3] * inv)};
          *reinterpret_cast<u32x2*>(ob + 32 * n + 8 * g + 4 * hh) = v2;
        }
    }
    if (qrow < T && hh == 0) lse[((long long)b * a.H + h) * T + qrow] = m * a.scale + logf(lt);
  }  // pass
}

// ------------------------------------------------------------------------------------------------
// backward prologue, per row [b][h][t]: nd = -sum_d dO * O and nl = -lse / scale (fp32), the two
// row constants of the backward in the form its products start from: S - lse / scale and dP - delta
// are the MFMA accumulators initialised with nl and nd (no negate / scale per element and tile)
// ------------------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_delta(const __bf16* __restrict__ o, const __bf16* __restrict__ dout,
                                                      const float* __restrict__ lse, float* __restrict__ nl,
                                                      float* __restrict__ nd, AttnShape a) {
  constexpr int LPR = D / 8;        // lanes per row (16 B each)
  constexpr int RPB = 256 / LPR;    // rows per block
  const long long nrows = (long long)a.B * a.H * a.T;
  const long long row = (long long)blockIdx.x * RPB + threadIdx.x / LPR;
  const int part = threadIdx.x % LPR;
  float s = 0.f;
  if (row < nrows) {
    const int t = (int)(row % a.T);
    const int h = (int)((row / a.T) % a.H);
    const int b = (int)(row / ((long long)a.T * a.H));
    const u32x4 x = gload16(o + base_off(a, TO, b, h) + t * a.s[TO][2] + part * 8);
    const u32x4 y = gload16(dout + base_off(a, TDO, b, h) + t * a.s[TDO][2] + part * 8);
    const bf16x8 xb = __builtin_bit_cast(bf16x8, x), yb = __builtin_bit_cast(bf16x8, y);
#pragma unroll
    for (int e = 0; e < 8; ++e) s = fmaf((float)xb[e], (float)yb[e], s);
  }
  s = kfw::group_sum<LPR>(s);
  if (row < nrows && part == 0) {
    nd[row] = -s;
    nl[row] = -lse[row] / a.scale;
  }
}

// ------------------------------------------------------------------------------------------------
// backward dQ without atomics (KFATT_DQ_SPLIT): the forward's structure with the log-sum-exp known.
// One workgroup = 4 waves = 128 query rows; 64-key K / V tiles by LDS-DMA into a double-buffered
// image; per tile S^T = K Q^T and dP^T = V dO^T (keys on registers, the lane's query on the column),
// P^T = exp(scale S - lse), dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T with dS^T straight from the
// registers as the B operand (the permuted k order, as P^T feeds PV in the forward). dQ is written
// once, scaled, in bf16: no fp32 workspace, no atomics, no conversion pass. Costs the S and dP
// products a second time (the dK / dV kernel computes them too).
// ------------------------------------------------------------------------------------------------
// DELTA (KFATT_DQ_DELTA): this kernel runs first and is also the backward's prologue: each lane's
// query row computes delta = sum_d dO * O from the dO fragments it holds anyway plus one pass over O,
// and writes nl / nd for the dK / dV kernel (lse, delta arrive raw; the separate prologue is gone)
// PAIR: as attn_fwd's (query blocks nq - 1 - i and i in one workgroup; KFATT_DQ_PAIR)
template <int D, bool CAUSAL, bool DELTA = false, bool PAIR = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_split(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                            const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                            const float* __restrict__ lse, const float* __restrict__ delta,
                                                            __bf16* __restrict__ dq, AttnShape a,
                                                            const __bf16* __restrict__ o, float* __restrict__ nl_out,
                                                            float* __restrict__ nd_out) {
  constexpr int KS = D / 16;
  constexpr int ND = D / 32;
  constexpr int CH = D / 8;
  constexpr int TILE = FK * D * 2;             // one K (or V) tile image
  constexpr int NPC = TILE / 1024 / 4;         // LDS-DMA pieces (1 KiB) per wave per image
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // [buf][K, V]

  const int T = a.T;
  const int nq = (T + FQ - 1) / FQ;
  const BlockId bo = block_order(blockIdx.x, PAIR ? nq / 2 : nq, a.H * a.B, 64);
  const int bh = bo.bh, h = bh % a.H, b = bh / a.H;
#pragma unroll 1
  for (int pass = 0; pass < (PAIR ? 2 : 1); ++pass) {
  if (PAIR && pass) __syncthreads();  // the first block's last LDS reads are done before the refill
  const int qblk = pass ? bo.rank : nq - 1 - bo.rank;  // the heaviest first
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int q0 = qblk * FQ, qw = q0 + 32 * w, qrow = qw + r;

  const __bf16* qb = q + base_off(a, TQ, b, h);
  const __bf16* kb = k + base_off(a, TK, b, h);
  const __bf16* vb = v + base_off(a, TV, b, h);
  const __bf16* dob = dout + base_off(a, TDO, b, h);
  const long long qt = a.s[TQ][2], kt = a.s[TK][2], vt = a.s[TV][2], dot = a.s[TDO][2];
  const auto rq = slice_rsrc(qb, 2LL * T * qt), rdo = slice_rsrc(dob, 2LL * T * dot);
  const i32x4 dk_desc = slice_desc(kb, 2LL * T * kt), dv_desc = slice_desc(vb, 2LL * T * vt);

  // this lane's query: Q and dO rows as the B operands, lse and delta (rows past T: zeros)
  bf16x8 qf[KS], dof[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    qf[kk] = __builtin_bit_cast(bf16x8, bload16(rq, 2 * (qrow * (int)qt + kk * 16 + 8 * hh)));
    dof[kk] = __builtin_bit_cast(bf16x8, bload16(rdo, 2 * (qrow * (int)dot + kk * 16 + 8 * hh)));
  }
  const long long rowbase = ((long long)b * a.H + h) * T;
  float nlc, nd_q;
  if constexpr (DELTA) {
    const auto ro = slice_rsrc(o + base_off(a, TO, b, h), 2LL * T * a.s[TO][2]);
    float dd = 0.f;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const bf16x8 of = __builtin_bit_cast(bf16x8, bload16(ro, 2 * (qrow * (int)a.s[TO][2] + kk * 16 + 8 * hh)));
#pragma unroll
      for (int e = 0; e < 8; ++e) dd = fmaf((float)of[e], (float)dof[kk][e], dd);
    }
    const float delta_q = kfw::sum_halves(dd);  // the row's other half of d (lane ^ 32)
    const float lq = qrow < T ? lse[rowbase + qrow] : 0.f;
    nlc = -lq * kLog2e;
    nd_q = -delta_q;
    if (hh == 0 && qrow < T) {
      nl_out[rowbase + qrow] = -lq / a.scale;
      nd_out[rowbase + qrow] = nd_q;
    }
  } else {
    // (lse / delta arrive as the prologue's nl = -lse / scale and nd = -delta)
    nlc = qrow < T ? lse[rowbase + qrow] * (a.scale * kLog2e) : 0.f;
    nd_q = qrow < T ? delta[rowbase + qrow] : 0.f;
  }

  const int ntiles = CAUSAL ? min((T + FK - 1) / FK, (q0 + FQ) / FK) : (T + FK - 1) / FK;
  // K / V tile `tile` -> image buffer `buf`, each lane fetching the chunk the swizzle puts at its slot
  // LDS-DMA pieces: the wave index as a uniform value, each piece's per-lane source offset computed
  // once (image chunk sc of row `row` holds source chunk sc ^ swz(row, 0))
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int dvo_k[NPC], dvo_v[NPC];
#pragma unroll
  for (int i = 0; i < NPC; ++i) {
    const int byte = (wu * NPC + i) * 1024 + lane * 16;
    const int row = byte / (D * 2), ch = ((byte % (D * 2)) >> 4) ^ swz<D>(row, 0);
    dvo_k[i] = 2 * (row * (int)kt + ch * 8);
    dvo_v[i] = 2 * (row * (int)vt + ch * 8);
  }
  auto stage_dma = [&](int tile, int buf) {
    const int k0 = tile * FK;
    char* kimg = smem + buf * 2 * TILE;
    char* vimg = kimg + TILE;
#pragma unroll
    for (int i = 0; i < NPC; ++i) {
      dma16(dk_desc, lds_addr(kimg + (wu * NPC + i) * 1024), dvo_k[i], 2 * k0 * (int)kt);
      dma16(dv_desc, lds_addr(vimg + (wu * NPC + i) * 1024), dvo_v[i], 2 * k0 * (int)vt);
    }
  };

  const float c = a.scale * kLog2e;
  f32x16 dqacc[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) dqacc[n] = (f32x16){};

  if (ntiles > 0) stage_dma(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // per-lane LDS read offsets computed once; the tile loop unrolled over the two buffers (as the forward)
  int koff[KS], voff0[ND], voff1[ND];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) koff[kk] = img_off<D>(r, 2 * kk + hh);
  {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const int col = 32 * n + 16 * (g & 1) + 4 * pp;
      voff0[n] = img_off<D>(4 * hh + qq, col >> 3) + 8 * (pp & 1);
      voff1[n] = img_off<D>(4 * hh + qq + 8, col >> 3) + 8 * (pp & 1);
    }
  }
  auto tile_body = [&](int j, auto BUFC) __attribute__((always_inline)) {
    constexpr int BUF = decltype(BUFC)::value;
    const int k0 = j * FK;
    if (j + 1 < ntiles) stage_dma(j + 1, 1 - BUF);  // buffer 1 - BUF was last read before the barrier
    const char* kimg = smem + BUF * 2 * TILE;
    const char* vimg = kimg + TILE;
    if (!(CAUSAL && k0 > qw + 31)) {
      f32x16 sacc[2] = {(f32x16){}, (f32x16){}}, dpacc[2] = {(f32x16){}, (f32x16){}};
      if constexpr (KFATT_DQ_RA > 0 && D == 128) {
        // KFATT_DQ_RA: the K / V fragment of MFMA i + RA read before MFMA i issues (as attn_fwd_pp);
        // MFMA i: k-step i / 4, t = (i / 2) & 1, S for even i, dP for odd
        constexpr int RA = KFATT_DQ_RA, NM = 4 * KS;
        bf16x8 fa[NM];
        auto rd = [&](int i) __attribute__((always_inline)) {
          fa[i] = lds_row(((i & 1) ? vimg : kimg) + 32 * ((i >> 1) & 1) * D * 2, koff[i >> 2]);
        };
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i == 0)
#pragma unroll
            for (int u = 0; u < RA; ++u) rd(u);
          if (i + RA < NM) rd(i + RA);
          const int t = (i >> 1) & 1;
          if (i & 1) dpacc[t] = mfma32(fa[i], dof[i >> 2], dpacc[t]);
          else sacc[t] = mfma32(fa[i], qf[i >> 2], sacc[t]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, RA, 0);
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i + RA < NM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
      } else
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          sacc[t] = mfma32(lds_row(kimg + 32 * t * D * 2, koff[kk]), qf[kk], sacc[t]);
          dpacc[t] = mfma32(lds_row(vimg + 32 * t * D * 2, koff[kk]), dof[kk], dpacc[t]);
        }
      }
      const bool need_mask = (CAUSAL && k0 + FK - 1 > qw) || k0 + FK > T;
      uint32_t sf[2][2][4];  // [t][s][pair]: dS^T as the B operand of K^T dS^T
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int e = 0; e < 16; e += 2) {
          float p0 = fast_exp2(fmaf(sacc[t][e], c, nlc)), p1 = fast_exp2(fmaf(sacc[t][e + 1], c, nlc));
          if (need_mask) {
            const int key = k0 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * hh;
            if ((CAUSAL && key > qrow) || key >= T) p0 = 0.f;
            if ((CAUSAL && key + 1 > qrow) || key + 1 >= T) p1 = 0.f;
          }
          sf[t][e >> 3][(e & 7) >> 1] = pack2(p0 * (dpacc[t][e] + nd_q), p1 * (dpacc[t][e + 1] + nd_q));
        }
      }
      if constexpr (KFATT_DQ_RA > 0 && D == 128) {
        constexpr int RA = KFATT_DQ_RA, NM = 4 * ND;  // MFMA i: n = i / 4, t = (i / 2) & 1, s2 = i & 1
        bf16x8 fk[NM];
        auto rd = [&](int i) __attribute__((always_inline)) {
          const char* base = kimg + (32 * ((i >> 1) & 1) + 16 * (i & 1)) * D * 2;
          fk[i] = join(tr_read(base, voff0[i >> 2]), tr_read(base, voff1[i >> 2]));
        };
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i == 0)
#pragma unroll
            for (int u = 0; u < RA; ++u) rd(u);
          if (i + RA < NM) rd(i + RA);
          const int t = (i >> 1) & 1, s2 = i & 1;
          const u32x4 sw = {sf[t][s2][0], sf[t][s2][1], sf[t][s2][2], sf[t][s2][3]};
          dqacc[i >> 2] = mfma32(fk[i], __builtin_bit_cast(bf16x8, sw), dqacc[i >> 2]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * RA, 0);
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i + RA < NM) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
      } else
#pragma unroll
      for (int n = 0; n < ND; ++n) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const bf16x8 kf = join(tr_read(kimg + (32 * t + 16 * s2) * D * 2, voff0[n]),
                                   tr_read(kimg + (32 * t + 16 * s2) * D * 2, voff1[n]));
            const u32x4 sw = {sf[t][s2][0], sf[t][s2][1], sf[t][s2][2], sf[t][s2][3]};
            dqacc[n] = mfma32(kf, __builtin_bit_cast(bf16x8, sw), dqacc[n]);
          }
        }
      }
    }
    // the next tile's pieces (the only vector-memory operations in the loop) have landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  for (int j = 0; j < ntiles; j += 2) {
    tile_body(j, std::integral_constant<int, 0>{});
    if (j + 1 < ntiles) tile_body(j + 1, std::integral_constant<int, 1>{});
  }

  // lane (r, hh) holds row qrow, d = 32 n + (e & 3) + 8 (e >> 2) + 4 hh
  __bf16* dqr = dq + base_off(a, TDQ, b, h) + qrow * a.s[TDQ][2];
  if constexpr (KFATT_BWD_WIDE) {
    store_rows16<ND>(dqr, dqacc, a.scale, qrow < T, hh);
  } else if (qrow < T) {
    const float sc = a.scale;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u32x2 v2 = {pack2(dqacc[n][4 * g] * sc, dqacc[n][4 * g + 1] * sc),
                          pack2(dqacc[n][4 * g + 2] * sc, dqacc[n][4 * g + 3] * sc)};
        *reinterpret_cast<u32x2*>(dqr + 32 * n + 8 * g + 4 * hh) = v2;
      }
    }
  }
  }  // pass
}

// dS^T image [128 keys][64 queries]: 128-B rows of sixteen 8-B slots (4 queries each), slot ^ f(row),
// f(row) = (row & 15) ^ (((row >> 1) & 1) << 3). The accumulator's stores (16 lanes = 16 consecutive
// keys, one slot each) cover all 32 write banks (unswizzled: one slot column, 16-way); the dQ
// product's transposed reads (4 consecutive keys x 32 queries per 32-lane half) put rows r and r+2,
// which share a 256-B bank window, on opposite 8-slot halves. (The round-5 first cut's 32-query image
// without a swizzle cost SQ_LDS_BANK_CONFLICT 4.7e7 cycles per 3 gpt-1b backward passes.)
__device__ __forceinline__ int dst_off(int row, int slot8) {
  return row * 128 + ((slot8 ^ ((row & 15) ^ (((row >> 1) & 1) << 3))) << 3);
}

// ------------------------------------------------------------------------------------------------
// backward: one workgroup = 4 waves = 128 keys of one (b, h); 64-row query tiles (Q, dO, lse,
// delta) double-buffered through LDS, two 32-row S / dP sub-tiles per wave; dK / dV in registers
// for the whole sweep
// ------------------------------------------------------------------------------------------------
constexpr int BK = 128, BQ = 64, QS = BQ / 32;

// ------------------------------------------------------------------------------------------------
// dK / dV with two waves per SIMD (KFATT_DKDV8, used with the split dQ kernel): 8 waves = 4 key
// groups of 32 keys x 2 query halves. Wave (w, jh) takes rows 32 jh .. 32 jh + 31 of every 64-row
// query tile for the keys of group w, so the two waves of a SIMD interleave their LDS waits and
// barriers with each other's MFMAs (the 4-wave kernel runs one wave per SIMD at D = 128 and waits
// half its cycles). K and V both sit in LDS (V rows are the dP product's B operand) to keep a wave
// within 256 registers; the two halves' partial dK^T / dV^T are summed through LDS at the end.
// ------------------------------------------------------------------------------------------------
template <int D, bool CAUSAL>
__global__ __launch_bounds__(512, D == 64 ? 2 : 1) void attn_bwd_dkdv8(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                         const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                         const float* __restrict__ nl, const float* __restrict__ nd,
                                                         __bf16* __restrict__ dk, __bf16* __restrict__ dv, AttnShape a) {
  constexpr int KS = D / 16;
  constexpr int ND = D / 32;
  constexpr int CH = D / 8;
  constexpr int KIMG = BK * D * 2;          // K (and V) image: [128 keys][D]
  constexpr int QT = BQ * D * 2;            // one Q (or dO) tile image: [64][D]
  constexpr int NPC = QT / 1024 / 8;        // LDS-DMA pieces per wave per tile image
  static_assert(NPC >= 1, "head dim");
  static_assert(4 * QT >= 4 * ND * 4 * 1024, "partial-sum staging fits the Q / dO region");
  __shared__ __attribute__((aligned(16))) char smem[2 * KIMG + 4 * QT + 4 * BQ * 4];
  char* const kimg = smem;
  char* const vimg = smem + KIMG;
  char* const qtiles = smem + 2 * KIMG;     // [buf][Q, dO]
  float* const rowc = reinterpret_cast<float*>(qtiles + 4 * QT);  // [buf][nl(64), nd(64)]

  const int T = a.T;
  const int nk = (T + BK - 1) / BK;
  const BlockId bo = block_order(blockIdx.x, nk, a.H * a.B, D == 64 ? 64 : 32);
  const int kblk = bo.rank;  // block 0 (all queries) first
  const int bh = bo.bh, h = bh % a.H, b = bh / a.H;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // 0..7, uniform
  const int w = wv & 3, jh = wv >> 2;                       // key group, query half
  const int k0 = kblk * BK, kw = k0 + 32 * w, key = kw + r;

  const __bf16* qb = q + base_off(a, TQ, b, h);
  const __bf16* kb = k + base_off(a, TK, b, h);
  const __bf16* vb = v + base_off(a, TV, b, h);
  const __bf16* dob = dout + base_off(a, TDO, b, h);
  const long long qt = a.s[TQ][2], kt = a.s[TK][2], vt = a.s[TV][2], dot = a.s[TDO][2];
  const float* nlb = nl + ((long long)b * a.H + h) * T;
  const float* ndb = nd + ((long long)b * a.H + h) * T;
  const auto rk = slice_rsrc(kb, 2LL * T * kt), rv = slice_rsrc(vb, 2LL * T * vt);

  // K and V images of the block's 128 keys (rows past T: zeros)
#pragma unroll
  for (int i = 0; i < BK * CH / 512; ++i) {
    const int c = tid + 512 * i, row = c / CH, ch = c % CH;
    *reinterpret_cast<u32x4*>(kimg + img_off<D>(row, ch)) = bload16(rk, 2 * (row * (int)kt + ch * 8), 2 * k0 * (int)kt);
    *reinterpret_cast<u32x4*>(vimg + img_off<D>(row, ch)) = bload16(rv, 2 * (row * (int)vt + ch * 8), 2 * k0 * (int)vt);
  }

  const int qstart = CAUSAL ? k0 : 0;
  const int ntiles = (T - qstart + BQ - 1) / BQ;

  const i32x4 dq_desc = slice_desc(qb, 2LL * T * qt), ddo_desc = slice_desc(dob, 2LL * T * dot);
  const i32x4 drow_desc = slice_desc(wv == 0 ? nlb : ndb, 4LL * T);
  int dvo_q[NPC], dvo_o[NPC];
#pragma unroll
  for (int i = 0; i < NPC; ++i) {
    const int byte = (wv * NPC + i) * 1024 + lane * 16;
    const int row = byte / (D * 2), ch = ((byte % (D * 2)) >> 4) ^ swz<D>(row, 0);
    dvo_q[i] = 2 * (row * (int)qt + ch * 8);
    dvo_o[i] = 2 * (row * (int)dot + ch * 8);
  }
  auto stage_dma = [&](int tile, int buf) {
    const int q0 = qstart + tile * BQ;
    char* qi = qtiles + buf * 2 * QT;
    char* oi = qi + QT;
#pragma unroll
    for (int i = 0; i < NPC; ++i) {
      dma16(dq_desc, lds_addr(qi + (wv * NPC + i) * 1024), dvo_q[i], 2 * q0 * (int)qt);
      dma16(ddo_desc, lds_addr(oi + (wv * NPC + i) * 1024), dvo_o[i], 2 * q0 * (int)dot);
    }
    if (wv < 2) dma4(drow_desc, lds_addr(reinterpret_cast<const char*>(rowc + buf * 2 * BQ + wv * BQ)), 4 * lane, 4 * q0);
  };

  int koff[KS], voff0[ND], voff1[ND];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) koff[kk] = img_off<D>(r, 2 * kk + hh);
  {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const int col = 32 * n + 16 * (g & 1) + 4 * pp;
      voff0[n] = img_off<D>(4 * hh + qq, col >> 3) + 8 * (pp & 1);
      voff1[n] = img_off<D>(4 * hh + qq + 8, col >> 3) + 8 * (pp & 1);
    }
  }
  const char* const kimg_w = kimg + 32 * w * D * 2;
  const char* const vimg_w = vimg + 32 * w * D * 2;

  const float c = a.scale * kLog2e;
  f32x16 dkacc[ND], dvacc[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) {
    dkacc[n] = (f32x16){};
    dvacc[n] = (f32x16){};
  }

  if (ntiles > 0) stage_dma(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto tile_body = [&](int it, auto BUFC) __attribute__((always_inline)) {
    constexpr int BUF = decltype(BUFC)::value;
    const int q0 = qstart + it * BQ;
    if ((KFATT_DKDV_ABL & 1) == 0 && it + 1 < ntiles) stage_dma(it + 1, 1 - BUF);  // ABL 1: no staging
    const char* qi = qtiles + BUF * 2 * QT + 32 * jh * D * 2;  // this wave's 32 query rows
    const char* oi = qi + QT;
    const float* nl_s = rowc + BUF * 2 * BQ + 32 * jh;
    const float* nd_s = nl_s + BQ;
    const int qw = q0 + 32 * jh;
    // causal: every query of the half precedes every key of the wave -> P = dS = 0
    if (!(CAUSAL && qw + 31 < kw)) {
      const bool need_mask = (CAUSAL && qw < kw + 31) || qw + 32 > T || key >= T;
      f32x16 sacc, dpacc;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(nl_s + 8 * g + 4 * hh);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(nd_s + 8 * g + 4 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sacc[4 * g + e] = l4[e];
          dpacc[4 * g + e] = d4[e];
        }
      }
      // S^T-free form as the 4-wave kernel: rows = this wave's queries, column = the lane's key
      if constexpr (KFATT_BWD_RA > 0 && D == 128) {
        // KFATT_BWD_RA: both operands of MFMA i + RA read before MFMA i issues, pinned by sched
        // groups (MFMA i: k-step i / 2, S for even i, dP for odd)
        constexpr int RA = KFATT_BWD_RA, NM = 2 * KS;
        bf16x8 fa[NM], fb[NM];
        auto rd = [&](int i) __attribute__((always_inline)) {
          fa[i] = lds_row((i & 1) ? oi : qi, koff[i >> 1]);
          fb[i] = lds_row((i & 1) ? vimg_w : kimg_w, koff[i >> 1]);
        };
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i == 0)
#pragma unroll
            for (int u = 0; u < RA; ++u) rd(u);
          if (i + RA < NM) rd(i + RA);
          if (i & 1) dpacc = mfma32(fa[i], fb[i], dpacc);
          else sacc = mfma32(fa[i], fb[i], sacc);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * RA, 0);
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i + RA < NM) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const int kr = (KFATT_DKDV_ABL & 4) ? 0 : kk;  // ABL 4: one K / V fragment read per tile (timing only)
          sacc = mfma32(lds_row(qi, koff[kk]), lds_row(kimg_w, koff[kr]), sacc);
          dpacc = mfma32(lds_row(oi, koff[kk]), lds_row(vimg_w, koff[kr]), dpacc);
        }
      }
      uint32_t pf[2][4], sf[2][4];
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        float p0 = fast_exp2(sacc[e] * c), p1 = fast_exp2(sacc[e + 1] * c);
        if (need_mask) {
          const int qa0 = qw + (e & 3) + 8 * (e >> 2) + 4 * hh;
          if ((CAUSAL && qa0 < key) || qa0 >= T || key >= T) p0 = 0.f;
          if ((CAUSAL && qa0 + 1 < key) || qa0 + 1 >= T || key >= T) p1 = 0.f;
        }
        pf[e >> 3][(e & 7) >> 1] = pack2(p0, p1);
        sf[e >> 3][(e & 7) >> 1] = pack2(p0 * dpacc[e], p1 * dpacc[e + 1]);
      }
      // dV^T += dO^T . P and dK^T += Q^T . dS over this half's rows (permuted k order)
      if constexpr (KFATT_BWD_RA > 0 && D == 128) {
        constexpr int RA = 2 * KFATT_BWD_RA, NM = 4 * ND;  // MFMA i: n = i / 4, sx = (i / 2) & 1, dV for even i
        bf16x8 fa[NM];
        auto rd = [&](int i) __attribute__((always_inline)) {
          const char* base = ((i & 1) ? qi : oi) + 16 * ((i >> 1) & 1) * D * 2;
          fa[i] = join(tr_read(base, voff0[i >> 2]), tr_read(base, voff1[i >> 2]));
        };
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i == 0)
#pragma unroll
            for (int u = 0; u < RA; ++u) rd(u);
          if (i + RA < NM) rd(i + RA);
          const int sx = (i >> 1) & 1, n = i >> 2;
          if (i & 1) {
            const u32x4 sw = {sf[sx][0], sf[sx][1], sf[sx][2], sf[sx][3]};
            dkacc[n] = mfma32(fa[i], __builtin_bit_cast(bf16x8, sw), dkacc[n]);
          } else {
            const u32x4 pw = {pf[sx][0], pf[sx][1], pf[sx][2], pf[sx][3]};
            dvacc[n] = mfma32(fa[i], __builtin_bit_cast(bf16x8, pw), dvacc[n]);
          }
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * RA, 0);
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i + RA < NM) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
      } else
#pragma unroll
      for (int n = 0; n < ND; ++n) {
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const u32x4 pw = {pf[sx][0], pf[sx][1], pf[sx][2], pf[sx][3]};
          const u32x4 sw = {sf[sx][0], sf[sx][1], sf[sx][2], sf[sx][3]};
          const bf16x8 doa = join(tr_read(oi + 16 * sx * D * 2, voff0[n]), tr_read(oi + 16 * sx * D * 2, voff1[n]));
          dvacc[n] = mfma32(doa, __builtin_bit_cast(bf16x8, pw), dvacc[n]);
          const bf16x8 qa = join(tr_read(qi + 16 * sx * D * 2, voff0[n]), tr_read(qi + 16 * sx * D * 2, voff1[n]));
          dkacc[n] = mfma32(qa, __builtin_bit_cast(bf16x8, sw), dkacc[n]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next tile's pieces (the loop's only VMEM)
    if ((KFATT_DKDV_ABL & 2) == 0) __syncthreads();       // ABL 2: no barrier (timing only)
  };
  for (int it = 0; it < ntiles; it += 2) {
    tile_body(it, std::integral_constant<int, 0>{});
    if (it + 1 < ntiles) tile_body(it + 1, std::integral_constant<int, 1>{});
  }

  // the two query halves' partial sums: half 1 stages its accumulators (f32, lane-major) in the
  // Q / dO region, half 0 adds them and stores; dK first, then dV
  float* const part = reinterpret_cast<float*>(qtiles);
  auto reduce = [&](f32x16 (&acc)[ND]) __attribute__((always_inline)) {
    if (jh == 1) {
#pragma unroll
      for (int n = 0; n < ND; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4*>(part + (((w * ND + n) * 4 + g) * 64 + lane) * 4) =
              (f32x4){acc[n][4 * g], acc[n][4 * g + 1], acc[n][4 * g + 2], acc[n][4 * g + 3]};
    }
    __syncthreads();
    if (jh == 0) {
#pragma unroll
      for (int n = 0; n < ND; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(part + (((w * ND + n) * 4 + g) * 64 + lane) * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[n][4 * g + e] += x[e];
        }
    }
    __syncthreads();
  };
  reduce(dkacc);
  reduce(dvacc);
  // lane = key, rows d = 32 n + (e & 3) + 8 (e >> 2) + 4 hh
  if (KFATT_BWD_WIDE && jh == 0) {  // (jh: wave-uniform, so whole waves run the swaps)
    store_rows16<ND>(dk + base_off(a, TDK, b, h) + key * a.s[TDK][2], dkacc, a.scale, key < T, hh);
    store_rows16<ND>(dv + base_off(a, TDV, b, h) + key * a.s[TDV][2], dvacc, 1.f, key < T, hh);
  } else if (jh == 0 && key < T) {
    __bf16* dkr = dk + base_off(a, TDK, b, h) + key * a.s[TDK][2];
    __bf16* dvr = dv + base_off(a, TDV, b, h) + key * a.s[TDV][2];
#pragma unroll
    for (int n = 0; n < ND; ++n) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * n + 8 * g + 4 * hh;
        const float sc = a.scale;
        *reinterpret_cast<u32x2*>(dkr + d) =
            (u32x2){pack2(dkacc[n][4 * g] * sc, dkacc[n][4 * g + 1] * sc), pack2(dkacc[n][4 * g + 2] * sc, dkacc[n][4 * g + 3] * sc)};
        *reinterpret_cast<u32x2*>(dvr + d) =
            (u32x2){pack2(dvacc[n][4 * g], dvacc[n][4 * g + 1]), pack2(dvacc[n][4 * g + 2], dvacc[n][4 * g + 3])};
      }
    }
  }
}

// D = 128 holds dK^T, dV^T (128 registers) and V (32) for the whole sweep: one wave per SIMD
// (512-register budget, no spills); D = 64 fits two
template <int D, bool CAUSAL, bool DQS = false>
__global__ __launch_bounds__(256, D == 128 ? 1 : 2) void attn_bwd(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                   const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                   const float* __restrict__ lse, const float* __restrict__ delta,
                                                   float* __restrict__ dq_acc, __bf16* __restrict__ dk,
                                                   __bf16* __restrict__ dv, AttnShape a, long long dq_st,
                                                   long long dq_sh, long long dq_sb) {
  constexpr int KS = D / 16;
  constexpr int ND = D / 32;
  constexpr int CH = D / 8;
  constexpr int KIMG = BK * D * 2;          // K image: [128 keys][D]
  constexpr int QT = BQ * D * 2;            // one Q (or dO) tile image: [64][D]
  constexpr int DST = BK * BQ * 2;          // dS^T image: [128 keys][64 q]
  constexpr int NQC = BQ * CH / 256;        // chunks per thread per Q (and per dO) tile
  constexpr int DQT = QS * ND / 4;          // 32x32 dQ tiles per wave per query tile
  static_assert(NQC >= 1 && DQT >= 1, "head dim");
  __shared__ __attribute__((aligned(16))) char smem[KIMG + 4 * QT + DST + 4 * BQ * 4];
  char* const kimg = smem;
  char* const qtiles = smem + KIMG;         // [buf][Q, dO]
  char* const dst = qtiles + 4 * QT;
  float* const rowc = reinterpret_cast<float*>(dst + DST);  // [buf][lse(64), delta(64)]

  const int T = a.T;
  const int nk = (T + BK - 1) / BK;
  const BlockId bo = block_order(blockIdx.x, nk, a.H * a.B, D == 128 ? 32 : 64);
  const int kblk = bo.rank;  // block 0 (all queries) first
  const int bh = bo.bh, h = bh % a.H, b = bh / a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int k0 = kblk * BK, kw = k0 + 32 * w, key = kw + r;

  const __bf16* qb = q + base_off(a, TQ, b, h);
  const __bf16* kb = k + base_off(a, TK, b, h);
  const __bf16* vb = v + base_off(a, TV, b, h);
  const __bf16* dob = dout + base_off(a, TDO, b, h);
  const long long qt = a.s[TQ][2], kt = a.s[TK][2], vt = a.s[TV][2], dot = a.s[TDO][2];
  const float* lseb = lse + ((long long)b * a.H + h) * T;
  const float* deltab = delta + ((long long)b * a.H + h) * T;
  const auto rdq = slice_rsrc(dq_acc + b * dq_sb + h * dq_sh, 4LL * T * dq_st);

  // K image for the dQ product (tr reads) and the S product (row reads); V rows in registers
#pragma unroll
  for (int i = 0; i < BK * CH / 256; ++i) {
    const int c = tid + 256 * i, row = c / CH, ch = c % CH;
    u32x4 x = {0u, 0u, 0u, 0u};
    if (k0 + row < T) x = gload16(kb + (k0 + row) * kt + ch * 8);
    *reinterpret_cast<u32x4*>(kimg + img_off<D>(row, ch)) = x;
  }
  bf16x8 vf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    u32x4 x = {0u, 0u, 0u, 0u};
    if (key < T) x = gload16(vb + key * vt + kk * 16 + 8 * hh);
    vf[kk] = __builtin_bit_cast(bf16x8, x);
  }

  const int qstart = CAUSAL ? k0 : 0;
  const int ntiles = (T - qstart + BQ - 1) / BQ;

  constexpr bool kDma = KFATT_DMA && KFATT_BUF;
  u32x4 qreg[kDma ? 1 : NQC], oreg[kDma ? 1 : NQC];
  float rreg = 0.f;
  const auto rq = slice_rsrc(qb, 2LL * T * qt), rdo = slice_rsrc(dob, 2LL * T * dot);
  // (the selector through readfirstlane: a per-lane select of the base would make the compiler wrap
  // the load in a waterfall loop over descriptor values)
  const auto rrow = slice_rsrc(__builtin_amdgcn_readfirstlane(w) == 0 ? lseb : deltab, 4LL * T);
  const i32x4 dq_desc = slice_desc(qb, 2LL * T * qt), ddo_desc = slice_desc(dob, 2LL * T * dot);
  const i32x4 drow_desc = slice_desc(__builtin_amdgcn_readfirstlane(w) == 0 ? lseb : deltab, 4LL * T);
  auto stage_load = [&](int tile) {
    const int q0 = qstart + tile * BQ;
#pragma unroll
    for (int i = 0; i < (kDma ? 0 : NQC); ++i) {
      const int c = tid + 256 * i, row = c / CH, ch = c % CH;
      if constexpr (KFATT_BUF) {
        qreg[i] = bload16(rq, 2 * ((q0 + row) * (int)qt + ch * 8));
        oreg[i] = bload16(rdo, 2 * ((q0 + row) * (int)dot + ch * 8));
      } else {
        u32x4 xq = {0u, 0u, 0u, 0u}, xo = {0u, 0u, 0u, 0u};
        if (q0 + row < T) {
          xq = gload16(qb + (q0 + row) * qt + ch * 8);
          xo = gload16(dob + (q0 + row) * dot + ch * 8);
        }
        qreg[i] = xq;
        oreg[i] = xo;
      }
    }
    if (!kDma && tid < 2 * BQ) {  // waves 0 / 1: the tile's lse / delta (rows past T read 0)
      const int row = tid & (BQ - 1);
      if constexpr (KFATT_BUF) {
        rreg = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rrow, 4 * (q0 + row), 0, 0));
      } else {
        rreg = 0.f;
        if (q0 + row < T) rreg = tid < BQ ? lseb[q0 + row] : deltab[q0 + row];
      }
    }
  };
  auto stage_write = [&](int buf) {
    char* qi = qtiles + buf * 2 * QT;
    char* oi = qi + QT;
    if constexpr (!kDma) {
#pragma unroll
      for (int i = 0; i < NQC; ++i) {
        const int c = tid + 256 * i, row = c / CH, ch = c % CH;
        const int off = img_off<D>(row, ch);
        *reinterpret_cast<u32x4*>(qi + off) = qreg[i];
        *reinterpret_cast<u32x4*>(oi + off) = oreg[i];
      }
    }
    if (!kDma && tid < 2 * BQ) rowc[buf * 2 * BQ + tid] = rreg;
  };
  // KFATT_DMA: the Q / dO tiles go global -> LDS by LDS-DMA (buffer_load ... lds), no staging
  // registers. A wave instruction fills 1 KiB of the image linearly (lane L at +16 L), so each lane
  // fetches the chunk that the swizzle puts there: image chunk sc of row `row` holds source chunk
  // sc ^ swz(row, 0) (the swizzle is an XOR per row). Rows past T land as zeros (buffer range).
  // LDS-DMA pieces: uniform wave index, per-lane source offsets computed once (as the forward's)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int dvo_q[kDma ? NQC : 1], dvo_o[kDma ? NQC : 1];
#pragma unroll
  for (int i = 0; i < (kDma ? NQC : 0); ++i) {
    const int byte = (wu * NQC + i) * 1024 + lane * 16;
    const int row = byte / (D * 2), ch = ((byte % (D * 2)) >> 4) ^ swz<D>(row, 0);
    dvo_q[i] = 2 * (row * (int)qt + ch * 8);
    dvo_o[i] = 2 * (row * (int)dot + ch * 8);
  }
  auto stage_dma = [&](int tile, int buf) {
    const int q0 = qstart + tile * BQ;
    char* qi = qtiles + buf * 2 * QT;
    char* oi = qi + QT;
#pragma unroll
    for (int i = 0; i < NQC; ++i) {
      dma16(dq_desc, lds_addr(qi + (wu * NQC + i) * 1024), dvo_q[i], 2 * q0 * (int)qt);
      dma16(ddo_desc, lds_addr(oi + (wu * NQC + i) * 1024), dvo_o[i], 2 * q0 * (int)dot);
    }
    // waves 0 / 1: the tile's 64 lse / delta values (no register staging: a pending load into a
    // register made the compiler wait vmcnt(0) before the tile's first MFMA)
    if (wu < 2) dma4(drow_desc, lds_addr(reinterpret_cast<const char*>(rowc + buf * 2 * BQ + wu * BQ)), 4 * lane, 4 * q0);
  };

  const float c = a.scale * kLog2e;
  f32x16 dkacc[ND], dvacc[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) {
    dkacc[n] = (f32x16){};
    dvacc[n] = (f32x16){};
  }

  if (ntiles > 0) {
    if constexpr (kDma) stage_dma(0, 0);
    stage_load(0);
    if constexpr (kDma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stage_write(0);
  }
  __syncthreads();

  // per-lane LDS read offsets computed once; the q-tile loop unrolled over the two buffers so the
  // buffer / sub-tile / k-step parts of every read ride in the ds_read immediate (as the forward)
  int koff[KS], voff0[ND], voff1[ND];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) koff[kk] = img_off<D>(r, 2 * kk + hh);  // + 32 j / 32 w rows
  {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const int col = 32 * n + 16 * (g & 1) + 4 * pp;
      voff0[n] = img_off<D>(4 * hh + qq, col >> 3) + 8 * (pp & 1);
      voff1[n] = img_off<D>(4 * hh + qq + 8, col >> 3) + 8 * (pp & 1);
    }
  }
  const char* const kimg_w = kimg + 32 * w * D * 2;  // this wave's 32 key rows
  auto tile_body = [&](int it, auto BUFC) __attribute__((always_inline)) {
    constexpr int BUF = decltype(BUFC)::value;
    const int q0 = qstart + it * BQ;
    const bool more = it + 1 < ntiles;
    if (more) {
      if constexpr (kDma) stage_dma(it + 1, 1 - BUF);
      stage_load(it + 1);
    }
    const char* qi = qtiles + BUF * 2 * QT;
    const char* oi = qi + QT;
    const float* lse_s = rowc + BUF * 2 * BQ;
    const float* del_s = lse_s + BQ;

    // causal: every query of the tile precedes every key of the wave -> P = dS = 0
    const bool idle = CAUSAL && q0 + BQ - 1 < kw;
    if (!idle) {
      const bool need_mask = (CAUSAL && q0 < kw + 31) || q0 + BQ > T || key >= T;
#pragma unroll
      for (int j = 0; j < QS; ++j) {
        // one 32-row sub-tile at a time: its P / dS fragments are consumed before the next one's exist
        uint32_t pf[2][4], sf[2][4];
        f32x16 sacc, dpacc;
        // row constants nl = -lse / scale and nd = -delta (the prologue's) for this lane's query rows
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(lse_s + 32 * j + 8 * g + 4 * hh);
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(del_s + 32 * j + 8 * g + 4 * hh);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sacc[4 * g + e] = l4[e];   // nl = -lse / scale
            dpacc[4 * g + e] = d4[e];  // nd = -delta
          }
        }
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const bf16x8 qa = lds_row(qi + 32 * j * D * 2, koff[kk]);
          const bf16x8 kbf = lds_row(kimg_w, koff[kk]);
          sacc = mfma32(qa, kbf, sacc);
          const bf16x8 oa = lds_row(oi + 32 * j * D * 2, koff[kk]);
          dpacc = mfma32(oa, vf[kk], dpacc);
        }
        // P and dS; rows q = q0 + 32 j + (e & 3) + 8 (e >> 2) + 4 hh, column = this lane's key
#pragma unroll
        for (int e = 0; e < 16; e += 2) {
          float p0 = fast_exp2(sacc[e] * c), p1 = fast_exp2(sacc[e + 1] * c);
          if (need_mask) {
            const int qa0 = q0 + 32 * j + (e & 3) + 8 * (e >> 2) + 4 * hh;
            if ((CAUSAL && qa0 < key) || qa0 >= T || key >= T) p0 = 0.f;
            if ((CAUSAL && qa0 + 1 < key) || qa0 + 1 >= T || key >= T) p1 = 0.f;
          }
          pf[e >> 3][(e & 7) >> 1] = pack2(p0, p1);
          sf[e >> 3][(e & 7) >> 1] = pack2(p0 * dpacc[e], p1 * dpacc[e + 1]);
        }
        // dS^T image [key][q]: registers 4g..4g+3 are queries 32 j + 8 g + 4 hh .. +3 of this lane's key
        if constexpr (!DQS) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const u32x2 v2 = {sf[g >> 1][2 * (g & 1)], sf[g >> 1][2 * (g & 1) + 1]};
            *reinterpret_cast<u32x2*>(dst + dst_off(32 * w + r, 8 * j + 2 * g + hh)) = v2;
          }
        }
        // dV^T += dO^T . P and dK^T += Q^T . dS over this sub-tile's rows (permuted k order)
#pragma unroll
        for (int n = 0; n < ND; ++n) {
#pragma unroll
          for (int sx = 0; sx < 2; ++sx) {
            const u32x4 pw = {pf[sx][0], pf[sx][1], pf[sx][2], pf[sx][3]};
            const u32x4 sw = {sf[sx][0], sf[sx][1], sf[sx][2], sf[sx][3]};
            const bf16x8 doa = join(tr_read(oi + (32 * j + 16 * sx) * D * 2, voff0[n]),
                                    tr_read(oi + (32 * j + 16 * sx) * D * 2, voff1[n]));
            dvacc[n] = mfma32(doa, __builtin_bit_cast(bf16x8, pw), dvacc[n]);
            const bf16x8 qa = join(tr_read(qi + (32 * j + 16 * sx) * D * 2, voff0[n]),
                                   tr_read(qi + (32 * j + 16 * sx) * D * 2, voff1[n]));
            dkacc[n] = mfma32(qa, __builtin_bit_cast(bf16x8, sw), dkacc[n]);
          }
        }
      }
    } else if constexpr (!DQS) {
      // this wave's 32 rows of the dS^T image are zero (lane half hh clears slots 8 hh .. 8 hh + 7)
#pragma unroll
      for (int sl = 0; sl < 8; ++sl)
        *reinterpret_cast<u32x2*>(dst + dst_off(32 * w + r, 8 * hh + sl)) = (u32x2){0u, 0u};
    }
    if constexpr (!DQS) __syncthreads();

    // dQ[q][d]: this wave's 32x32 output tiles (query sub-tile j, d tile n), all 128 keys: A = dS rows
    // from the [key][q] image by tr reads, B = K columns from the K image by tr reads
    // (DQS: dQ is the atomic-free attn_bwd_dq_split kernel's)
    if constexpr (!DQS) {
      const int g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
#pragma unroll
      for (int tt = 0; tt < DQT; ++tt) {
        const int t = w + 4 * tt, j = t / ND, dqn = t % ND;
        f32x16 dqacc = (f32x16){};
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
          const int kr = 16 * kk + 8 * hh + qq;          // key row of this lane's tr-read address
          const int qs = 8 * j + 4 * (g & 1) + p;        // 8-B slot of queries 32 j + 16 (g & 1) + 4 p .. +3
          const bf16x8 da = join(tr_read(dst, dst_off(kr, qs)), tr_read(dst, dst_off(kr + 4, qs)));
          const int dc = 32 * dqn + 16 * (g & 1) + 4 * p;
          const bf16x8 kbf = join(tr_read(kimg, img_off<D>(kr, dc >> 3) + 8 * (p & 1)),
                                  tr_read(kimg, img_off<D>(kr + 4, dc >> 3) + 8 * (p & 1)));
          dqacc = mfma32(da, kbf, dqacc);
        }
        // rows q0 + 32 j + (e & 3) + 8 (e >> 2) + 4 hh, column d = 32 dqn + r: f32 atomics, each wave
        // instruction two 128-B row segments
        if constexpr (KFATT_BUF) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int qr = q0 + 32 * j + (e & 3) + 8 * (e >> 2) + 4 * hh;
            // (KFATT_ABL == 1, timing ablation only: every atomic out of range, dropped by the address unit)
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(dqacc[e], rdq,
                                                            4 * (qr * (int)dq_st + 32 * dqn + r) | (KFATT_ABL == 1 ? 0x70000000 : 0), 0, 0);
          }
        } else {
          float* dqb = dq_acc + b * dq_sb + h * dq_sh + 32 * dqn + r;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int qr = q0 + 32 * j + (e & 3) + 8 * (e >> 2) + 4 * hh;
            if (qr < T) __hip_atomic_fetch_add(dqb + qr * dq_st, dqacc[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
    }
    if (more) {
      // the next tile's LDS-DMA pieces (and the lse / delta load) were issued before this tile's
      // DQT x 16 dQ atomics: waiting down to that many outstanding lands exactly them
      if constexpr (kDma) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DQS ? 0 : DQT * 16) : "memory");
      stage_write(1 - BUF);
    }
    __syncthreads();
  };
  for (int it = 0; it < ntiles; it += 2) {
    tile_body(it, std::integral_constant<int, 0>{});
    if (it + 1 < ntiles) tile_body(it + 1, std::integral_constant<int, 1>{});
  }

  // epilogue: dK = scale * (dK^T)^T, dV; lane = key, rows d = 32 n + (e & 3) + 8 (e >> 2) + 4 hh
  if (key < T) {
    __bf16* dkr = dk + base_off(a, TDK, b, h) + key * a.s[TDK][2];
    __bf16* dvr = dv + base_off(a, TDV, b, h) + key * a.s[TDV][2];
#pragma unroll
    for (int n = 0; n < ND; ++n) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * n + 8 * g + 4 * hh;
        const float s = a.scale;
        *reinterpret_cast<u32x2*>(dkr + d) =
            (u32x2){pack2(dkacc[n][4 * g] * s, dkacc[n][4 * g + 1] * s), pack2(dkacc[n][4 * g + 2] * s, dkacc[n][4 * g + 3] * s)};
        *reinterpret_cast<u32x2*>(dvr + d) =
            (u32x2){pack2(dvacc[n][4 * g], dvacc[n][4 * g + 1]), pack2(dvacc[n][4 * g + 2], dvacc[n][4 * g + 3])};
      }
    }
  }
}

// dq (bf16, strided) = scale * dq_acc (f32 [B][T][H][D] with strides st / sh / sb)
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_dq(const float* __restrict__ dq_acc, __bf16* __restrict__ dq,
                                                   AttnShape a, long long st, long long sh, long long sb) {
  constexpr int LPR = D / 8;
  constexpr int RPB = 256 / LPR;
  const long long nrows = (long long)a.B * a.H * a.T;
  const long long row = (long long)blockIdx.x * RPB + threadIdx.x / LPR;
  const int part = threadIdx.x % LPR;
  if (row >= nrows) return;
  const int t = (int)(row % a.T);
  const int h = (int)((row / a.T) % a.H);
  const int b = (int)(row / ((long long)a.T * a.H));
  const float* src = dq_acc + b * sb + h * sh + t * st + part * 8;
  const f32x4 x0 = *reinterpret_cast<const f32x4*>(src), x1 = *reinterpret_cast<const f32x4*>(src + 4);
  const float s = a.scale;
  const u32x4 y = {pack2(x0[0] * s, x0[1] * s), pack2(x0[2] * s, x0[3] * s), pack2(x1[0] * s, x1[1] * s),
                   pack2(x1[2] * s, x1[3] * s)};
  *reinterpret_cast<u32x4*>(dq + base_off(a, TDQ, b, h) + t * a.s[TDQ][2] + part * 8) = y;
}

bool fill_shape(AttnShape& s, int B, int H, int T, int D, float scale, const long long* strides, int ntensors) {
  if (B <= 0 || H <= 0 || T <= 0 || (D != 64 && D != 128) || !strides) return false;
  s.B = B;
  s.H = H;
  s.T = T;
  s.scale = scale;
  for (int t = 0; t < 8; ++t)
    for (int j = 0; j < 3; ++j) s.s[t][j] = t < ntensors ? strides[3 * t + j] : 0;
  for (int t = 0; t < ntensors; ++t)
    for (int j = 0; j < 3; ++j)
      if (strides[3 * t + j] & 7) return false;  // 16-B aligned rows
  return true;
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// compute units of the current device, queried once (256 on MI355X)
int device_cus() {
  static const int n = [] {
    int cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return cus > 0 ? cus : 256;
  }();
  return n;
}

// a (b, h) slice of T rows read through a buffer descriptor (KFATT_BUF): 32-bit byte offsets
bool slice_ok(int T, long long row_stride, int elem_bytes) {
  return row_stride > 0 && (long long)T * row_stride * elem_bytes < (1ll << 31);
}

}  // namespace

extern "C" int kfamd_attn_fwd_bf16(const void* q, const void* k, const void* v, void* o, void* lse, int B, int H, int T,
                                   int D, float scale, int causal, const long long* strides, void* stream) {
  AttnShape s;
  if (!q || !k || !v || !o || !lse) return KFAMD_EINVAL;
  if (!fill_shape(s, B, H, T, D, scale, strides, 4)) return KFAMD_EINVAL;
  if (!al16(q) || !al16(k) || !al16(v) || !al16(o)) return KFAMD_EALIGN;
  const long long nwg = (long long)((T + FQ - 1) / FQ) * H * B;
  if (nwg >= (1ll << 31)) return KFAMD_EINVAL;
  if (!slice_ok(T, s.s[TK][2], 2) || !slice_ok(T, s.s[TV][2], 2)) return KFAMD_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(256), 0, st, static_cast<const __bf16*>(q),
                       static_cast<const __bf16*>(k), static_cast<const __bf16*>(v), static_cast<__bf16*>(o),
                       static_cast<float*>(lse), s);
  };
  const int nq = (T + FQ - 1) / FQ;
  const int nq4 = (T + 255) / 256;
  const bool pair4 = causal && nq4 % 2 == 0;
  const long long g4 = (long long)(pair4 ? nq4 / 2 : nq4) * H * B;
  // attn_fwd_pp where its grid fills the chip (one workgroup per CU); attn_fwd otherwise and at
  // D = 64, where the two-workgroups-per-CU kernel measured faster (profiles/r6d_attn_pp)
  if (KFATT_FWD_PP && D == 128 && g4 >= device_cus()) {
    const bool pair = pair4;
    auto go4 = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((unsigned)g4), dim3(512), 0, st, static_cast<const __bf16*>(q),
                         static_cast<const __bf16*>(k), static_cast<const __bf16*>(v), static_cast<__bf16*>(o),
                         static_cast<float*>(lse), s);
    };
    pair ? go4(attn_fwd_pp<128, true, true>) : causal ? go4(attn_fwd_pp<128, true, false>)
                                                   : go4(attn_fwd_pp<128, false, false>);
  } else if constexpr (KFATT_FWD_NW == 8) {  // 8 waves x 32 rows per workgroup (A/B knob)
    const int nq8 = (T + 255) / 256;
    const bool pair = KFATT_FWD_PAIR && causal && nq8 % 2 == 0;
    const long long g8 = (long long)(pair ? nq8 / 2 : nq8) * H * B;
    auto go8 = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((unsigned)g8), dim3(512), 0, st, static_cast<const __bf16*>(q),
                         static_cast<const __bf16*>(k), static_cast<const __bf16*>(v), static_cast<__bf16*>(o),
                         static_cast<float*>(lse), s);
    };
    if (D == 128) pair ? go8(attn_fwd<128, true, true, 8>) : causal ? go8(attn_fwd<128, true, false, 8>)
                                                                    : go8(attn_fwd<128, false, false, 8>);
    else pair ? go8(attn_fwd<64, true, true, 8>) : causal ? go8(attn_fwd<64, true, false, 8>)
                                                          : go8(attn_fwd<64, false, false, 8>);
  } else if (KFATT_FWD_PAIR && causal && nq % 2 == 0) {
    auto go2 = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((unsigned)(nwg / 2)), dim3(256), 0, st, static_cast<const __bf16*>(q),
                         static_cast<const __bf16*>(k), static_cast<const __bf16*>(v), static_cast<__bf16*>(o),
                         static_cast<float*>(lse), s);
    };
    if (D == 128) go2(attn_fwd<128, true, true>);
    else go2(attn_fwd<64, true, true>);
  } else if (D == 128) {
    causal ? go(attn_fwd<128, true>) : go(attn_fwd<128, false>);
  } else {
    causal ? go(attn_fwd<64, true>) : go(attn_fwd<64, false>);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

extern "C" long long kfamd_attn_bwd_workspace(int B, int H, int T, int D) {
  // nl, nd f32 [B][H][T] (+ dq_acc f32 [B][T][H][D] in front of them when dQ goes through atomics)
  return (KFATT_DQ_SPLIT ? 0LL : (long long)B * T * H * D * 4) + 2LL * B * H * T * 4;
}

// strides: 8 tensors x (b, h, t): q, k, v, o, do, dq, dk, dv. workspace: kfamd_attn_bwd_workspace bytes
// (16-B aligned); it is zeroed here on the stream (memset node) before the dQ atomics.
extern "C" int kfamd_attn_bwd_bf16(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                   const void* lse, void* dq, void* dk, void* dv, void* workspace, int B, int H, int T,
                                   int D, float scale, int causal, const long long* strides, void* stream) {
  AttnShape s;
  if (!q || !k || !v || !o || !dout || !lse || !dq || !dk || !dv || !workspace) return KFAMD_EINVAL;
  if (!fill_shape(s, B, H, T, D, scale, strides, 8)) return KFAMD_EINVAL;
  if (!al16(q) || !al16(k) || !al16(v) || !al16(o) || !al16(dout) || !al16(dq) || !al16(dk) || !al16(dv) ||
      !al16(workspace))
    return KFAMD_EALIGN;
  const long long nk = (long long)((T + BK - 1) / BK) * H * B;
  if (nk >= (1ll << 31)) return KFAMD_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* dq_acc = static_cast<float*>(workspace);  // (unused with KFATT_DQ_SPLIT)
  // the prologue's row constants: nl = -lse / scale and nd = -delta, [B][H][T] each
  float* nl = dq_acc + (KFATT_DQ_SPLIT ? 0LL : (long long)B * T * H * D);
  float* nd = nl + (long long)B * H * T;
  const long long dq_st = (long long)H * D, dq_sh = D, dq_sb = (long long)T * H * D;
  if (!slice_ok(T, s.s[TQ][2], 2) || !slice_ok(T, s.s[TDO][2], 2) || !slice_ok(T, dq_st, 4)) return KFAMD_EINVAL;
  const long long rows = (long long)B * H * T;
  const unsigned rblocks = (unsigned)((rows + 256 / (D / 8) - 1) / (256 / (D / 8)));
  hipError_t e = hipSuccess;
  if constexpr (KFATT_DQ_SPLIT) {
    // dK / dV kernel without the dQ phase, then the atomic-free dQ kernel (no fp32 workspace)
    const long long nq = (long long)((T + FQ - 1) / FQ) * H * B;
    if (!slice_ok(T, s.s[TK][2], 2) || !slice_ok(T, s.s[TV][2], 2)) return KFAMD_EINVAL;
    auto run = [&](auto delta_k, auto main_k, auto dq_k) {
      hipLaunchKernelGGL(delta_k, dim3(rblocks), dim3(256), 0, st, static_cast<const __bf16*>(o),
                         static_cast<const __bf16*>(dout), static_cast<const float*>(lse), nl, nd, s);
      hipLaunchKernelGGL(main_k, dim3((unsigned)nk), dim3(256), 0, st, static_cast<const __bf16*>(q),
                         static_cast<const __bf16*>(k), static_cast<const __bf16*>(v), static_cast<const __bf16*>(dout),
                         static_cast<const float*>(nl), static_cast<const float*>(nd), dq_acc,
                         static_cast<__bf16*>(dk), static_cast<__bf16*>(dv), s, dq_st, dq_sh, dq_sb);
      hipLaunchKernelGGL(dq_k, dim3((unsigned)nq), dim3(256), 0, st, static_cast<const __bf16*>(q),
                         static_cast<const __bf16*>(k), static_cast<const __bf16*>(v), static_cast<const __bf16*>(dout),
                         static_cast<const float*>(nl), static_cast<const float*>(nd), static_cast<__bf16*>(dq), s,
                         static_cast<const __bf16*>(nullptr), static_cast<float*>(nullptr), static_cast<float*>(nullptr));
    };
    if (KFATT_DQ_DELTA && (D == 128 ? KFATT_DKDV8 : KFATT_DKDV8_64)) {
      // the dQ kernel first, as the prologue too (nl / nd), then the 8-wave dK / dV kernel
      const bool pair = KFATT_DQ_PAIR && causal && ((T + FQ - 1) / FQ) % 2 == 0;
      auto runq = [&](auto dq_k, auto main_k) {
        hipLaunchKernelGGL(dq_k, dim3((unsigned)(pair ? nq / 2 : nq)), dim3(256), 0, st, static_cast<const __bf16*>(q),
                           static_cast<const __bf16*>(k), static_cast<const __bf16*>(v),
                           static_cast<const __bf16*>(dout), static_cast<const float*>(lse),
                           static_cast<const float*>(nullptr), static_cast<__bf16*>(dq), s,
                           static_cast<const __bf16*>(o), nl, nd);
        hipLaunchKernelGGL(main_k, dim3((unsigned)nk), dim3(512), 0, st, static_cast<const __bf16*>(q),
                           static_cast<const __bf16*>(k), static_cast<const __bf16*>(v),
                           static_cast<const __bf16*>(dout), static_cast<const float*>(nl),
                           static_cast<const float*>(nd), static_cast<__bf16*>(dk), static_cast<__bf16*>(dv), s);
      };
      if (pair) D == 128 ? runq(attn_bwd_dq_split<128, true, true, true>, attn_bwd_dkdv8<128, true>)
                         : runq(attn_bwd_dq_split<64, true, true, true>, attn_bwd_dkdv8<64, true>);
      else if (D == 128) causal ? runq(attn_bwd_dq_split<128, true, true>, attn_bwd_dkdv8<128, true>)
                                : runq(attn_bwd_dq_split<128, false, true>, attn_bwd_dkdv8<128, false>);
      else causal ? runq(attn_bwd_dq_split<64, true, true>, attn_bwd_dkdv8<64, true>)
                  : runq(attn_bwd_dq_split<64, false, true>, attn_bwd_dkdv8<64, false>);
    } else if (KFATT_DKDV8 && D == 128) {
      auto run8 = [&](auto delta_k, auto main_k, auto dq_k) {
        hipLaunchKernelGGL(delta_k, dim3(rblocks), dim3(256), 0, st, static_cast<const __bf16*>(o),
                           static_cast<const __bf16*>(dout), static_cast<const float*>(lse), nl, nd, s);
        hipLaunchKernelGGL(main_k, dim3((unsigned)nk), dim3(512), 0, st, static_cast<const __bf16*>(q),
                           static_cast<const __bf16*>(k), static_cast<const __bf16*>(v),
                           static_cast<const __bf16*>(dout), static_cast<const float*>(nl),
                           static_cast<const float*>(nd), static_cast<__bf16*>(dk), static_cast<__bf16*>(dv), s);
        hipLaunchKernelGGL(dq_k, dim3((unsigned)nq), dim3(256), 0, st, static_cast<const __bf16*>(q),
                           static_cast<const __bf16*>(k), static_cast<const __bf16*>(v),
                           static_cast<const __bf16*>(dout), static_cast<const float*>(nl),
                           static_cast<const float*>(nd), static_cast<__bf16*>(dq), s,
                           static_cast<const __bf16*>(nullptr), static_cast<float*>(nullptr), static_cast<float*>(nullptr));
      };
      causal ? run8(attn_bwd_delta<128>, attn_bwd_dkdv8<128, true>, attn_bwd_dq_split<128, true>)
             : run8(attn_bwd_delta<128>, attn_bwd_dkdv8<128, false>, attn_bwd_dq_split<128, false>);
    } else if (D == 128) causal ? run(attn_bwd_delta<128>, attn_bwd<128, true, true>, attn_bwd_dq_split<128, true>)
                         : run(attn_bwd_delta<128>, attn_bwd<128, false, true>, attn_bwd_dq_split<128, false>);
    else if (KFATT_DKDV8_64) {
      auto run8 = [&](auto delta_k, auto main_k, auto dq_k) {
        hipLaunchKernelGGL(delta_k, dim3(rblocks), dim3(256), 0, st, static_cast<const __bf16*>(o),
                           static_cast<const __bf16*>(dout), static_cast<const float*>(lse), nl, nd, s);
        hipLaunchKernelGGL(main_k, dim3((unsigned)nk), dim3(512), 0, st, static_cast<const __bf16*>(q),
                           static_cast<const __bf16*>(k), static_cast<const __bf16*>(v),
                           static_cast<const __bf16*>(dout), static_cast<const float*>(nl),
                           static_cast<const float*>(nd), static_cast<__bf16*>(dk), static_cast<__bf16*>(dv), s);
        hipLaunchKernelGGL(dq_k, dim3((unsigned)nq), dim3(256), 0, st, static_cast<const __bf16*>(q),
                           static_cast<const __bf16*>(k), static_cast<const __bf16*>(v),
                           static_cast<const __bf16*>(dout), static_cast<const float*>(nl),
                           static_cast<const float*>(nd), static_cast<__bf16*>(dq), s,
                           static_cast<const __bf16*>(nullptr), static_cast<float*>(nullptr), static_cast<float*>(nullptr));
      };
      causal ? run8(attn_bwd_delta<64>, attn_bwd_dkdv8<64, true>, attn_bwd_dq_split<64, true>)
             : run8(attn_bwd_delta<64>, attn_bwd_dkdv8<64, false>, attn_bwd_dq_split<64, false>);
    } else causal ? run(attn_bwd_delta<64>, attn_bwd<64, true, true>, attn_bwd_dq_split<64, true>)
                : run(attn_bwd_delta<64>, attn_bwd<64, false, true>, attn_bwd_dq_split<64, false>);
    e = hipGetLastError();
    return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
  }
  e = hipMemsetAsync(dq_acc, 0, (size_t)B * T * H * D * 4, st);
  if (e != hipSuccess) return static_cast<int>(e);
  auto run = [&](auto delta_k, auto main_k, auto dq_k) {
    hipLaunchKernelGGL(delta_k, dim3(rblocks), dim3(256), 0, st, static_cast<const __bf16*>(o),
                       static_cast<const __bf16*>(dout), static_cast<const float*>(lse), nl, nd, s);
    hipLaunchKernelGGL(main_k, dim3((unsigned)nk), dim3(256), 0, st, static_cast<const __bf16*>(q),
                       static_cast<const __bf16*>(k), static_cast<const __bf16*>(v), static_cast<const __bf16*>(dout),
                       static_cast<const float*>(nl), static_cast<const float*>(nd), dq_acc,
                       static_cast<__bf16*>(dk), static_cast<__bf16*>(dv), s, dq_st, dq_sh, dq_sb);
    hipLaunchKernelGGL(dq_k, dim3(rblocks), dim3(256), 0, st, static_cast<const float*>(dq_acc),
                       static_cast<__bf16*>(dq), s, dq_st, dq_sh, dq_sb);
  };
  if (D == 128) causal ? run(attn_bwd_delta<128>, attn_bwd<128, true>, attn_bwd_dq<128>)
                       : run(attn_bwd_delta<128>, attn_bwd<128, false>, attn_bwd_dq<128>);
  else causal ? run(attn_bwd_delta<64>, attn_bwd<64, true>, attn_bwd_dq<64>)
              : run(attn_bwd_delta<64>, attn_bwd<64, false>, attn_bwd_dq<64>);
  e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
