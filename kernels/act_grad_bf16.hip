// act_grad_bf16.hip — the elementwise tail of a linear layer's backward, fused into one HBM pass:
//   g = dY * act'(z)            (z = the pre-activation the forward GEMM stored as its Aux output;
//                                relu takes the forward OUTPUT y instead: act'(.) = y > 0)
//   db[n] = sum_m g[m][n]       (bias gradient, fp32, optional)
// so autograd reads dY and z once and writes g once, instead of torch's gelu-backward + a separate
// column reduction. g then feeds the dgrad/wgrad GEMMs (gemm_bf16_w4_t.hip).
//
// Layout: [rows][cols] bf16, cols % 8 == 0, 16-B aligned rows. A block is 4 waves over 512
// columns (one 16-B vector per lane) and kRowsPerBlock rows (each wave a quarter of them, so every
// SIMD keeps several 16-B loads in flight); the waves' fp32 column sums meet in LDS and one
// [row blocks][cols] workspace row per block is folded by a second, column-parallel launch
// (deterministic: no float atomics). 8192x4096: 8 x 256 = 2048 blocks, 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kfamd_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kThreads = 256, kWaves = 4, kRowsPerBlock = 32, kCols = 64 * 8;

__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

__device__ __forceinline__ float dact(float z, int act) {
  switch (act) {
    case KFAMD_ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case KFAMD_ACT_GELU_TANH: {
      // gelu_tanh(z) = z * s(2u), u = c (z + 0.044715 z^3): d/dz = s + z s (1 - s) 2u'
      const float c2 = 1.5957691216057308f;
      const float z2 = z * z;
      const float sg = sigm(c2 * (z + 0.044715f * z2 * z));
      return sg + z * sg * (1.f - sg) * c2 * (1.f + 3.f * 0.044715f * z2);
    }
    case KFAMD_ACT_SILU: {
      const float sg = sigm(z);
      return sg * (1.f + z * (1.f - sg));
    }
    default: return 1.f;
  }
}

template <int ACT, bool WRITE_G, bool SUM>
__global__ __launch_bounds__(kThreads) void act_grad(const __bf16* __restrict__ dy, const __bf16* __restrict__ z,
                                                     __bf16* __restrict__ g, float* __restrict__ ws, int rows,
                                                     int cols) {
  __shared__ float red[kWaves - 1][kCols];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c8 = blockIdx.x * kCols + lane * 8;
  const bool col_ok = c8 < cols;
  const int r0 = blockIdx.y * kRowsPerBlock, r1 = min(rows, r0 + kRowsPerBlock);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col_ok) {
#pragma unroll 4
    for (int r = r0 + wave; r < r1; r += kWaves) {
      const long long off = (long long)r * cols + c8;
      const bf16x8 d = *reinterpret_cast<const bf16x8*>(dy + off);
      if (ACT != KFAMD_ACT_NONE) {
        const bf16x8 zz = *reinterpret_cast<const bf16x8*>(z + off);
        bf16x8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          o[i] = (__bf16)((float)d[i] * dact((float)zz[i], ACT));
          // the bias gradient sums what the GEMMs consume: the bf16-rounded g
          if (SUM) acc[i] += (float)o[i];
        }
        if (WRITE_G) *reinterpret_cast<bf16x8*>(g + off) = o;
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += (float)d[i];
      }
    }
  }
  if (!SUM) return;
  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[wave - 1][lane * 8 + i] = acc[i];
  }
  __syncthreads();
  if (wave == 0 && col_ok) {
#pragma unroll
    for (int w = 0; w < kWaves - 1; ++w)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += red[w][lane * 8 + i];
    float* o = ws + (long long)blockIdx.y * cols + c8;
    *reinterpret_cast<float4*>(o) = float4{acc[0], acc[1], acc[2], acc[3]};
    *reinterpret_cast<float4*>(o + 4) = float4{acc[4], acc[5], acc[6], acc[7]};
  }
}

// db[c] = sum over row blocks of ws[b][c]: 64 columns x 4 row-slices per 256-thread block
// OB: write the sums as bf16 (the bias dtype: saves autograd a separate cast launch per bias)
template <bool OB>
__global__ __launch_bounds__(256) void colsum_finalize(const float* __restrict__ ws, void* __restrict__ db, int nblk,
                                                       int cols) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < cols) {
#pragma unroll 8
    for (int b = sl; b < nblk; b += 4) s += ws[(long long)b * cols + c];
  }
  red[sl][cl] = s;
  __syncthreads();
  if (sl == 0 && c < cols) {
    const float v = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    if (OB) static_cast<__bf16*>(db)[c] = (__bf16)v;
    else static_cast<float*>(db)[c] = v;
  }
}

// Forward activation as its own HBM pass: y = act(z), n elements (n % 8 == 0, 16-B aligned). For
// large linears this beats applying gelu / silu in the GEMM epilogue: there the exp / rcp run at one
// wave per SIMD with the MFMA pipe idle, after every CU's tile finishes at the same moment
// (profiles/r3_train_step); here they run at full occupancy under the memory stream. Used by
// ops.gemm_nt_preact in its "split" mode (A/B runs; the fused epilogue is the default).
__global__ __launch_bounds__(256) void act_fwd(const __bf16* __restrict__ z, __bf16* __restrict__ y, long long n8, int act) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const bf16x8 v = reinterpret_cast<const bf16x8*>(z)[i];
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float x = (float)v[k];
      float r;
      if (act == KFAMD_ACT_GELU_TANH) r = x * sigm(1.5957691216057308f * (x + 0.044715f * x * x * x));
      else if (act == KFAMD_ACT_SILU) r = x * sigm(x);
      else if (act == KFAMD_ACT_RELU) r = x > 0.f ? x : 0.f;
      else r = x;
      o[k] = (__bf16)r;
    }
    reinterpret_cast<bf16x8*>(y)[i] = o;
  }
}

}  // namespace

extern "C" int kfamd_act_fwd_bf16(const void* z, void* y, long long n, int act, void* stream) {
  if (!z || !y || n <= 0 || n % 8 || act < KFAMD_ACT_NONE || act > KFAMD_ACT_SILU) return KFAMD_EINVAL;
  if ((reinterpret_cast<uintptr_t>(z) | reinterpret_cast<uintptr_t>(y)) & 15) return KFAMD_EALIGN;
  const long long n8 = n / 8;
  const long long want = (n8 + 255) / 256;
  dim3 grid((unsigned)(want < 256 * 16 ? want : 256 * 16)), block(256);
  hipLaunchKernelGGL(act_fwd, grid, block, 0, reinterpret_cast<hipStream_t>(stream), static_cast<const __bf16*>(z),
                     static_cast<__bf16*>(y), n8, act);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

extern "C" long long kfamd_act_grad_workspace(int rows, int cols) {
  return (long long)((rows + kRowsPerBlock - 1) / kRowsPerBlock) * cols * (long long)sizeof(float);
}

// g = dy * act'(z) (g may be null when act == NONE: only the column sums are produced);
// db ([cols], optional; fp32, or bf16 when db_bf16) = column sums of g (accumulated in fp32);
// workspace: kfamd_act_grad_workspace bytes (when db).
extern "C" int kfamd_act_grad_bf16_v2(const void* dy, const void* z, void* g, void* db, int db_bf16, float* workspace,
                                      int rows, int cols, int act, void* stream) {
  if (!dy || rows <= 0 || cols <= 0 || cols % 8) return KFAMD_EINVAL;
  if (act < KFAMD_ACT_NONE || act > KFAMD_ACT_SILU) return KFAMD_EINVAL;
  if (act != KFAMD_ACT_NONE && (!z || !g)) return KFAMD_EINVAL;
  if (act == KFAMD_ACT_NONE && !db) return KFAMD_EINVAL;
  if (db && !workspace) return KFAMD_EINVAL;
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al(dy) || !al(z) || !al(g) || !al(workspace)) return KFAMD_EALIGN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nblk = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
  dim3 grid((cols + kCols - 1) / kCols, nblk), block(kThreads);
  const __bf16* d = static_cast<const __bf16*>(dy);
  const __bf16* zz = static_cast<const __bf16*>(z);
  __bf16* gg = static_cast<__bf16*>(g);
  const bool sum = db != nullptr;
#define AG(ACTV)                                                                                              \
  if (sum) hipLaunchKernelGGL((act_grad<ACTV, true, true>), grid, block, 0, s, d, zz, gg, workspace, rows, cols); \
  else hipLaunchKernelGGL((act_grad<ACTV, true, false>), grid, block, 0, s, d, zz, gg, workspace, rows, cols)
  switch (act) {
    case KFAMD_ACT_NONE:
      hipLaunchKernelGGL((act_grad<KFAMD_ACT_NONE, false, true>), grid, block, 0, s, d, zz, gg, workspace, rows, cols);
      break;
    case KFAMD_ACT_RELU: AG(KFAMD_ACT_RELU); break;
    case KFAMD_ACT_GELU_TANH: AG(KFAMD_ACT_GELU_TANH); break;
    case KFAMD_ACT_SILU: AG(KFAMD_ACT_SILU); break;
  }
#undef AG
  if (sum) {
    if (db_bf16) hipLaunchKernelGGL(colsum_finalize<true>, dim3((cols + 63) / 64), dim3(256), 0, s, workspace, db, nblk, cols);
    else hipLaunchKernelGGL(colsum_finalize<false>, dim3((cols + 63) / 64), dim3(256), 0, s, workspace, db, nblk, cols);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

extern "C" int kfamd_colsum_finalize(const float* ws, void* db, int db_bf16, int nblk, int cols, void* stream) {
  if (!ws || !db || nblk <= 0 || cols <= 0) return KFAMD_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (db_bf16) hipLaunchKernelGGL(colsum_finalize<true>, dim3((cols + 63) / 64), dim3(256), 0, s, ws, db, nblk, cols);
  else hipLaunchKernelGGL(colsum_finalize<false>, dim3((cols + 63) / 64), dim3(256), 0, s, ws, db, nblk, cols);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

extern "C" int kfamd_act_grad_bf16(const void* dy, const void* z, void* g, float* db, float* workspace, int rows,
                                   int cols, int act, void* stream) {
  return kfamd_act_grad_bf16_v2(dy, z, g, db, 0, workspace, rows, cols, act, stream);
}
