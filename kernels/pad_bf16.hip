// pad_bf16.hip — K-padding pack for GEMM operands whose inner extent is off the 8-element grid
// (e.g. K = 1500): dst[r][0:Kp] = src[r][0:K], dst[r][K:Kp] = 0, for up to two matrices in ONE
// launch (both GEMM operands), so the w4 MFMA kernel's 16-B buffer loads see aligned rows. The
// output side needs no pack: the w4 epilogue stores any N / ldc itself (gemm_w4.h, odd path).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kfamd_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct PadJob {
  const __bf16* src;
  __bf16* dst;
  long long chunks;  // rows * (Kp / 8)
  long long ld;      // source row stride (elements)
  int K;
};

// One 16-B output chunk per thread; source reads V elements wide (V = the widest the source rows'
// alignment allows: 4 when ld % 4 == 0 and the base is 8-B aligned, ...).
template <int V>
__device__ __forceinline__ void pad_chunk(const PadJob& j, unsigned c, unsigned kp8) {
  const unsigned row = c / kp8;  // 32-bit: the launcher bounds the chunk count (no 64-bit divide)
  const int k0 = (int)(c - row * kp8) * 8;
  const __bf16* s = j.src + (long long)row * j.ld + k0;
  bf16x8 o;
  if (k0 + 8 <= j.K) {
#pragma unroll
    for (int q = 0; q < 8; q += V) {
      if constexpr (V == 4) {
        const uint2 u = *reinterpret_cast<const uint2*>(s + q);
        const auto p = __builtin_bit_cast(__bf16 __attribute__((ext_vector_type(4))), u);
        o[q] = p[0]; o[q + 1] = p[1]; o[q + 2] = p[2]; o[q + 3] = p[3];
      } else if constexpr (V == 2) {
        const unsigned u = *reinterpret_cast<const unsigned*>(s + q);
        const auto p = __builtin_bit_cast(__bf16 __attribute__((ext_vector_type(2))), u);
        o[q] = p[0]; o[q + 1] = p[1];
      } else {
        o[q] = s[q];
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = k0 + q < j.K ? s[q] : (__bf16)0.f;
  }
  *reinterpret_cast<bf16x8*>(j.dst + (long long)row * kp8 * 8 + k0) = o;
}

template <int V0, int V1>
__global__ void __launch_bounds__(256) pad_k(PadJob j0, PadJob j1, unsigned kp8) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < j0.chunks) pad_chunk<V0>(j0, t, kp8);
  else if (t - j0.chunks < j1.chunks) pad_chunk<V1>(j1, t - (unsigned)j0.chunks, kp8);
}

int vec_width(const void* p, long long ld) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  if ((a & 7) == 0 && ld % 4 == 0) return 4;
  if ((a & 3) == 0 && ld % 2 == 0) return 2;
  return 1;
}

}  // namespace

// dst0 = pad(src0 [rows0][K] (row stride ld0)) to [rows0][Kp] (Kp % 8 == 0, Kp >= K), same for
// src1/dst1 (rows1 = 0: single matrix). dst rows are dense (stride Kp) and 16-B aligned.
extern "C" int kfamd_pad_k_bf16(const void* src0, void* dst0, long long rows0, long long ld0, const void* src1,
                                void* dst1, long long rows1, long long ld1, int K, int Kp, void* stream) {
  if (!src0 || !dst0 || rows0 <= 0 || rows1 < 0 || K <= 0 || Kp < K || Kp % 8 || ld0 < K) return KFAMD_EINVAL;
  if (rows1 > 0 && (!src1 || !dst1 || ld1 < K)) return KFAMD_EINVAL;
  if ((reinterpret_cast<uintptr_t>(dst0) & 15) || (rows1 > 0 && (reinterpret_cast<uintptr_t>(dst1) & 15)) ||
      (reinterpret_cast<uintptr_t>(src0) & 1) || (rows1 > 0 && (reinterpret_cast<uintptr_t>(src1) & 1)))
    return KFAMD_EALIGN;
  const int kp8 = Kp / 8;
  PadJob j0{static_cast<const __bf16*>(src0), static_cast<__bf16*>(dst0), rows0 * kp8, ld0, K};
  PadJob j1{static_cast<const __bf16*>(src1), static_cast<__bf16*>(dst1), rows1 * kp8, ld1, K};
  const long long total = j0.chunks + j1.chunks;
  if (total >= (1LL << 31)) return KFAMD_EINVAL;
  dim3 grid((unsigned)((total + 255) / 256)), block(256);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int v0 = vec_width(src0, ld0), v1 = rows1 > 0 ? vec_width(src1, ld1) : v0;
#define PAD_L(A_, B_) if (v0 == A_ && v1 == B_) hipLaunchKernelGGL((pad_k<A_, B_>), grid, block, 0, s, j0, j1, kp8)
  PAD_L(4, 4); else PAD_L(4, 2); else PAD_L(4, 1); else PAD_L(2, 4); else PAD_L(2, 2); else PAD_L(2, 1);
  else PAD_L(1, 4); else PAD_L(1, 2); else PAD_L(1, 1);
#undef PAD_L
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
