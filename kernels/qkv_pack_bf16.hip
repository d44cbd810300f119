// qkv_pack_bf16.hip — the attention backward's dq / dk / dv ([B, H, T, D] each, any strides with a
// contiguous head dim) written straight into the fused QKV projection's gradient layout
// out[b][t][s][h][d] (s = q, k, v), one pass. Autograd's own route for the view/permute of the QKV
// output stacks the three ([3, B, H, T, D]) and then permutes that copy: two full passes over
// 96 MiB per gpt-1b layer at 1.4 TB/s (204 us, profiles/r4_train_trace), where this is one
// read and one write at 16 B per thread.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kfamd_kernels.h"

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void qkv_pack(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                const __bf16* __restrict__ v, __bf16* __restrict__ out, int B, int T,
                                                int H, int D8, long long qb, long long qh, long long qt, long long kb,
                                                long long kh, long long kt, long long vb, long long vh, long long vt) {
  const long long n = (long long)B * T * 3 * H * D8;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  long long r = idx;
  const int d8 = (int)(r % D8);
  r /= D8;
  const int h = (int)(r % H);
  r /= H;
  const int s = (int)(r % 3);
  r /= 3;
  const int t = (int)(r % T);
  const int b = (int)(r / T);
  const __bf16* src = s == 0 ? q : (s == 1 ? k : v);
  const long long sb = s == 0 ? qb : (s == 1 ? kb : vb), sh = s == 0 ? qh : (s == 1 ? kh : vh),
                  st = s == 0 ? qt : (s == 1 ? kt : vt);
  u32x4 val = {0u, 0u, 0u, 0u};
  if (src) val = *reinterpret_cast<const u32x4*>(src + b * sb + h * sh + t * st + d8 * 8);
  *reinterpret_cast<u32x4*>(out + idx * 8) = val;
}

}  // namespace

// dq / dk / dv: [B][H][T][D] with element strides (b, h, t) each, head dim contiguous; a null source
// packs zeros (a gradient autograd did not produce). out: [B][T][3][H][D] contiguous. D % 8, every
// source row and out 16-B aligned.
extern "C" int kfamd_qkv_pack_bf16(const void* dq, const void* dk, const void* dv, void* out, int B, int T, int H, int D,
                                   long long qb, long long qh, long long qt, long long kb, long long kh, long long kt,
                                   long long vb, long long vh, long long vt, void* stream) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!out || B <= 0 || T <= 0 || H <= 0 || D <= 0 || D % 8) return KFAMD_EINVAL;
  if (!al16(out) || !al16(dq) || !al16(dk) || !al16(dv)) return KFAMD_EALIGN;
  if ((qb | qh | qt | kb | kh | kt | vb | vh | vt) & 7) return KFAMD_EALIGN;
  const long long n = (long long)B * T * 3 * H * (D / 8);
  hipLaunchKernelGGL(qkv_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const __bf16*>(dq), static_cast<const __bf16*>(dk), static_cast<const __bf16*>(dv),
                     static_cast<__bf16*>(out), B, T, H, D / 8, qb, qh, qt, kb, kh, kt, vb, vh, vt);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
