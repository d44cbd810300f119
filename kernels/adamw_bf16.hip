// adamw_bf16.hip — multi-tensor AdamW (decoupled weight decay) over bf16 parameters, gradients and
// moments in ONE launch per step. A tensor table (device memory, rebuilt by the host only when a
// pointer changes) lists every tensor with its first chunk index; block b finds its tensor by a binary
// search over those chunk starts and updates 8 elements per thread per step (16-B loads / stores).
// The update is torch's: p -= lr*wd*p; m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g^2;
// p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps), in fp32, rounded once to bf16 per tensor.
// It moves 14 B per parameter (p, m, v read + written, g read): gpt-1b's 1.28 G parameters are 18 GB,
// ~3.3 ms at the HBM roof, where torch's fused AdamW took 5.7 ms (profiles/r4_train_trace).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "kfamd_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct AdamWTensor {  // 48 bytes, host-written (kfamd_adamw_tensor_bytes)
  __bf16* p;
  const __bf16* g;
  __bf16* m;
  __bf16* v;
  long long n;
  long long chunk0;  // first chunk of this tensor in the launch
};

constexpr int kChunk = 8 * 256 * 8;  // elements per block: 8 steps of 8 elements per thread

__global__ __launch_bounds__(256) void adamw(const AdamWTensor* __restrict__ tab, const int* __restrict__ owner,
                                             float lr, float b1, float b2, float eps, float wd, float step_size,
                                             float inv_sqrt_bc2) {
  const long long cb = blockIdx.x;
  const AdamWTensor t = tab[owner[cb]];  // the tensor this chunk belongs to (host-built map)
  const long long base = (cb - t.chunk0) * kChunk;
  const long long end = min(t.n, base + kChunk);
  const float decay = 1.f - lr * wd;
  const bool vec = !((reinterpret_cast<uintptr_t>(t.p) | reinterpret_cast<uintptr_t>(t.g) |
                      reinterpret_cast<uintptr_t>(t.m) | reinterpret_cast<uintptr_t>(t.v)) & 15);
  if (vec) {
    for (long long i = base + threadIdx.x * 8; i + 8 <= end; i += 256 * 8) {
      bf16x8 P = *reinterpret_cast<const bf16x8*>(t.p + i);
      const bf16x8 G = *reinterpret_cast<const bf16x8*>(t.g + i);
      bf16x8 Mv = *reinterpret_cast<const bf16x8*>(t.m + i);
      bf16x8 Vv = *reinterpret_cast<const bf16x8*>(t.v + i);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = (float)G[e];
        const float m = b1 * (float)Mv[e] + (1.f - b1) * g;
        const float v = b2 * (float)Vv[e] + (1.f - b2) * g * g;
        const float p = (float)P[e] * decay - step_size * m / (sqrtf(v) * inv_sqrt_bc2 + eps);
        P[e] = (__bf16)p;
        Mv[e] = (__bf16)m;
        Vv[e] = (__bf16)v;
      }
      *reinterpret_cast<bf16x8*>(t.p + i) = P;
      *reinterpret_cast<bf16x8*>(t.m + i) = Mv;
      *reinterpret_cast<bf16x8*>(t.v + i) = Vv;
    }
    // the tail of a tensor whose length is not a multiple of 8
    const long long tail = base + ((end - base) / 8) * 8;
    for (long long i = tail + threadIdx.x; i < end; i += 256) {
      const float g = (float)t.g[i];
      const float m = b1 * (float)t.m[i] + (1.f - b1) * g;
      const float v = b2 * (float)t.v[i] + (1.f - b2) * g * g;
      t.p[i] = (__bf16)((float)t.p[i] * decay - step_size * m / (sqrtf(v) * inv_sqrt_bc2 + eps));
      t.m[i] = (__bf16)m;
      t.v[i] = (__bf16)v;
    }
  } else {
    for (long long i = base + threadIdx.x; i < end; i += 256) {
      const float g = (float)t.g[i];
      const float m = b1 * (float)t.m[i] + (1.f - b1) * g;
      const float v = b2 * (float)t.v[i] + (1.f - b2) * g * g;
      t.p[i] = (__bf16)((float)t.p[i] * decay - step_size * m / (sqrtf(v) * inv_sqrt_bc2 + eps));
      t.m[i] = (__bf16)m;
      t.v[i] = (__bf16)v;
    }
  }
}

}  // namespace

// bytes per table entry and elements per chunk (the host builds the table: p, g, m, v pointers, n,
// first chunk; chunks of one tensor are consecutive, tensors in table order)
extern "C" int kfamd_adamw_tensor_bytes() { return (int)sizeof(AdamWTensor); }
extern "C" int kfamd_adamw_chunk() { return kChunk; }

// one AdamW step over every tensor of a device-resident table; nchunks = the table's total chunks,
// step_size = lr / (1 - b1^t), inv_sqrt_bc2 = 1 / sqrt(1 - b2^t).
// owner: nchunks int32, the table row of each chunk.
extern "C" int kfamd_adamw_bf16(const void* table, const void* owner, long long nchunks, float lr, float b1, float b2,
                                float eps, float wd, float step_size, float inv_sqrt_bc2, void* stream) {
  if (!table || !owner || nchunks <= 0 || nchunks > 0x7fffffffLL) return KFAMD_EINVAL;
  if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(owner) & 3)) return KFAMD_EALIGN;
  hipLaunchKernelGGL(adamw, dim3((unsigned)nchunks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const AdamWTensor*>(table), static_cast<const int*>(owner), lr, b1, b2, eps, wd,
                     step_size, inv_sqrt_bc2);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
