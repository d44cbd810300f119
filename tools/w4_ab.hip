// w4 GEMM schedule A/B builds (tools/w4_ab.py): the production NT kernel (no epilogue options) and its
// stamped diagnostic twin, compiled with one set of -DKFW4_* schedule knobs per library
// (gemm_w4.h; the defaults are the production schedule). Scratch builds only, never linked into
// libkfamd_kernels.so.
#include "gemm_w4.h"

using namespace kfw4;

extern "C" int w4ab_nt(const void* A, const void* B, void* C, int M, int N, int K, void* stream) {
  const int rc = check_shape(0, 0, 256, A, B, C, nullptr, nullptr, nullptr, M, N, K, K, K, N, 0, 0, 0, 0, 0);
  if (rc != KFAMD_OK) return rc;
  dim3 grid(((M + 255) / 256) * ((N + 255) / 256), 1), block(kThreads);
  hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, 0, 0, 256>), grid, block, 0,
                     reinterpret_cast<hipStream_t>(stream), static_cast<const __bf16*>(A),
                     static_cast<const __bf16*>(B), static_cast<__bf16*>(C), nullptr, nullptr, nullptr, M, N, K,
                     (long long)K, (long long)K, (long long)N, 0LL, 0LL, 0LL, 0LL, 0LL, 1.0f, nullptr);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

// diag: [tiles][4 waves][16] u64 per wave (gemm_w4.h DIAG block); needs M, N % 256 and K % 64
extern "C" int w4ab_diag(const void* A, const void* B, void* C, int M, int N, int K, unsigned long long* diag,
                         void* stream) {
  if (M % 256 || N % 256 || K % kBK || !diag) return KFAMD_EINVAL;
  dim3 grid((M / 256) * (N / 256), 1), block(kThreads);
  hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, 0, 0, 256, false, true, 0>), grid, block, 0,
                     reinterpret_cast<hipStream_t>(stream), static_cast<const __bf16*>(A),
                     static_cast<const __bf16*>(B), static_cast<__bf16*>(C), nullptr, nullptr, nullptr, M, N, K,
                     (long long)K, (long long)K, (long long)N, 0LL, 0LL, 0LL, 0LL, 0LL, 1.0f, diag);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

// persistent, overlapped schedule (gemm_w4.h PO): `grid` blocks (a multiple of 8, e.g. the CU count)
// each run tiles b, b + grid, ... of the XCD-remapped order
extern "C" int w4ab_po(const void* A, const void* B, void* C, int M, int N, int K, int grid_blocks, void* stream) {
  const int rc = check_shape(0, 0, 256, A, B, C, nullptr, nullptr, nullptr, M, N, K, K, K, N, 0, 0, 0, 0, 0);
  if (rc != KFAMD_OK) return rc;
  const int nwg = ((M + 255) / 256) * ((N + 255) / 256);
  if (grid_blocks <= 0 || grid_blocks % 8) return KFAMD_EINVAL;
  dim3 grid(grid_blocks < nwg ? grid_blocks : nwg, 1), block(kThreads);
  hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, 0, 0, 256, 0, false, 0, false, true>), grid,
                     block, 0, reinterpret_cast<hipStream_t>(stream), static_cast<const __bf16*>(A),
                     static_cast<const __bf16*>(B), static_cast<__bf16*>(C), nullptr, nullptr, nullptr, M, N, K,
                     (long long)K, (long long)K, (long long)N, 0LL, 0LL, 0LL, 0LL, 0LL, 1.0f, nullptr);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
