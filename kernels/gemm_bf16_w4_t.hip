// gemm_bf16_w4_t.hip — the w4 GEMM template (gemm_w4.h) in the operand layouts of a linear layer's
// backward, so autograd never materialises a transposed copy:
//   dgrad  dX[M][K]  = dY[M][N] · W[N][K]      -> LA = 0 (dY K-contiguous), LB = 1 (W k-major)
//   wgrad  dW[N][K]  = dY[M][N]^T · X[M][K]    -> LA = 1 (dY k-major),      LB = 1 (X k-major)
//   and LA = 1, LB = 0 for completeness (A^T B^T products).
// Epilogue: alpha and an optional residual R (R may alias C: gradient accumulation, C += A·B).
#include "gemm_w4.h"

using namespace kfw4;

namespace {

template <int LA, int LB, int BM>
int launch_t(const void* A, const void* B, void* C, const void* R, int M, int N, int K, int batch, long long lda,
             long long ldb, long long ldc, long long ldr, long long sa, long long sb, long long sc, long long sr,
             float alpha, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(((M + BM - 1) / BM) * ((N + BM - 1) / BM), batch), block(kThreads);
  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
  __bf16* c = static_cast<__bf16*>(C);
  const __bf16* r = static_cast<const __bf16*>(R);
  if (R)
    hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, true, false, LA, LB, BM>), grid, block, 0, s, a, b, c, nullptr,
                       r, nullptr, M, N, K, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, nullptr);
  else
    hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, LA, LB, BM>), grid, block, 0, s, a, b, c,
                       nullptr, nullptr, nullptr, M, N, K, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, nullptr);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

}  // namespace

// Split-K partials of the transposed layouts on the 128x128 tile (see kfamd_w4_splitk_nt).
extern "C" int kfamd_w4_splitk_t(int la, int lb, const void* A, const void* B, float* W, int M, int N, int K,
                                 int batch, int splits, int kper, long long lda, long long ldb, long long sa,
                                 long long sb, void* stream) {
  const int rc = check_shape(la, lb, 128, A, B, W, nullptr, nullptr, nullptr, M, N, K, lda, ldb, N, 0, sa, sb, 0, 0);
  if (rc != KFAMD_OK) return rc;
  if (splits < 1 || kper < kBK || kper % kBK || (long long)kper * (splits - 1) >= K || !W || N % 8) return KFAMD_EINVAL;
  if (reinterpret_cast<uintptr_t>(W) & 15) return KFAMD_EALIGN;
  dim3 grid(((M + 127) / 128) * ((N + 127) / 128), batch, splits), block(kThreads);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
#define W4S(LA_, LB_)                                                                                             \
  if (la == LA_ && lb == LB_) {                                                                                   \
    hipLaunchKernelGGL((gemm_w4<KFAMD_ACT_NONE, false, false, false, LA_, LB_, 128, true>), grid, block, 0, s, a, b, \
                       nullptr, nullptr, nullptr, nullptr, M, N, K, lda, ldb, 0LL, 0LL, sa, sb, 0LL, 0LL, 1.0f,     \
                       nullptr, W, kper);                                                                         \
    const hipError_t e = hipGetLastError();                                                                       \
    return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);                                                      \
  }
  W4S(0, 1)
  W4S(1, 1)
  W4S(1, 0)
#undef W4S
  return KFAMD_EINVAL;
}

// la/lb: 0 = K-contiguous operand, 1 = k-major (see gemm_w4.h); (0, 0) is kfamd_w4_launch_nt.
extern "C" int kfamd_w4_launch_t(int la, int lb, int bm, const void* A, const void* B, void* C, const void* R, int M,
                                 int N, int K, int batch, long long lda, long long ldb, long long ldc, long long ldr,
                                 long long sa, long long sb, long long sc, long long sr, float alpha, void* stream) {
  const int rc = check_shape(la, lb, bm, A, B, C, nullptr, R, nullptr, M, N, K, lda, ldb, ldc, ldr, sa, sb, sc, sr);
  if (rc != KFAMD_OK) return rc;
#define W4T(LA_, LB_)                                                                                              \
  if (la == LA_ && lb == LB_) {                                                                                    \
    if (bm == 256) return launch_t<LA_, LB_, 256>(A, B, C, R, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr,  \
                                                   alpha, stream);                                                 \
    if (bm == 128) return launch_t<LA_, LB_, 128>(A, B, C, R, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr,  \
                                                   alpha, stream);                                                 \
    return KFAMD_EINVAL;                                                                                           \
  }
  W4T(0, 1)
  W4T(1, 1)
  W4T(1, 0)
#undef W4T
  return KFAMD_EINVAL;
}

// the split-K fixup kernels, one operand layout per translation unit (kernels/tu/w4_fix_*.hip)
extern "C" {
#define KFW4_FIX_DECL(NAME)                                                                                        \
  int NAME(const void*, const void*, void*, const void*, int, int, int, int, long long, long long, long long,      \
           long long, long long, long long, long long, long long, float, float*, unsigned*, int, int, void*);
KFW4_FIX_DECL(kfw4_fix_00)
KFW4_FIX_DECL(kfw4_fix_11)
KFW4_FIX_DECL(kfw4_fix_01)
#undef KFW4_FIX_DECL
}

// Split-K with the in-kernel fixup on the 256x256 tile (gemm_w4.h SPLIT == 2): `splits` blocks per
// tile over K ranges of kper (kper % 64 == 0, every split non-empty); the last block of each tile to
// arrive adds the others' fp32 partials and runs the epilogue (alpha, optional residual R, which may
// alias C). W: splits * batch * tiles partial tiles of 256 x 256 fp32 (16-B aligned); cnt: batch *
// tiles arrival counters, zero on entry and left zero on exit (one buffer per stream).
extern "C" int kfamd_w4_splitk_fix(int la, int lb, const void* A, const void* B, void* C, const void* R, int M, int N,
                                   int K, int batch, long long lda, long long ldb, long long ldc, long long ldr,
                                   long long sa, long long sb, long long sc, long long sr, float alpha, float* W,
                                   unsigned* cnt, int splits, int kper, void* stream) {
  const int rc = check_shape(la, lb, 256, A, B, C, nullptr, R, nullptr, M, N, K, lda, ldb, ldc, ldr, sa, sb, sc, sr);
  if (rc != KFAMD_OK) return rc;
  if (!W || !cnt || splits < 2 || splits > 64 || kper < kBK || kper % kBK || (long long)kper * (splits - 1) >= K)
    return KFAMD_EINVAL;
  if ((reinterpret_cast<uintptr_t>(W) & 15) || (reinterpret_cast<uintptr_t>(cnt) & 3)) return KFAMD_EALIGN;
#define FIX(LA_, LB_)                                                                                              \
  if (la == LA_ && lb == LB_)                                                                                      \
    return kfw4_fix_##LA_##LB_(A, B, C, R, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, alpha, W, cnt, splits, \
                               kper, stream);
  FIX(0, 0)
  FIX(1, 1)
  FIX(0, 1)
#undef FIX
  return KFAMD_EINVAL;
}
