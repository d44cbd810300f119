// gemm_bf16_w4_sk.hip — stream-K on the w4 template (gemm_w4.h SK): the argument checks and the
// dispatch to the kernel variants, which build one per translation unit (kernels/tu/w4_sk_*.hip).
#include "gemm_w4.h"

using namespace kfw4;

// the kernel variants, one translation unit each (kernels/tu/w4_sk_*.hip, gemm_w4_sk.h)
extern "C" {
int kfw4_sk_none_11(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
int kfw4_sk_none_10(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
int kfw4_sk_none_01(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
int kfw4_sk_none_00(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
int kfw4_sk_relu_10(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
int kfw4_sk_relu_00(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
int kfw4_sk_gelu_10(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
int kfw4_sk_gelu_00(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
int kfw4_sk_silu_10(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
int kfw4_sk_silu_00(const void*, const void*, void*, const void*, const void*, int, int, int, long long, long long, long long,
                    long long, float, float*, unsigned*, unsigned, int, int, void*);
}

// Stream-K on the 256x256 tile (NT layout, batch 1): a persistent grid of `grid` blocks (one per CU)
// runs the whole waves of tiles, then the remaining rem = tiles % grid tiles in `splits` K-splits
// each, round-robin over all blocks (gemm_w4.h SK). W: (splits - 1) * rem partial tiles of 256 x 256
// fp32; flags: splits * rem words, never holding `epoch` from an earlier call (the caller keeps one
// buffer per stream and a strictly increasing epoch). Negative `splits`: every owner recomputes its
// producers' splits after the deadline (tests of that path).
extern "C" int kfamd_w4_streamk_nt(const void* A, const void* B, void* C, const void* bias, const void* R, void* Aux,
                                   int M, int N, int K, long long lda, long long ldb, long long ldc, long long ldr,
                                   float alpha, int act, float* W, unsigned* flags, unsigned epoch, int grid,
                                   int splits, void* stream) {
  const int rc = check_shape(0, 0, 256, A, B, C, bias, R, Aux, M, N, K, lda, ldb, ldc, ldr, 0, 0, 0, 0);
  if (rc != KFAMD_OK) return rc;
  if (!W || !flags || epoch == 0 || grid < 8 || grid > 4096) return KFAMD_EINVAL;
  // no pre-activation output: the second output's registers push the persistent loop's accumulators
  // into scratch (the Aux forward runs on the plain kernel)
  if (Aux) return KFAMD_EINVAL;
  if (R && act != KFAMD_ACT_NONE) return KFAMD_EINVAL;
  if ((reinterpret_cast<uintptr_t>(W) & 15) || (reinterpret_cast<uintptr_t>(flags) & 3)) return KFAMD_EALIGN;
  // an owner tracks its producers in a 64-bit mask; every split holds at least one K-tile
  const int KT = (K + kBK - 1) / kBK;
  // (splits < 0: the deadline path's test mode, see gemm_w4.h)
  const int S = splits < 0 ? -splits : splits;
  if (S < 1 || S > 64 || S > KT) return KFAMD_EINVAL;
  const bool hb = bias != nullptr, hr = R != nullptr;
#define SK_LAUNCH(A_, B_, R_) \
  return kfw4_sk_##A_##_##B_##R_(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, W, flags, epoch, grid, splits, stream)
  switch (act) {
    case KFAMD_ACT_NONE:
      if (hb && hr) SK_LAUNCH(none, 1, 1);
      if (hb) SK_LAUNCH(none, 1, 0);
      if (hr) SK_LAUNCH(none, 0, 1);
      SK_LAUNCH(none, 0, 0);
    case KFAMD_ACT_RELU:
      if (hb) SK_LAUNCH(relu, 1, 0);
      SK_LAUNCH(relu, 0, 0);
    case KFAMD_ACT_GELU_TANH:
      if (hb) SK_LAUNCH(gelu, 1, 0);
      SK_LAUNCH(gelu, 0, 0);
    case KFAMD_ACT_SILU:
      if (hb) SK_LAUNCH(silu, 1, 0);
      SK_LAUNCH(silu, 0, 0);
    default:
      return KFAMD_EINVAL;
  }
#undef SK_LAUNCH
}

