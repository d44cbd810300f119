// gemm_w4_nt.h — the forward ("NT") launcher of the w4 template for ONE activation: each
// kernels/tu/w4_nt_<act>.hip instantiates it for its activation, so the kernel variants build
// as separate translation units in parallel (and never perturb each other's code generation:
// cdna_hip_programming.md §5.4 rule 19); kernels/gemm_bf16_w4.hip dispatches on the activation.
#pragma once
#include "gemm_w4.h"

namespace kfw4 {
namespace {

template <int BM, int ACT>
int launch_nt_act(const void* A, const void* B, void* C, const void* bias, const void* R, void* Aux, int M, int N,
                  int K, int batch, long long lda, long long ldb, long long ldc, long long ldr, long long sa,
                  long long sb, long long sc, long long sr, float alpha, void* stream) {
  const int rc = check_shape(0, 0, BM, A, B, C, bias, R, Aux, M, N, K, lda, ldb, ldc, ldr, sa, sb, sc, sr);
  if (rc != KFAMD_OK) return rc;
  if (Aux && (ACT == KFAMD_ACT_NONE || R)) return KFAMD_EINVAL;
  if (R && ACT != KFAMD_ACT_NONE) return KFAMD_EINVAL;
  if (Aux && ACT == KFAMD_ACT_RELU) return KFAMD_EINVAL;  // relu's backward needs only the output's sign
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(((M + BM - 1) / BM) * ((N + BM - 1) / BM), batch), block(kThreads);
  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
  __bf16* c = static_cast<__bf16*>(C);
  const __bf16* bs = static_cast<const __bf16*>(bias);
  const __bf16* r = static_cast<const __bf16*>(R);
  __bf16* x = static_cast<__bf16*>(Aux);
  const bool hb = bias != nullptr, hr = R != nullptr, hx = Aux != nullptr;
#define W4_LAUNCH(HB, HR, HX)                                                                                     \
  hipLaunchKernelGGL((gemm_w4<ACT, HB, HR, HX, 0, 0, BM>), grid, block, 0, s, a, b, c, bs, r, x, M, N, K, lda, ldb, \
                     ldc, ldr, sa, sb, sc, sr, alpha, nullptr)
  if constexpr (ACT == KFAMD_ACT_NONE) {
    if (hb && hr) W4_LAUNCH(true, true, false);
    else if (hb) W4_LAUNCH(true, false, false);
    else if (hr) W4_LAUNCH(false, true, false);
    else W4_LAUNCH(false, false, false);
  } else if constexpr (ACT == KFAMD_ACT_RELU) {
    if (hb) W4_LAUNCH(true, false, false);
    else W4_LAUNCH(false, false, false);
  } else {
    if (hx) {
      if (hb) W4_LAUNCH(true, false, true);
      else W4_LAUNCH(false, false, true);
    } else {
      if (hb) W4_LAUNCH(true, false, false);
      else W4_LAUNCH(false, false, false);
    }
  }
#undef W4_LAUNCH
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

}  // namespace
}  // namespace kfw4

// the per-activation entry points (tu/w4_nt_<act>.hip); bm = 256 ("w4") or 128 ("w4s")
#define KFW4_NT_ENTRY(NAME, ACT)                                                                                     \
  extern "C" int NAME(int bm, const void* A, const void* B, void* C, const void* bias, const void* R, void* Aux,       \
                      int M, int N, int K, int batch, long long lda, long long ldb, long long ldc, long long ldr,      \
                      long long sa, long long sb, long long sc, long long sr, float alpha, void* stream) {             \
    if (bm == 256)                                                                                                   \
      return kfw4::launch_nt_act<256, ACT>(A, B, C, bias, R, Aux, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, \
                                           alpha, stream);                                                           \
    if (bm == 128)                                                                                                   \
      return kfw4::launch_nt_act<128, ACT>(A, B, C, bias, R, Aux, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, \
                                           alpha, stream);                                                           \
    return KFAMD_EINVAL;                                                                                             \
  }
