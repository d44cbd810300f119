// tu/w4_nt_gelu.hip — the w4 forward GEMM kernels with the gelu epilogue (gemm_w4_nt.h);
// one translation unit per activation so the library builds them in parallel.
#include "gemm_w4_nt.h"

KFW4_NT_ENTRY(kfw4_nt_gelu, KFAMD_ACT_GELU_TANH)
