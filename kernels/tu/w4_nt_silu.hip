// tu/w4_nt_silu.hip — the w4 forward GEMM kernels with the silu epilogue (gemm_w4_nt.h);
// one translation unit per activation so the library builds them in parallel.
#include "gemm_w4_nt.h"

KFW4_NT_ENTRY(kfw4_nt_silu, KFAMD_ACT_SILU)
