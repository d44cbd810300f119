// tu/w4_sk_silu_00.hip — stream-K kernel: silu epilogue, bias false, residual false (gemm_w4_sk.h).
#include "gemm_w4_sk.h"

KFW4_SK_ENTRY(kfw4_sk_silu_00, KFAMD_ACT_SILU, false, false)
