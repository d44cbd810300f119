// tu/w4_sk_none_10.hip — stream-K kernel: none epilogue, bias true, residual false (gemm_w4_sk.h).
#include "gemm_w4_sk.h"

KFW4_SK_ENTRY(kfw4_sk_none_10, KFAMD_ACT_NONE, true, false)
