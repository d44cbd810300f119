// tu/w4_sk_none_01.hip — stream-K kernel: none epilogue, bias false, residual true (gemm_w4_sk.h).
#include "gemm_w4_sk.h"

KFW4_SK_ENTRY(kfw4_sk_none_01, KFAMD_ACT_NONE, false, true)
