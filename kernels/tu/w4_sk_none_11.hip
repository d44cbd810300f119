// tu/w4_sk_none_11.hip — stream-K kernel: none epilogue, bias true, residual true (gemm_w4_sk.h).
#include "gemm_w4_sk.h"

KFW4_SK_ENTRY(kfw4_sk_none_11, KFAMD_ACT_NONE, true, true)
