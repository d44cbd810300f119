// tu/w4_sk_relu_10.hip — stream-K kernel: relu epilogue, bias true, residual false (gemm_w4_sk.h).
#include "gemm_w4_sk.h"

KFW4_SK_ENTRY(kfw4_sk_relu_10, KFAMD_ACT_RELU, true, false)
