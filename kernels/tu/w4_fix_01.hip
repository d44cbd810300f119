// tu/w4_fix_01.hip — split-K with the in-kernel fixup, operand layouts LA = 0, LB = 1 (gemm_w4_fix.h).
#include "gemm_w4_fix.h"

KFW4_FIX_ENTRY(kfw4_fix_01, 0, 1)
