// tu/w4_fix_00.hip — split-K with the in-kernel fixup, operand layouts LA = 0, LB = 0 (gemm_w4_fix.h).
#include "gemm_w4_fix.h"

KFW4_FIX_ENTRY(kfw4_fix_00, 0, 0)
