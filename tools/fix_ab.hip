// tools/fix_ab.hip — the split-K fixup kernel (gemm_w4.h SPLIT == 2) built once per ablation
// (KFW4_FIX_AB, see tools/fix_ab.py); the entry has kfw4_fix_*'s signature.
#include "gemm_w4_fix.h"

KFW4_FIX_ENTRY(fixab_11, 1, 1)
