#!/bin/bash
# kernel-level split of the production attention backward (dK/dV kernel, dQ kernel, delta) at the
# gpt-1b and gpt-small shapes, rocprofv3 kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5s_attn_prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o attn -- python3 $R/tools/attn_bench.py --shapes 4x16x2048x128,16x12x2048x64 --rounds 2 > $OUT/prof.log 2>&1 || exit $?
grep -i "attn" $OUT/prof/attn_kernel_stats.csv | cut -d, -f1-4 | sed 's/(bool _Accum[^"]*//'
