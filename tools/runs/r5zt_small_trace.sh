#!/bin/bash
# gpt-small step (16 x 2048 tokens) kernel trace on the native kernels, grouped by role
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zt_small_trace
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/native -o run -- python3 $R/tools/prof_train.py native gpt-small 16 2048 > $OUT/native.log 2>&1 || exit $?
f=$(ls $OUT/native/*kernel_stats.csv $OUT/native/*/*kernel_stats.csv 2>/dev/null | head -1)
python3 $R/tools/train_kernel_summary.py $f > $OUT/summary_native.json || exit 1
cat $OUT/summary_native.json
