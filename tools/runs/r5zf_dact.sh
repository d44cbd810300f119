#!/bin/bash
# the act-grad GEMM epilogue alone: fused vs GEMM + act_grad pass, then a kernel trace of the same
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zf_dact
mkdir -p $OUT
timeout -k 10 200 python3 -u $R/tools/dact_bench.py > $OUT/bench.jsonl 2> $OUT/bench.err || exit $?
cat $OUT/bench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/tools/dact_bench.py --rounds 2 --iters 5 > $OUT/prof.log 2>&1 || exit $?
f=$(ls $OUT/prof/*kernel_stats.csv $OUT/prof/*/*kernel_stats.csv 2>/dev/null | head -1)
python3 -c "
import csv,sys
for r in sorted(csv.DictReader(open('$f')), key=lambda r:-float(r['TotalDurationNs']))[:8]:
    print(round(float(r['AverageNs'])/1e3,1), r['Calls'], r['Name'][:120])"
