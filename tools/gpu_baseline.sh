#!/bin/bash
# BASELINE.md §3 numbers on one MI355X: cold start (20 runs, phase breakdown), GEMM / LayerNorm
# sweeps, headline bench, rocprofv3 kernel stats of the bench. Each GPU step time-limited.
set -o pipefail
O=gpurun_out/baseline
mkdir -p $O
export TMPDIR=/tmp
echo "== coldstart" && timeout -k 10 300 python -m kubeflow_rm_amd.bench_coldstart --runs 20 > $O/coldstart.json 2> $O/coldstart.err || exit $?
head -c 600 $O/coldstart.json; echo
echo "== kbench" && timeout -k 10 500 python tools/kbench.py --rounds 3 --out $O/kbench.jsonl > $O/kbench.log 2>&1 || exit $?
cat $O/kbench.jsonl
echo "== bench" && timeout -k 10 300 python bench.py --steps 50 --warmup 10 --compare-torch > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log
echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --coldstart-runs 0 > $O/prof.log 2>&1 || exit $?
find $O/prof -name '*kernel_stats.csv' -exec head -5 {} \;
