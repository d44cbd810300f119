#!/bin/bash
# Round-2 final evidence: kernel trace of the headline bench (bench.py, GEMM only) and of K2/K3, plus
# one PMC pass over K2/K3 for waves in flight. Counters in their own runs (no sys-trace), each pass
# time-limited.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_r2; mkdir -p $OUT
echo "== bench trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o run -- python3 $R/bench.py --steps 20 --warmup 5 --coldstart-runs 0 > $OUT/bench.log 2>&1 || exit $?
D="python3 $R/tools/prof_ln_k3_driver.py"
echo "== ln/k3 trace" && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lnk3 -o run -- $D 10 > $OUT/lnk3.log 2>&1 || exit $?
echo "== ln/k3 pmc waves" && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_waves -o run -- $D 3 > $OUT/pmc_waves.log 2>&1 || exit $?
echo ok
