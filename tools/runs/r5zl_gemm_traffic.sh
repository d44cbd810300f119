#!/bin/bash
# HBM / L2 traffic of the 8192^3 GEMM, ours vs hipBLASLt (energy per MFMA on a power-limited part):
# FETCH_SIZE, WRITE_SIZE, L2 hit / miss, each pass in its own bounded run; kernel trace for times
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zl_gemm_traffic
mkdir -p $OUT
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 10 --variants w4 > $OUT/trace.log 2>&1 || exit $?
echo "== pmc 1" && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc1 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 --variants w4 > $OUT/pmc1.log 2>&1 || exit $?
echo "== pmc 2" && timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc2 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 --variants w4 > $OUT/pmc2.log 2>&1 || exit $?
echo "== pmc 3" && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc3 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 --variants w4 > $OUT/pmc3.log 2>&1 || exit $?
python3 $R/tools/prof_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
