#!/bin/bash
# PMC profile of the GEMM variants vs hipBLASLt at 8192^3: effective clock (GRBM_GUI_ACTIVE / 8 /
# dispatch time), MFMA busy, LDS bank conflicts, L2 hit/miss, HBM fetch. Counters in their own
# runs (no sys-trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_gemm
V=${PROF_VARIANTS:-pipe_sched,w4}
mkdir -p $OUT
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 20 --variants $V > $OUT/trace.log 2>&1 || exit $?
echo "== pmc 1" && timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 --variants $V > $OUT/pmc1.log 2>&1 || exit $?
echo "== pmc 2" && timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc2 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 --variants $V > $OUT/pmc2.log 2>&1 || exit $?
echo "== pmc 3" && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 --variants $V > $OUT/pmc3.log 2>&1 || exit $?
echo "== pmc 4" && timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc4 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 --variants $V > $OUT/pmc4.log 2>&1 || exit $?
echo ok
