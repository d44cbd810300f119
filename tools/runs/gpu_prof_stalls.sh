#!/bin/bash
# Where the GEMM's wave cycles go, ours vs hipBLASLt at 8192^3: SQ wave-cycle buckets (issue stalls,
# waitcnt/barrier waits, active instructions) in one PMC pass; kernel trace for dispatch times.
# Counters in their own run (no sys-trace); summary: tools/prof_summary.py <out dir>.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-prof_stalls}
mkdir -p $OUT
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 10 --variants w4 > $OUT/trace.log 2>&1 || exit $?
echo "== pmc 1" && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 --variants w4 > $OUT/pmc1.log 2>&1 || exit $?
echo "== pmc 2" && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --output-format csv -d $OUT/pmc2 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 --variants w4 > $OUT/pmc2.log 2>&1 || exit $?
python3 $R/tools/prof_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
