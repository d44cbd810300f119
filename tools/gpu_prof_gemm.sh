#!/bin/bash
# PMC profile of the GEMM variants vs hipBLASLt at 8192^3: busy cycles (-> effective clock with the
# kernel-trace durations), MFMA busy, LDS bank conflicts. Counters in their own runs (no sys-trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_gemm
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o -E "^\s*(GRBM_GUI_ACTIVE|SQ_BUSY_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES|SQ_LDS_BANK_CONFLICT|SQ_INSTS_MFMA|SQ_WAVE_CYCLES|SQ_BUSY_CU_CYCLES)\b" $OUT/avail.txt | sort -u > $OUT/found.txt || true
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 20 > $OUT/trace.log 2>&1 || exit $?
echo "== pmc 1" && timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 > $OUT/pmc1.log 2>&1 || exit $?
echo "== pmc 2" && timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc2 -o run -- python3 $R/tools/prof_gemm_driver.py --size 8192 --iters 5 > $OUT/pmc2.log 2>&1 || exit $?
ls -R $OUT | head -40
