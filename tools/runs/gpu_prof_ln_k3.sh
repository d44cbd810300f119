#!/bin/bash
# rocprofv3 on K2 (LayerNorm) and K3 (one-shot all-reduce): kernel stats + HBM bytes + LDS conflicts.
# Counters in their own passes (no sys-trace), each pass time-limited.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_ln_k3; mkdir -p $OUT
D="python3 $R/tools/prof_ln_k3_driver.py"
echo "== trace" && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $D 10 > $OUT/trace.log 2>&1 || exit $?
echo "== pmc fetch" && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- $D 3 > $OUT/pmc1.log 2>&1 || exit $?
echo "== pmc write" && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $OUT/pmc2 -o run -- $D 3 > $OUT/pmc2.log 2>&1 || exit $?
echo "== pmc clocks" && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc3 -o run -- $D 3 > $OUT/pmc3.log 2>&1 || exit $?
echo ok
