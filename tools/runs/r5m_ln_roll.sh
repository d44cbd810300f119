#!/bin/bash
# hidden 8192: rolling-prefetch streaming kernel (KFAMD_LN_ROLL=1) vs the gamma/beta-prefetch one-shot kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5m_ln_roll
mkdir -p $OUT
cd $R
KFAMD_LN_ROLL=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "norm" > $OUT/pytest_roll.log 2>&1
rc=$?; echo "roll pytest rc=$rc $(tail -1 $OUT/pytest_roll.log)"; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u tools/kbench.py --sizes "" --ln 8192x8192,16384x8192,32768x8192,4096x8192 --rounds 5 --no-torch --out $OUT/kbench_$tag.jsonl > $OUT/kbench_$tag.log 2>&1 || return $?
  echo "== $tag"; grep layernorm_fwd $OUT/kbench_$tag.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['rows'], d['hidden'], d['ours_us'], d['ours_GBps'], d['copy_GBps'])"
}
run base KFAMD_LN_X=0 && run roll KFAMD_LN_ROLL=1 && run base2 KFAMD_LN_X=0 && run roll2 KFAMD_LN_ROLL=1
