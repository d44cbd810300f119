#!/bin/bash
# LayerNorm forward A/B in one process tree on one box: the DPP reduction vs the ds_bpermute
# butterfly (KFAMD_LN_BP=1), the streaming kernel (KFAMD_LN_STREAM=<max VPL>), gamma/beta prefetch
# for VPL 16 (KFAMD_LN_PF=16); numerics of every variant first
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5j_ln_ab
mkdir -p $OUT
cd $R
for env in "KFAMD_LN_STREAM=8" "KFAMD_LN_BP=1" "KFAMD_LN_PF=16"; do
  env $env timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layernorm_residual.py tests/test_gpu_kernels.py -k "norm or layer" > $OUT/pytest_${env%%=*}.log 2>&1
  rc=$?; echo "$env pytest rc=$rc $(tail -1 $OUT/pytest_${env%%=*}.log)"; [ $rc -eq 0 ] || exit $rc
done
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u tools/kbench.py --sizes "" --ln 8192x4096,8192x8192,32768x8192,8192x2048,16384x4096 --rounds 5 --no-torch --out $OUT/kbench_$tag.jsonl > $OUT/kbench_$tag.log 2>&1 || return $?
  echo "== $tag"; grep layernorm_fwd $OUT/kbench_$tag.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['rows'], d['hidden'], d['ours_us'], d['ours_GBps'], d['copy_GBps'], d['ours_of_copy_roof'])"
}
run base KFAMD_LN_X=0 && run bp KFAMD_LN_BP=1 && run st8 KFAMD_LN_STREAM=8 && run pf16 KFAMD_LN_PF=16 \
  && run st8pf16 KFAMD_LN_STREAM=8 KFAMD_LN_PF=16 && run base2 KFAMD_LN_X=0 && run st8b KFAMD_LN_STREAM=8
