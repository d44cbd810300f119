#!/bin/bash
# LayerNorm backward: the one-pass fused kernel (dx + residual + dgamma/dbeta partials) vs the split
# path (KFAMD_LN_BWD_SPLIT=1: dx kernel, then the partial-sum kernel re-reading dy and x); numerics
# first, then kbench alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zc_ln_bwd
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm or norm_forward or rmsnorm" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
SH=8192x2048,16384x2048,8192x768,32768x768,8192x1024
for r in 1 2; do
  timeout -k 10 200 python -u tools/kbench.py --sizes "" --ln $SH --rounds 5 --out $OUT/fused_$r.jsonl > $OUT/fused_$r.log 2>&1 || exit $?
  KFAMD_LN_BWD_SPLIT=1 timeout -k 10 200 python -u tools/kbench.py --sizes "" --ln $SH --rounds 5 --out $OUT/split_$r.jsonl > $OUT/split_$r.log 2>&1 || exit $?
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r5zc_ln_bwd/*.jsonl")):
    for l in open(f):
        d=json.loads(l)
        if d["kind"]=="layernorm_bwd_bf16":
            print(f.split("/")[-1], d["rows"], d["hidden"], "dx", d["dx_us"], "full", d["full_us"], "full_res", d["full_res_us"], "torch", d["torch_full_us"])
PY
