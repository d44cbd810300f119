#!/bin/bash
# one-pass LayerNorm backward with the next row prefetched (KFLN_FUSED_PF=1, production) vs without
# (tuab lnpf0): LayerNorm numerics of both, then kbench alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zs_lnpf
mkdir -p $OUT
cd $R
for v in prod lnpf0; do
  lib=$R/kubeflow_rm_amd/lib/libkfamd_kernels.so; [ $v = prod ] || lib=$R/kubeflow_rm_amd/lib/tuab/libkfamd_kernels_$v.so
  KFAMD_KERNEL_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm or norm_forward or rmsnorm" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
SH=8192x2048,16384x2048,8192x768,32768x768,8192x1024
for r in 1 2; do
  for v in prod lnpf0; do
    lib=$R/kubeflow_rm_amd/lib/libkfamd_kernels.so; [ $v = prod ] || lib=$R/kubeflow_rm_amd/lib/tuab/libkfamd_kernels_$v.so
    KFAMD_KERNEL_LIB=$lib timeout -k 10 200 python -u tools/kbench.py --sizes "" --ln $SH --rounds 5 --out $OUT/${v}_$r.jsonl > $OUT/${v}_$r.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r5zs_lnpf/*.jsonl")):
    for l in open(f):
        d=json.loads(l)
        if d["kind"]=="layernorm_bwd_bf16":
            print(f.split("/")[-1], d["rows"], d["hidden"], "full", d["full_us"], "full_res", d["full_res_us"])
PY
