#!/bin/bash
# forward gelu epilogue with packed-f32 polynomial parts (KFW4_ACT_PK=1, production) vs scalar
# (tuab pk0): numerics of both, then the preact GEMM, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zk_actpk
mkdir -p $OUT
cd $R
for v in prod pk0; do
  lib=$R/kubeflow_rm_amd/lib/libkfamd_kernels.so; [ $v = prod ] || lib=$R/kubeflow_rm_amd/lib/tuab/libkfamd_kernels_$v.so
  KFAMD_KERNEL_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or linear or mlp or preact" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in prod pk0; do
    lib=$R/kubeflow_rm_amd/lib/libkfamd_kernels.so; [ $v = prod ] || lib=$R/kubeflow_rm_amd/lib/tuab/libkfamd_kernels_$v.so
    KFAMD_KERNEL_LIB=$lib timeout -k 10 200 python3 -u tools/dact_bench.py --shapes "" --res "" > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    echo "== $v $r"; cat $OUT/bench_${v}_$r.jsonl
  done
done
