#!/bin/bash
# act-grad GEMM on the 128 tile (two workgroups per CU: one's epilogue under the other's K loop) vs
# the 256 tile (production): numerics of both, then tools/dact_bench.py alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zq_dact128
mkdir -p $OUT
cd $R
for v in prod dact128; do
  lib=$R/kubeflow_rm_amd/lib/libkfamd_kernels.so; [ $v = prod ] || lib=$R/kubeflow_rm_amd/lib/tuab/libkfamd_kernels_$v.so
  KFAMD_KERNEL_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dgrad_act or mlp" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in prod dact128; do
    lib=$R/kubeflow_rm_amd/lib/libkfamd_kernels.so; [ $v = prod ] || lib=$R/kubeflow_rm_amd/lib/tuab/libkfamd_kernels_$v.so
    KFAMD_KERNEL_LIB=$lib timeout -k 10 200 python3 -u tools/dact_bench.py --res "" --preact "" > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    echo "== $v $r"; cat $OUT/bench_${v}_$r.jsonl
  done
done
