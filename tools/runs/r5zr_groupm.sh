#!/bin/bash
# grouped raster height (KFW4_GROUP_M 4 = production vs 2 / 8) on the gpt-1b forward GEMMs
# (bias + residual, bias + gelu + pre-activation), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zr_groupm
mkdir -p $OUT
cd $R
for r in 1 2; do
  for v in prod gm2 gm8; do
    lib=$R/kubeflow_rm_amd/lib/libkfamd_kernels.so; [ $v = prod ] || lib=$R/kubeflow_rm_amd/lib/tuab/libkfamd_kernels_$v.so
    KFAMD_KERNEL_LIB=$lib timeout -k 10 200 python3 -u tools/dact_bench.py --shapes "" --res 8192x2048x2048,8192x2048x8192,8192x6144x2048 > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    echo "== $v $r"; cat $OUT/bench_${v}_$r.jsonl
  done
done
