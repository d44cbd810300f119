#!/bin/bash
# act-grad GEMM epilogue: R prefetch distance 2 (production) / 3 / 4 (tuab builds), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zi_pd
mkdir -p $OUT
cd $R
for r in 1 2; do
  for v in prod pd3 pd4; do
    lib=$R/kubeflow_rm_amd/lib/libkfamd_kernels.so; [ $v = prod ] || lib=$R/kubeflow_rm_amd/lib/tuab/libkfamd_kernels_$v.so
    KFAMD_KERNEL_LIB=$lib timeout -k 10 200 python3 -u tools/dact_bench.py --res "" > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    echo "== $v $r"; cat $OUT/bench_${v}_$r.jsonl
  done
done
