#!/bin/bash
# attention backward: what the dQ atomics cost (dma_noatomic drops them at the address unit: timing only)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5p_attn_abl
mkdir -p $OUT
cd $R
for r in 1 2; do
  for v in dma dma_noatomic; do
    KFAMD_KERNEL_LIB=$R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$v.so timeout -k 10 200 python -u tools/attn_bench.py --shapes 4x16x2048x128,1x16x4096x128 > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    echo "== $v round $r"; python3 -c "
import json
for l in open('$OUT/bench_${v}_$r.jsonl'):
    d=json.loads(l); print(d['shape'], d['pass'], d['ours_us'], d['sdpa_us'])"
  done
done
