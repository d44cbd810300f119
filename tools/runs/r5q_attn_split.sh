#!/bin/bash
# attention backward variants: prod (register-staged Q/dO, dQ atomics), dma (LDS-DMA staging),
# dma_noatomic (timing only: atomics dropped), dqsplit (atomic-free dQ kernel); numerics first
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5q_attn_split
mkdir -p $OUT
cd $R
for v in prod dma dqsplit; do
  KFAMD_KERNEL_LIB=$R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in prod dma dma_noatomic dqsplit; do
    KFAMD_KERNEL_LIB=$R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$v.so timeout -k 10 200 python -u tools/attn_bench.py > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    echo "== $v round $r"; python3 -c "
import json
for l in open('$OUT/bench_${v}_$r.jsonl'):
    d=json.loads(l); print(d['shape'], d['pass'], d['ours_us'], d['sdpa_us'])"
  done
done
for v in prod dqsplit; do
  KFAMD_KERNEL_LIB=$R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$v.so timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out $OUT/train_$v.jsonl > $OUT/train_$v.log 2>&1 || exit $?
  echo "== train $v"; cut -c1-300 $OUT/train_$v.jsonl
done
