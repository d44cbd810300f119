#!/bin/bash
# attention build A/B (tools/attn_ab.py variants): numerics of every variant first, then alternating
# bench rounds. TAG names the output directory, VARS the variants, SHAPES / ATTN_ARGS go to attn_bench
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-attn_ab}
mkdir -p $OUT
cd $R
VARS=${VARS:-prod head}
SHAPES=${SHAPES:-4x16x2048x128,16x12x2048x64,1x16x4096x128}
for v in $VARS; do
  KFAMD_KERNEL_LIB=$R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in $VARS; do
    KFAMD_KERNEL_LIB=$R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$v.so timeout -k 10 200 python -u tools/attn_bench.py --shapes $SHAPES $ATTN_ARGS > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    echo "== $v round $r"; python3 -c "
import json
for l in open('$OUT/bench_${v}_$r.jsonl'):
    d=json.loads(l); print(d['shape'], d['causal'], d['pass'], d['ours_us'], d['sdpa_us'], d['ours_tflops'])"
  done
done
