#!/bin/bash
# staggered 8-wave forward (attn_fwd_pp) A/B: numerics of each variant, then causal rounds and one
# non-causal round of tools/attn_bench.py, the variants back to back on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6d_attn_pp}
mkdir -p $OUT
cd $R
VARS=${VARS:-prod fwdold nostagger nofence}
SHAPES=${SHAPES:-4x16x2048x128,16x12x2048x64,1x16x4096x128}
lib() { echo $R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$1.so; }
for v in $VARS; do
  KFAMD_KERNEL_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
show() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['shape'], d['causal'], d['pass'], d['ours_us'], d['sdpa_us'], d['ours_tflops'])"; }
for r in 1 2; do
  for v in $VARS; do
    KFAMD_KERNEL_LIB=$(lib $v) timeout -k 10 200 python -u tools/attn_bench.py --shapes $SHAPES > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    echo "== $v round $r"; show $OUT/bench_${v}_$r.jsonl
  done
done
for v in $VARS; do
  KFAMD_KERNEL_LIB=$(lib $v) timeout -k 10 200 python -u tools/attn_bench.py --no-causal --shapes $SHAPES > $OUT/nc_${v}.jsonl 2> $OUT/nc_${v}.err || exit $?
  echo "== $v non-causal"; show $OUT/nc_${v}.jsonl
done
