#!/bin/bash
# attn_bwd_dkdv8 timing ablations (wrong results by design: no numerics): the backward at gpt-1b, 2 rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6j_bwd_abl}
mkdir -p $OUT
cd $R
VARS=${VARS:-prod babl1 babl2 babl4 babl7}
for r in 1 2; do
  for v in $VARS; do
    KFAMD_KERNEL_LIB=$R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$v.so timeout -k 10 200 python -u tools/attn_bench.py --shapes ${SHAPES:-4x16x2048x128} $ATTN_ARGS > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    python3 -c "
import json
for l in open('$OUT/bench_${v}_$r.jsonl'):
    d=json.loads(l)
    if d['pass']=='bwd': print('$v', '$r', d['shape'], d['causal'], d['ours_us'], d['ours_tflops'])"
  done
done
