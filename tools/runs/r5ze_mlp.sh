#!/bin/bash
# MLP backward with fc2's dgrad fused with fc1's gelu backward (gemm_w4.h DACT): numerics, then the
# gpt-1b step with the fused form vs the two-step form (KFAMD_FUSED_DGRAD_ACT=0), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5ze_mlp
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dgrad_act or mlp or linear or layernorm" tests/test_gpu_models.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 2 --out $OUT/train_fused.jsonl > $OUT/train_fused_$r.log 2>&1 || exit $?
  KFAMD_FUSED_DGRAD_ACT=0 timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 2 --backends native --out $OUT/train_split.jsonl > $OUT/train_split_$r.log 2>&1 || exit $?
done
cut -c1-330 $OUT/train_fused.jsonl $OUT/train_split.jsonl
