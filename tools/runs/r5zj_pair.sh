#!/bin/bash
# QKV + output-projection weight gradients in one launch (ops.attn_block / gemm_w4.h GRP): numerics,
# then the gpt-1b step (train_bench) and a kernel trace of it
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zj_pair
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad_pair or attn_block or dgrad_act or mlp" tests/test_gpu_models.py tests/test_gpu_attention.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out $OUT/train.jsonl > $OUT/train.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/train_bench.py --model gpt-small --batch 16 --seq 2048 --steps 10 --rounds 3 --out $OUT/train.jsonl >> $OUT/train.log 2>&1 || exit $?
cut -c1-330 $OUT/train.jsonl
export PROF_OUT=r5zj_pair/prof
bash $R/tools/runs/gpu_r4_proftrain.sh || exit $?
cat $OUT/prof/summary_native.json
