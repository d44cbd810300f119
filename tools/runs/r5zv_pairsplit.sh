#!/bin/bash
# weight-gradient pairs with split-K (gpt-small: MLP 36 + 36 tiles, attention 27 + 9): numerics, then
# the gpt-small and gpt-1b steps with the pairs on (default) and off (KFAMD_WGRAD_PAIR=0), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zv_pairsplit
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_models.py -k "wgrad_pair or attn_block or mlp or gpt" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_bench.py --model gpt-small --batch 16 --seq 2048 --steps 10 --rounds 2 --backends native --out $OUT/small_on.jsonl > $OUT/small_on_$r.log 2>&1 || exit $?
  KFAMD_WGRAD_PAIR=0 timeout -k 10 300 python -u tools/train_bench.py --model gpt-small --batch 16 --seq 2048 --steps 10 --rounds 2 --backends native --out $OUT/small_off.jsonl > $OUT/small_off_$r.log 2>&1 || exit $?
done
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 2 --out $OUT/big.jsonl > $OUT/big.log 2>&1 || exit $?
cut -c1-300 $OUT/small_on.jsonl $OUT/small_off.jsonl $OUT/big.jsonl
