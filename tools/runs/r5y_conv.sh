#!/bin/bash
# convergence parity: the GPT training test (native vs torch reference from the same init) and the
# gpt-1b step bench with comparable losses
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5y_conv
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_models.py > $OUT/pytest.log 2>&1
rc=$?; tail -30 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 2 --out $OUT/train.jsonl > $OUT/train.log 2>&1
rc=$?; cat $OUT/train.jsonl; exit $rc
