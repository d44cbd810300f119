#!/bin/bash
# r3: model-level tests, then GPT training steps on the framework kernels vs torch ops.
set -o pipefail
O=gpurun_out/r3t; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "${KSEL:-gpt or residual or linear}" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-"gpt-small 8 1024" "gpt-small 16 2048" "gpt-1b 4 2048"}; do
  set -- $cfg
  timeout -k 10 300 python -u tools/train_bench.py --model $1 --batch $2 --seq $3 --steps ${STEPS:-10} --rounds 3 \
    --out $O/train.jsonl >> $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
done
cat $O/train.jsonl
