#!/bin/bash
# r3: split-K cost-model plan — numerics, wgrad-shape A/B vs the unsplit kernel and torch, GPT train steps.
set -o pipefail
O=gpurun_out/r3s2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread \
  -k "splitk or linear or gpt or mm_" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/wgrad_ab.py 2304x768x32768,768x768x32768,3072x768x32768,768x3072x32768,6144x2048x8192,2048x2048x8192,1024x1024x4096,512x768x8192 \
  > $O/wgrad.jsonl 2>$O/wgrad.err || { tail $O/wgrad.err; exit 1; }
cat $O/wgrad.jsonl
for cfg in "gpt-small 16 2048" "gpt-1b 4 2048"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/train_bench.py --model $1 --batch $2 --seq $3 --steps 10 --rounds 3 \
    --out $O/train.jsonl >> $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
done
cat $O/train.jsonl
