# round 4: GEMM / model numerics on the full-line epilogue (incl. the pre-activation output), then the
# GPT training steps; each step bounded, stop at the first failure
out=gpurun_out/r4_train2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
for cfg in "gpt-small 16 2048" "gpt-1b 4 2048"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/train_bench.py --model $1 --batch $2 --seq $3 --steps 10 --rounds 3 \
    --out $out/train.jsonl >> $out/train.log 2>&1 || exit 1
done
