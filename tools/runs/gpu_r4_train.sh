# round 4 on one MI355X: the zygote cold start (10 runs, per-run times) after gc.freeze, then GPT
# training steps on the framework kernels (round-4 GEMM loop) vs torch ops; each step bounded
out=gpurun_out/r4_train
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 180 python -u -m kubeflow_rm_amd.bench_coldstart --runs 10 --server torch-ready --zygote --timeout 30 > $out/zygote.json 2> $out/zygote.err &&
for cfg in "gpt-small 16 2048" "gpt-1b 4 2048"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/train_bench.py --model $1 --batch $2 --seq $3 --steps 10 --rounds 3 \
    --out $out/train.jsonl >> $out/train.log 2>&1 || exit 1
done
