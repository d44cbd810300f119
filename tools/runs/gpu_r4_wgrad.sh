# round 4: GEMM numerics (split-K full-line partials), the wgrad-shaped A/B vs torch (gpt-1b / gpt-small
# weight gradients), then the gpt-1b training step; each step bounded, stop at the first failure
out=gpurun_out/r4_wgrad
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/wgrad_ab.py 6144x2048x8192,2048x2048x8192,8192x2048x8192,2048x8192x8192,32000x2048x8192,2304x768x32768,768x768x32768,3072x768x32768,768x3072x32768 > $out/ab.jsonl 2> $out/ab.err &&
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out $out/train.jsonl > $out/train.log 2>&1
