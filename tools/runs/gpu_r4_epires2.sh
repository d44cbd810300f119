# round 4: bias preloaded per epilogue + the measured split-K fixup plan: numerics, the fused-epilogue
# A/B, the fixup A/B on the wgrad shapes, then the gpt-1b training step; stop at the first failure
out=gpurun_out/r4_epires2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/epi_ab.py 8192x2048x2048,8192x2048x8192,8192x6144x2048,8192x8192x2048 > $out/ab.jsonl 2> $out/ab.err &&
timeout -k 10 400 python -u tools/fixk_ab.py 2048x2048x8192,4096x2048x8192,3072x768x32768,768x3072x32768,2304x768x32768 --splits 2,4,6,7 > $out/fixk.jsonl 2> $out/fixk.err &&
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out $out/train.jsonl > $out/train.log 2>&1
