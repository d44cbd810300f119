# round 4: bias / LayerNorm parameter grads written as bf16 by their finalize kernels: the whole GPU suite,
# then the gpt-1b / gpt-small training steps; stop at the first failure
out=gpurun_out/r4_gradbf16
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out $out/train.jsonl > $out/train.log 2>&1 &&
timeout -k 10 300 python -u tools/train_bench.py --model gpt-small --batch 16 --seq 2048 --steps 10 --rounds 3 --out $out/train.jsonl >> $out/train.log 2>&1
