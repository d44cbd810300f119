# round 4: split-K fixup (gemm_w4.h SPLIT == 2): numerics, then the wgrad-shaped A/B; stop at the first failure
out=gpurun_out/r4_fixk
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "fixk or splitk or mm_operand or streamk" > $out/pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/fixk_ab.py 2048x2048x8192,6144x2048x8192,4096x2048x8192,3072x768x32768,2304x768x32768,768x3072x32768,4096x4096x8192 > $out/ab.jsonl 2> $out/ab.err
