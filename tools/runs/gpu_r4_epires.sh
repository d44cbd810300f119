# round 4: full-line residual epilogue: numerics of every residual path, then the fused-epilogue A/B on
# the gpt-1b projections; stop at the first failure
out=gpurun_out/r4_epires
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "residual or epilogue or mm_operand or fixk or splitk or linear or streamk" > $out/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/epi_ab.py 8192x2048x2048,8192x2048x8192,8192x6144x2048,8192x8192x2048,8192x8192x8192 > $out/ab.jsonl 2> $out/ab.err &&
timeout -k 10 300 python -u tools/fix_ab.py 2048x2048x8192,4096x2048x8192 --splits 2,3,4 > $out/fixab.jsonl 2> $out/fixab.err
