# round-4 GEMM validation on one MI355X: GEMM numerics tests (unrolled K loop), the A/B against the
# round-3 loop (libw4ab_base.so) and torch, then the bench; each step bounded, stop at the first failure
out=gpurun_out/r4_gemm
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread > $out/pytest_kernels.log 2>&1 &&
timeout -k 10 300 python -u tools/w4_ab.py --variants base,f2u5,asmdma --rounds 7 --sizes 4096,8192,16384 --diag 8192 > $out/ab.jsonl 2> $out/ab.err &&
timeout -k 10 400 python -u bench.py --budget-s 240 > $out/bench.log 2>&1 &&
timeout -k 10 500 bash tools/gpu_prof_stalls.sh > $out/prof_stalls.log 2>&1
