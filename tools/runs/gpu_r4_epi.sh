# round 4: full-line epilogue stores: GEMM numerics tests, A/B + stamps against the half-line epilogue, bench
out=gpurun_out/r4_epi2
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/w4_ab.py --variants r4,noful,base --rounds 7 --sizes 4096,8192,16384 --diag 8192,4096 > $out/ab.jsonl 2> $out/ab.err &&
timeout -k 10 300 python -u bench.py --budget-s 60 --coldstart-runs 0 > $out/bench.log 2>&1
