# round-4 GEMM validation on one MI355X: every GPU test (the K loop is shared by all GEMM paths), smoke,
# the A/B against the round-3 loop (libw4ab_base.so) and torch, the bench, then the PMC stall pass;
# each step bounded, the chain stops at the first failure
out=gpurun_out/r4_gemm
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 300 python -u tools/w4_ab.py --variants base --rounds 7 --sizes 4096,8192,16384 --diag 8192 > $out/ab.jsonl 2> $out/ab.err &&
timeout -k 10 400 python -u bench.py --budget-s 240 > $out/bench.log 2>&1 &&
timeout -k 10 500 bash tools/runs/gpu_prof_stalls.sh > $out/prof_stalls.log 2>&1
