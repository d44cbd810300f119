# round-4 end-state check on one MI355X: every GPU test, smoke, the driver's bench (defaults), then the
# epilogue store-layout ablation (diag build); each step bounded, the chain stops at the first failure
out=gpurun_out/r4_final
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 560 python -u bench.py > $out/bench.log 2>&1 &&
timeout -k 10 300 python -u tools/w4_ab.py --variants r4,epi_fullline --rounds 3 --sizes 8192 --diag 8192,4096 > $out/epi_ab.jsonl 2> $out/epi_ab.err
