# round-4 validation on one MI355X: GPU tests, smoke, then the driver's bench (N=1, defaults) with the
# budgeted cold-start extras; each step bounded, the chain stops at the first failure
out=gpurun_out/r4_validate
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 560 python -u bench.py > $out/bench.log 2>&1
