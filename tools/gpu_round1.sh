#!/bin/bash
# First GPU validation: numerics tests, kernel sweep, headline bench, rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench" && timeout -k 10 400 python tools/kbench.py --out gpurun_out/kbench.jsonl > gpurun_out/kbench.log 2>&1 || exit $?
cat gpurun_out/kbench.jsonl
echo "== bench" && timeout -k 10 300 python bench.py --steps 50 --warmup 10 --compare-torch > gpurun_out/bench.log 2>&1 || exit $?
cat gpurun_out/bench.log
echo "== rocprof" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof.log 2>&1 || exit $?
find gpurun_out/prof -name '*stats*' | head
