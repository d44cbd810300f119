#!/bin/bash
# GPU validation: pytest -m gpu, smoke(), headline bench. Each GPU step time-limited; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out/check
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/check/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/check/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check/smoke.log 2>&1; rc=$?
tail -5 gpurun_out/check/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/check/bench.log 2>&1; rc=$?
tail -2 gpurun_out/check/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench" && timeout -k 10 400 python tools/kbench.py --sizes 4096,8192,16384 --ln "" --variants auto,pipe_sched --rounds 5 --out gpurun_out/check/kbench.jsonl > gpurun_out/check/kbench.log 2>&1; rc=$?
cat gpurun_out/check/kbench.jsonl; exit $rc
