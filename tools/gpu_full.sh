#!/bin/bash
# Full GPU validation: new K3 IPC test first (isolated, time-limited), then every GPU test, smoke, bench.
set -o pipefail
O=gpurun_out/full; mkdir -p $O; export TMPDIR=/tmp
echo "== ipc one-shot (2 processes, 1 GPU)" && timeout -k 10 240 python -u -m pytest tests/test_gpu_collectives.py -k ipc -x -v --timeout 200 --timeout-method thread > $O/ipc.log 2>&1; rc=$?
tail -4 $O/ipc.log; [ $rc -eq 0 ] || exit $rc
echo "== all gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
grep -E 'hipGraph|passed|failed' $O/pytest_gpu.log | tail -4; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > $O/bench.log 2>&1; rc=$?; tail -1 $O/bench.log | cut -c1-250; exit $rc
