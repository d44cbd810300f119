#!/bin/bash
# Round-2 GPU validation: new collective tests first (isolated, time-limited), then every GPU test,
# smoke, the 1-GPU bench (GEMM + 10-run cold start).
set -o pipefail
O=gpurun_out/${1:-r2v}; mkdir -p $O; export TMPDIR=/tmp
echo "== collectives" && timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives.py -x -v --timeout 200 --timeout-method thread > $O/coll.log 2>&1; rc=$?
tail -4 $O/coll.log; [ $rc -eq 0 ] || exit $rc
echo "== all gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 400 python bench.py --compare-torch > $O/bench.log 2>&1; rc=$?; tail -1 $O/bench.log | cut -c1-400; exit $rc
