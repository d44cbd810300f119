#!/bin/bash
# K3 one-shot all-reduce on the GPU box: numerics / protocol tests, then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out/k3
export TMPDIR=/tmp
echo "== k3 tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives.py -x -v --timeout 120 --timeout-method thread > gpurun_out/k3/pytest_k3.log 2>&1; rc=$?
tail -8 gpurun_out/k3/pytest_k3.log; [ $rc -eq 0 ] || exit $rc
echo "== all gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k3/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/k3/pytest_gpu.log; exit $rc
