#!/bin/bash
set -o pipefail
O=gpurun_out/w4s; mkdir -p $O; export TMPDIR=/tmp
echo "== gemm tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench" && timeout -k 10 400 python tools/kbench.py --sizes 1024,2048,3072,4096,8192 --ln "" --variants auto,w4,w4s --rounds 3 --out $O/kbench.jsonl > $O/kbench.log 2>&1 || exit $?
cat $O/kbench.jsonl
