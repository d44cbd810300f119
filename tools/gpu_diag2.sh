#!/bin/bash
set -o pipefail
O=gpurun_out/diag2; mkdir -p $O; export TMPDIR=/tmp
echo "== tp oneshot" && timeout -k 10 240 python -u -m pytest tests/test_gpu_collectives.py -k "tp_forward" -x -v --timeout 200 --timeout-method thread > $O/tp.log 2>&1; rc=$?; tail -3 $O/tp.log; [ $rc -eq 0 ] || exit $rc
echo "== diag" && timeout -k 10 200 python tools/w4_diag.py 4096,8192 > $O/diag.jsonl 2>&1 || exit $?
cat $O/diag.jsonl
