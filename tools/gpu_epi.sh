#!/bin/bash
set -o pipefail
O=gpurun_out/epi; mkdir -p $O; export TMPDIR=/tmp
echo "== gemm tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== diag" && timeout -k 10 200 python tools/w4_diag.py 4096,8192 > $O/diag.jsonl 2>&1 || exit $?
cat $O/diag.jsonl
echo "== kbench" && timeout -k 10 400 python tools/kbench.py --sizes 4096,8192,16384 --ln "" --variants auto,pipe_sched --rounds 5 --out $O/kbench.jsonl > $O/kbench.log 2>&1 || exit $?
cat $O/kbench.jsonl
echo "== bench" && timeout -k 10 300 python bench.py --coldstart-runs 0 > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
