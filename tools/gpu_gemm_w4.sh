#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/w4
export TMPDIR=/tmp
echo "== numerics" && timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" > gpurun_out/w4/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/w4/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench" && timeout -k 10 400 python tools/kbench.py --sizes 4096,8192,16384 --ln "" --variants ${W4_VARIANTS:-pipe_sched,w4} --rounds 5 --out gpurun_out/w4/kbench.jsonl > gpurun_out/w4/kbench.log 2>&1; rc=$?
cat gpurun_out/w4/kbench.jsonl; [ $rc -eq 0 ] || exit $rc
echo "== diag" && timeout -k 10 300 python tools/w4_diag.py > gpurun_out/w4/diag.jsonl 2>&1; rc=$?
cat gpurun_out/w4/diag.jsonl; exit $rc
