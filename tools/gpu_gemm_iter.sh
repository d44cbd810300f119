#!/bin/bash
# GEMM iteration: numerics of every variant, then an interleaved variant sweep.
set -o pipefail
mkdir -p gpurun_out
VARS=${VARS:-fast,pipe,pipe_sched}
SIZES=${SIZES:-4096,8192,16384}
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/pytest_gemm.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/kbench.py --sizes $SIZES --ln "" --variants $VARS --rounds 5 --out gpurun_out/kbench_iter.jsonl > gpurun_out/kbench_iter.log 2>&1 || exit $?
cat gpurun_out/kbench_iter.jsonl
