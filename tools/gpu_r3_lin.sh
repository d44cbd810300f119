#!/bin/bash
# r3: linear fwd+bwd — numerics of the epilogue/act-grad path, timing vs torch, kernel trace.
set -o pipefail
mkdir -p gpurun_out/r3l
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "epilogue or preact or act_grad or linear or edge" > gpurun_out/r3l/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r3l/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kbench.py --sizes "" --ln "" --rounds 5 --linear 8192x4096x4096,16384x4096x4096 \
  > gpurun_out/r3l/kbench.log 2>&1; rc=$?
grep kind gpurun_out/r3l/kbench.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3l/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_linear.py ours > $GRAFT_REPO_ROOT/gpurun_out/r3l/prof.log 2>&1
