#!/bin/bash
# r3: GEMM edge tiles / operand layouts / act-grad — numerics first, then the kbench sweep.
set -o pipefail
mkdir -p gpurun_out/r3g
export TMPDIR=/tmp
echo "== gemm tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "${KSEL:-edge or mm_ or preact or act_grad or linear or identity or fast_path or epilogue or residual}" \
  > gpurun_out/r3g/pytest.log 2>&1; rc=$?
tail -25 gpurun_out/r3g/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench"
timeout -k 10 500 python -u tools/kbench.py --sizes ${SIZES:-1500,3000,4000,4096,8000,8192} --ln "" --rounds 3 \
  --layouts ${LAYOUTS:-4096x4096x4096,8192x4096x8192,1000x1500x776} --linear ${LINEAR:-8192x4096x4096} \
  --out gpurun_out/r3g/kbench.jsonl > gpurun_out/r3g/kbench.log 2>&1; rc=$?
cat gpurun_out/r3g/kbench.log; exit $rc
