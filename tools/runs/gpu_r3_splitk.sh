#!/bin/bash
# r3: split-K numerics, then split vs unsplit vs torch on under-filled shapes, then a rocprof pass.
set -o pipefail
mkdir -p gpurun_out/r3s
export TMPDIR=/tmp
echo "== split-K tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "${KSEL:-splitk or mm_ or preact or linear or fast_path or odd or edge or epilogue or residual}" > gpurun_out/r3s/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r3s/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench split-K"
timeout -k 10 300 python -u tools/kbench.py --sizes "${SIZES:-1000,1024,1500,2048}" --ln "" --rounds 5 \
  --splitk "${SPLITS:-1000x1000x1000,1024x1024x4096,1000x1504x776,512x768x8192,2048x2048x8192,1024x4096x4096,256x4096x8192}" \
  --layouts "${LAYOUTS:-1000x1500x776,1024x1024x4096}" --linear "${LINEAR:-1024x4096x4096,8192x4096x4096}" \
  --out gpurun_out/r3s/kbench.jsonl > gpurun_out/r3s/kbench.log 2>&1; rc=$?
cat gpurun_out/r3s/kbench.log; exit $rc
