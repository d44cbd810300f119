#!/bin/bash
# r3: stream-K — numerics (plan, epilogues, the non-co-resident fallback), then timing vs the plain
# kernel and torch on the under-filled shapes.
set -o pipefail
mkdir -p gpurun_out/r3sk
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "${KSEL:-streamk}" > gpurun_out/r3sk/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r3sk/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/kbench.py --sizes "" --ln "" --rounds ${ROUNDS:-5} \
  --streamk ${SHAPES:-3072x3072x8192,6144x2048x8192,5120x5120x2048,3000x3000x3000,4000x4000x4000,6144x2048x4096,2048x6144x8192,8192x8192x8192} \
  --out gpurun_out/r3sk/kbench.jsonl > gpurun_out/r3sk/kbench.log 2>&1; rc=$?
grep kind gpurun_out/r3sk/kbench.log; exit $rc
