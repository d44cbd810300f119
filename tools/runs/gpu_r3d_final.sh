#!/bin/bash
# end-of-round GPU pass: kfctl top on the real node, then the full validation (tests, smoke, bench)
set -o pipefail
O=gpurun_out/r3d_final; mkdir -p $O; export TMPDIR=/tmp
echo "== top demo" && timeout -k 10 300 python -u tools/runs/gpu_top_demo.py > $O/top_demo.log 2>&1; rc=$?; tail -30 $O/top_demo.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/gpu_validate.sh r3d_final
