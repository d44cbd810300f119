#!/bin/bash
# Readiness op in profile mode on one MI355X: self-spawned rocprofv3 child, kernel stats merged.
set -o pipefail
O=gpurun_out/readiness_prof; mkdir -p $O; export TMPDIR=/tmp
echo "== readiness profile mode" && KFAMD_READINESS_PROFILE=1 KFAMD_PROFILE_DIR=$PWD/$O/prof KFAMD_TERMINATION_LOG=$PWD/$O/termination.json \
  timeout -k 10 180 ./kubeflow_rm_amd/bin/kfamd-readiness --skip-allreduce > $O/readiness.json 2> $O/readiness.err; rc=$?
python -c "import json; d=json.load(open('$O/readiness.json')); print(d['ok'], json.dumps(d['rocprof']['kernel_stats'])[:600])"
cat $O/termination.json | head -c 800; echo; exit $rc
