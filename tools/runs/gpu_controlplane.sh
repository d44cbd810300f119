#!/bin/bash
# GPU validation of the control-plane path: readiness op on a real MI355X, notebook cold-start
# through kflite with real KFD topology discovery, headline bench, rocprofv3 of the readiness op.
set -o pipefail
mkdir -p gpurun_out/cp
export TMPDIR=/tmp
echo "== readiness" && timeout -k 10 120 kubeflow_rm_amd/bin/kfamd-readiness > gpurun_out/cp/readiness.json 2> gpurun_out/cp/readiness.err || { cat gpurun_out/cp/readiness.*; exit 1; }
cat gpurun_out/cp/readiness.json
echo "== coldstart" && timeout -k 10 300 python -m kubeflow_rm_amd.bench_coldstart --runs 5 > gpurun_out/cp/coldstart.log 2>&1 || { tail -30 gpurun_out/cp/coldstart.log; exit 1; }
cat gpurun_out/cp/coldstart.log
echo "== coldstart (no readiness op)" && timeout -k 10 300 python -m kubeflow_rm_amd.bench_coldstart --runs 5 --no-readiness > gpurun_out/cp/coldstart_noop.log 2>&1 || { tail -30 gpurun_out/cp/coldstart_noop.log; exit 1; }
cat gpurun_out/cp/coldstart_noop.log
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/cp/bench.log 2>&1 || { tail -30 gpurun_out/cp/bench.log; exit 1; }
tail -1 gpurun_out/cp/bench.log
echo "== rocprof readiness" && cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/cp/prof -o readiness -- $GRAFT_REPO_ROOT/kubeflow_rm_amd/bin/kfamd-readiness > $GRAFT_REPO_ROOT/gpurun_out/cp/prof.log 2>&1 || exit $?
find $GRAFT_REPO_ROOT/gpurun_out/cp/prof -name '*stats*'
