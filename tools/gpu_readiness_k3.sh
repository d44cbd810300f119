#!/bin/bash
# Readiness op on one MI355X with the K3 one-shot all-reduce simulated over 2/4/8 ranks on device 0.
set -o pipefail
mkdir -p gpurun_out/readiness_k3
export TMPDIR=/tmp
for r in 2 4 8; do
  echo "== readiness --oneshot-sim $r" && timeout -k 10 120 ./kubeflow_rm_amd/bin/kfamd-readiness --oneshot-sim $r \
    > gpurun_out/readiness_k3/readiness_sim$r.json 2> gpurun_out/readiness_k3/readiness_sim$r.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/readiness_k3/readiness_sim$r.json')); o=d['allreduce_oneshot']; print(d['ok'], o['correct'], [(s['bytes'], round(s['us'],1)) for s in o['sweep']])"
done
