#!/bin/bash
# GPU runtime start-up breakdown (tools/probe/hipinit_probe), 4 fresh processes per mode, then the
# readiness op's RCCL stage on one device (JSON must stay clean on stdout).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/probe; mkdir -p $out
for m in hsa hip alloc hsa hip alloc; do
  for i in 1 2; do timeout -k 10 60 ./tools/probe/hipinit_probe $m || exit $?; done
done | tee $out/probe.jsonl &&
timeout -k 10 120 ./kubeflow_rm_amd/bin/kfamd-readiness --rccl-single --ar-max-bytes 8388608 > $out/rccl.json 2>$out/rccl.err &&
python3 -c "import json; d=json.load(open('$out/rccl.json')); a=d['allreduce']; print(d['ok'], a['correct'], round(a['comm_init_ms'],1), d['hip_init_ms'], d['total_ms'])"
