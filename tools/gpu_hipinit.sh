#!/bin/bash
# HIP runtime start-up cost of the in-pod readiness op under different runtime env settings
# (4 fresh processes each). Prints hip_init_ms / alloc_fill_ms / total_ms / process wall ms.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/hipinit; mkdir -p $out
run() {  # name, env...
  local name=$1; shift
  for i in 1 2 3 4; do
    t0=$(date +%s%N)
    env "$@" timeout -k 10 60 ./kubeflow_rm_amd/bin/kfamd-readiness --skip-allreduce > $out/$name.$i.json 2>$out/$name.$i.err || return $?
    t1=$(date +%s%N)
    python3 -c "import json,sys; d=json.load(open('$out/$name.$i.json')); g=d['gemm'][0]['stages']; print('$name', $i, round(d['hip_init_ms'],1), round(g['alloc_fill_ms'],1), round(g['first_gemm_ms'],1), round(d['total_ms'],1), ($t1-$t0)//1000000)"
  done
}
if [ "$1" = "--quick" ]; then
  run default X=1 && run default2 X=1 || exit $?
  echo "== RCCL stage (dlopen) on one device" &&
  timeout -k 10 120 ./kubeflow_rm_amd/bin/kfamd-readiness --rccl-single --ar-max-bytes 8388608 > $out/rccl.json 2>$out/rccl.err &&
  python3 -c "import json; d=json.load(open('$out/rccl.json')); a=d['allreduce']; print(d['ok'], a['correct'], round(a['rccl_load_ms'],1), round(a['comm_init_ms'],1), [(s['bytes'], round(s['us'],1)) for s in a['sweep']])"
  exit $?
fi
run default X=1 &&
run rocr_vis ROCR_VISIBLE_DEVICES=0 &&
run hip_vis HIP_VISIBLE_DEVICES=0 &&
run hwq1 GPU_MAX_HW_QUEUES=1 &&
run nosdma HSA_ENABLE_SDMA=0 &&
run eager HIP_ENABLE_DEFERRED_LOADING=0 &&
run noint HSA_ENABLE_INTERRUPT=0 &&
run combo ROCR_VISIBLE_DEVICES=0 GPU_MAX_HW_QUEUES=1 &&
run default2 X=1
