#!/bin/bash
# where config 4's 5.6 s RCCL communicator build goes: kfamd-readiness --rccl-single under HIP / RCCL
# loader settings, each its own bounded run
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6k_rccl_init
mkdir -p $OUT
B=$R/kubeflow_rm_amd/bin/kfamd-readiness
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 120 $B --rccl-single --skip-ln --no-fast-exit > $OUT/$tag.json 2> $OUT/$tag.err
  local rc=$?
  python3 -c "
import json
d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1])
ar=d.get('allreduce',{})
print('$tag rc=$rc', 'comm_init_ms', round(ar.get('comm_init_ms',-1)), 'rccl_load_ms', round(d.get('rccl_load_ms',-1)), 'hip_init_ms', round(d.get('hip_init_ms',-1)), 'total_ms', round(d.get('total_ms',-1)), 'correct', ar.get('correct'))" || tail -3 $OUT/$tag.err
  return $rc
}
run base X=1 &&
run deferred1 HIP_ENABLE_DEFERRED_LOADING=1 &&
run deferred0 HIP_ENABLE_DEFERRED_LOADING=0 &&
run nodebug NCCL_DEBUG=WARN NCCL_IB_DISABLE=1 NCCL_NET_PLUGIN=none &&
run infolog NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,ENV &&
grep -E "NCCL INFO|init" $OUT/infolog.err | head -60 > $OUT/infolog_head.txt; tail -30 $OUT/infolog.err > $OUT/infolog_tail.txt; true
