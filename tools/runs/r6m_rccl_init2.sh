#!/bin/bash
# RCCL communicator time on a fresh box: file read, then --rccl-single twice, then with another
# process holding a HIP context on the GPU (the zygote's warm children / warm ops do on a node)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6m_rccl_init2
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
print('$tag rc=$rc', 'comm_init_ms', round(ar.get('comm_init_ms',-1)), 'hip_init_ms', round(d.get('hip_init_ms',-1)), 'total_ms', round(d.get('total_ms',-1)))" || tail -3 $OUT/$tag.err
  return $rc
}
run first X=1 &&
run second X=1 &&
s=$(date +%s.%N) && cat /opt/rocm/lib/librccl.so.1 > /dev/null && e=$(date +%s.%N) && echo "read librccl (cached?) $(echo "$e - $s" | bc) s" &&
(timeout -k 5 60 python3 -c "import torch,time; torch.zeros(1,device='cuda'); open('$OUT/held','w').write('1'); time.sleep(40)" &) &&
for i in $(seq 1 60); do [ -f $OUT/held ] && break; sleep 1; done &&
run held X=1 &&
run held_deferred0 HIP_ENABLE_DEFERRED_LOADING=0
