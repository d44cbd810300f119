#!/bin/bash
# fresh box: librccl read into the page cache first, then the first RCCL communicator
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6n_rccl_cache
mkdir -p $OUT
B=$R/kubeflow_rm_amd/bin/kfamd-readiness
python3 -c "
import time
t=time.time(); n=0
with open('/opt/rocm/lib/librccl.so.1','rb') as f:
    while True:
        b=f.read(1<<20)
        if not b: break
        n+=len(b)
print('read', n>>20, 'MiB in', round(time.time()-t,2), 's')" &&
timeout -k 10 120 $B --rccl-single --skip-ln --no-fast-exit > $OUT/first.json 2> $OUT/first.err &&
python3 -c "
import json
d=json.loads(open('$OUT/first.json').read().strip().splitlines()[-1])
print('first after read: comm_init_ms', round(d['allreduce']['comm_init_ms']), 'total_ms', round(d['total_ms']))"
