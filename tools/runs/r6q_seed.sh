#!/bin/bash
# comgr seed: the GPU tests that drive the kubelet's GPU paths, then the default bench (config 4's
# first RCCL communicator in its namespace)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6q_seed
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread tests/test_zygote.py tests/test_gpu_rccl.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
ls -la ${XDG_CACHE_HOME:-$HOME/.cache}/kfamd/ > $OUT/seed_ls.txt 2>&1; du -sh ${XDG_CACHE_HOME:-$HOME/.cache}/kfamd/* >> $OUT/seed_ls.txt 2>&1
cat $OUT/seed_ls.txt
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
for k in ['value','ab_ratio_ours_over_hipblaslt','cold_start_p50_s','cold_start_p90_s','config4_ready_s','config4_rccl_comm_init_ms','config4_gpus']: print(k, d.get(k))"
