#!/bin/bash
# attn_fwd_pp epilogue / priority A/B (tests of each variant first), then the default bench (config 4
# with the kubelet's librccl page-cache prewarm)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
VARS="prod nowide prio" SHAPES=4x16x2048x128,2x32x4096x128 TAG=r6l_fwd_epi timeout -k 10 700 bash tools/runs/r6d_attn_pp.sh || exit $?
mkdir -p gpurun_out/r6l_bench
timeout -k 10 600 python -u bench.py > gpurun_out/r6l_bench/bench.json 2> gpurun_out/r6l_bench/bench.err || exit $?
python3 -c "
import json
d=json.loads(open('gpurun_out/r6l_bench/bench.json').read().strip().splitlines()[-1])
for k in ['value','ab_ratio_ours_over_hipblaslt','cold_start_p50_s','config4_ready_s','config4_rccl_comm_init_ms','config4_rccl_load_ms','config4_gpus','config4_gpu_ids']: print(k, d.get(k))"
