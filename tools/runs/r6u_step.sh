#!/bin/bash
# gpt-1b step kernel traces on the round-6 kernels (native vs torch ops, grouped by role), then the
# step timing
export PROF_OUT=r6u_step
bash $GRAFT_REPO_ROOT/tools/runs/gpu_r4_proftrain.sh || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out gpurun_out/r6u_step/train.jsonl > gpurun_out/r6u_step/train.log 2>&1
rc=$?
cat gpurun_out/r6u_step/summary_*.json gpurun_out/r6u_step/train.jsonl
exit $rc
