# round 5 end state: kernel traces of the gpt-1b step (native vs torch ops) with the final attention
# kernels, grouped by role
export PROF_OUT=r5z2_train
bash $GRAFT_REPO_ROOT/tools/runs/gpu_r4_proftrain.sh || exit $?
cat $GRAFT_REPO_ROOT/gpurun_out/r5z2_train/summary_*.json
