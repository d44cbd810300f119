# round 5: gpt-1b / gpt-small training step with the flash attention kernels: kernel traces of both
# backends (no aotriton kernel on the native side), then the step timing
export PROF_OUT=r5c_train
bash $GRAFT_REPO_ROOT/tools/runs/gpu_r4_proftrain.sh || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out gpurun_out/r5c_train/train.jsonl > gpurun_out/r5c_train/train.log 2>&1 &&
timeout -k 10 300 python -u tools/train_bench.py --model gpt-small --batch 16 --seq 2048 --steps 10 --rounds 3 --out gpurun_out/r5c_train/train.jsonl >> gpurun_out/r5c_train/train.log 2>&1
rc=$?
cat gpurun_out/r5c_train/summary_*.json gpurun_out/r5c_train/train.jsonl
grep -c aotriton gpurun_out/r5c_train/native/*kernel_stats.csv gpurun_out/r5c_train/native/*/*kernel_stats.csv 2>/dev/null || true
exit $rc
