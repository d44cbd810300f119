# round 4: the gpt-1b step after the epilogue / split-K fixup changes: kernel traces of both backends (by
# op and role), then the step timing; each step bounded, stop at the first failure
export PROF_OUT=r4_proftrain2
bash $GRAFT_REPO_ROOT/tools/runs/gpu_r4_proftrain.sh || exit $?
cd $GRAFT_REPO_ROOT
for b in native torch; do
  f=$(ls gpurun_out/r4_proftrain2/$b/*kernel_trace.csv gpurun_out/r4_proftrain2/$b/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/train_gemm_roles.py $f > gpurun_out/r4_proftrain2/gemm_roles_$b.json || exit 1
done
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out gpurun_out/r4_proftrain2/train.jsonl > gpurun_out/r4_proftrain2/train.log 2>&1 &&
timeout -k 10 300 python -u tools/train_bench.py --model gpt-small --batch 16 --seq 2048 --steps 10 --rounds 3 --out gpurun_out/r4_proftrain2/train.jsonl >> gpurun_out/r4_proftrain2/train.log 2>&1
