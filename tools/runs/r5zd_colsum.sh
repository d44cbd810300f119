# gpt-1b step kernel traces after the LPT attention order and the one-pass LayerNorm backward (native
# vs torch ops), then the step timing. (Run with a 16 x 16 column-sum finalize, since reverted: it
# took the same 4.8-4.9 us as the 64 x 4 one.)
export PROF_OUT=r5zd_colsum
bash $GRAFT_REPO_ROOT/tools/runs/gpu_r4_proftrain.sh || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm or linear or act_grad or bias" > gpurun_out/r5zd_colsum/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5zd_colsum/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out gpurun_out/r5zd_colsum/train.jsonl > gpurun_out/r5zd_colsum/train.log 2>&1
rc=$?
cat gpurun_out/r5zd_colsum/summary_*.json gpurun_out/r5zd_colsum/train.jsonl
exit $rc
