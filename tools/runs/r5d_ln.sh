# round 5: LayerNorm residual-gradient fusion (numerics + model tests), LN fwd/bwd bandwidth vs torch
# and the copy roof with a rocprofv3 kernel trace, then the gpt-1b step trace again
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5d_ln
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_layernorm_residual.py tests/test_gpu_models.py tests/test_gpu_kernels.py -k "norm or gpt or layer" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kbench.py --sizes "" --ln 8192x4096,8192x8192,32768x8192,8192x2048 --rounds 5 --no-torch --out $OUT/kbench_ln.jsonl > $OUT/kbench.log 2>&1 || exit $?
cat $OUT/kbench_ln.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o ln -- python3 $R/tools/kbench.py --sizes "" --ln 8192x4096,8192x8192,32768x8192 --rounds 2 > $OUT/prof.log 2>&1 || exit $?
export PROF_OUT=r5d_ln/train
bash $R/tools/runs/gpu_r4_proftrain.sh || exit $?
cd $R && timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out $OUT/train.jsonl > $OUT/train.log 2>&1
rc=$?; cat $OUT/train.jsonl $OUT/train/summary_native.json; exit $rc
