#!/bin/bash
# LayerNorm forward with the round-5 launch policy (streaming kernel at 1-2 generations, gamma/beta
# prefetch at hidden 8192, DPP reductions): numerics, kbench fwd+bwd vs torch and the copy roof,
# rocprofv3 kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5k_ln
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_layernorm_residual.py tests/test_gpu_kernels.py -k "norm or layer" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kbench.py --sizes "" --ln 8192x4096,8192x8192,32768x8192,8192x2048,16384x4096 --rounds 5 --out $OUT/kbench_ln.jsonl > $OUT/kbench.log 2>&1 || exit $?
cut -c1-260 $OUT/kbench_ln.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o ln -- python3 $R/tools/kbench.py --sizes "" --ln 8192x4096,8192x8192,32768x8192 --rounds 2 > $OUT/prof.log 2>&1 || exit $?
grep -i "norm_fwd\|layer_norm_kernel\|ln_bwd" $OUT/prof/ln_kernel_stats.csv | cut -c1-200
cd $R && timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out $OUT/train.jsonl > $OUT/train.log 2>&1 || exit $?
cat $OUT/train.jsonl
