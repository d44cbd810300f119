#!/bin/bash
# the act-grad GEMM epilogue with packed-f32 act' : numerics, then fused vs GEMM + act_grad
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5zg_dact2
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dgrad_act or mlp" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/dact_bench.py > $OUT/bench.jsonl 2> $OUT/bench.err || exit $?
cat $OUT/bench.jsonl
