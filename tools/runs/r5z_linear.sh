#!/bin/bash
# gelu linear at the gpt-1b fc1 shape: the fused pre-activation epilogue vs the split (GEMM + one
# elementwise pass), forward alone and fwd+bwd, vs torch
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5z_linear
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/kbench.py --sizes "" --ln "" --linear 8192x2048x8192,8192x2048x6144,16384x2048x8192 --rounds 5 --out $OUT/linear.jsonl > $OUT/linear.log 2>&1 || exit $?
cat $OUT/linear.jsonl
