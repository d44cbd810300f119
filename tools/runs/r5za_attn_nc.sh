#!/bin/bash
# forward / backward attention throughput causal and non-causal, at the gpt-1b shape and at the
# B 16 x H 64 x N 2048 x D 128 shape the CDNA4 guide quotes its forward figures on
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5za_attn_nc
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u tools/attn_bench.py --shapes 4x16x2048x128,16x64x2048x128 --rounds 3 > $OUT/causal.jsonl 2> $OUT/causal.err || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --shapes 4x16x2048x128,16x64x2048x128 --rounds 3 --no-causal > $OUT/noncausal.jsonl 2> $OUT/noncausal.err || exit $?
cut -c1-200 $OUT/causal.jsonl $OUT/noncausal.jsonl
