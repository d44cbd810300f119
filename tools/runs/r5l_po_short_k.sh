#!/bin/bash
# persistent-overlapped w4 GEMM at the gpt-1b projection shapes (K = 2048: the epilogue is ~9 % of
# a tile's cycles there, vs ~3 % at K = 8192)
set -o pipefail
mkdir -p gpurun_out/r5l_po
timeout -k 10 300 python -u tools/w4_ab.py --variants r4 --sizes 8192x6144x2048,8192x8192x2048,8192x2048x8192,16384x8192x2048 --rounds 7 --diag "" \
  > gpurun_out/r5l_po/ab.jsonl 2> gpurun_out/r5l_po/ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r5l_po/ab.jsonl; tail -3 gpurun_out/r5l_po/ab.err; exit $rc
