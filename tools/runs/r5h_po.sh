#!/bin/bash
# persistent-overlapped (PO) w4 GEMM vs production vs torch.matmul (tools/w4_ab.py), bitwise check first
set -o pipefail
mkdir -p gpurun_out/r5h_po
timeout -k 10 300 python -u tools/w4_ab.py --variants r4 --sizes 4096,8192,16384 --rounds 7 --diag "" \
  > gpurun_out/r5h_po/ab.jsonl 2> gpurun_out/r5h_po/ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r5h_po/ab.jsonl; tail -5 gpurun_out/r5h_po/ab.err; exit $rc
