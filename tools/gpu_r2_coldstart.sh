#!/bin/bash
# Cold start at N>=20: stub server and torch-ready server (1-GPU notebook), then the bench line.
set -o pipefail
O=gpurun_out/r2cs; mkdir -p $O; export TMPDIR=/tmp
echo "== coldstart stub x20" && timeout -k 10 300 python -m kubeflow_rm_amd.bench_coldstart --runs 20 > $O/stub.json 2> $O/stub.err || exit $?
head -c 600 $O/stub.json; echo
echo "== coldstart torch-ready x20" && timeout -k 10 400 python -m kubeflow_rm_amd.bench_coldstart --runs 20 --server torch-ready > $O/torch.json 2> $O/torch.err || exit $?
head -c 600 $O/torch.json; echo
echo "== bench" && timeout -k 10 400 python bench.py > $O/bench.log 2>&1; rc=$?; tail -1 $O/bench.log | cut -c1-300; exit $rc
