#!/bin/bash
# warm GPU children (zygote.py): the GPU tests that drive the zygote + in-pod RCCL configs, then the
# default-path cold start (torch-ready server, zygote, warm child) and the fresh-interpreter baseline
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${RUN_TAG:-r6c_warm}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread tests/test_zygote.py tests/test_gpu_rccl.py > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m kubeflow_rm_amd.bench_coldstart --runs 10 --server torch-ready --zygote --timeout 60 > $OUT/cs_zygote.jsonl 2> $OUT/cs_zygote.err || exit $?
head -c 3000 $OUT/cs_zygote.jsonl
