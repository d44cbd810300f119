#!/bin/bash
# superblock raster adopted (KFW4_SUPER, operands past the MALL): the GEMM GPU tests on the production
# library, then the 7-round A/B of production vs the row-group raster vs hipBLASLt
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6zn_super}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r6zn_super} VARS=r4,nosuper bash tools/runs/r6g_w4_ab.sh
