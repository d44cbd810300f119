#!/bin/bash
# r3: kernel trace of odd-size GEMMs (K pack + odd epilogue) and split-K, ours vs torch.
set -o pipefail
mkdir -p gpurun_out/r3q
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for shape in ${SHAPES:-1500x1500x1500 1000x1000x2056}; do
  for w in ours torch; do
    timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/r3q/${w}_$shape -o run -- python3 $R/tools/prof_gemm.py $w $shape \
      > $R/gpurun_out/r3q/${w}_$shape.log 2>&1 || exit $?
    echo "== $w $shape"; python3 $R/tools/rocpd_stats.py $(ls $R/gpurun_out/r3q/${w}_$shape/*.db | head -1) --gaps || exit $?
  done
done
