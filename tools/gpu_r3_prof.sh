#!/bin/bash
# r3: kernel traces of the shapes still behind torch (odd-size padded GEMM, small linear fwd+bwd).
set -o pipefail
mkdir -p gpurun_out/r3p
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "splitk" > gpurun_out/r3p/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r3p/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
for w in ours torch; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/r3p/g_$w -o run -- python3 $R/tools/prof_gemm.py $w 1500x1500x1500 \
    > $R/gpurun_out/r3p/g_$w.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/r3p/l_$w -o run -- python3 $R/tools/prof_linear.py $w 1024x4096x4096 \
    > $R/gpurun_out/r3p/l_$w.log 2>&1 || exit $?
done
for d in g_ours g_torch l_ours l_torch; do
  echo "== $d"; python3 $R/tools/rocpd_stats.py $(ls $R/gpurun_out/r3p/$d/*/*.db $R/gpurun_out/r3p/$d/*.db 2>/dev/null | head -1) || true
done
