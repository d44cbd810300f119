set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/skp
timeout -k 10 150 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k streamk > gpurun_out/skp/t.log 2>&1; rc=$?; tail -2 gpurun_out/skp/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/sk_sweep.py 3072x3072x8192,2304x2304x4096,6144x2048x4096,5120x5120x2048 || exit $?
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/skp/kt -o run -- python3 $R/tools/sk_prof.py 2304x2304x4096 1,3,8 > $R/gpurun_out/skp/kt.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d $R/gpurun_out/skp/pmc -o run -- python3 $R/tools/sk_prof.py 2304x2304x4096 1,3,8 > $R/gpurun_out/skp/pmc.log 2>&1 || exit $?
echo ok
