set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_rccl.py > gpurun_out/r5a/pytest_rccl.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 gpurun_out/r5a/pytest_rccl.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --force-dist --coldstart-runs 3 --coldstart-torch-runs 2 > gpurun_out/r5a/bench_force_dist.json 2> gpurun_out/r5a/bench_force_dist.err
echo "bench rc=$?"
tail -c 1500 gpurun_out/r5a/bench_force_dist.json
