# cold start of the torch-ready notebook server: forked from the kubelet's zygote vs a fresh
# interpreter, and the stub server through the zygote (profiles/r3d_zygote)
set -o pipefail
mkdir -p gpurun_out/r3d_zygote
timeout -k 10 400 python -u -m kubeflow_rm_amd.bench_coldstart --runs ${RUNS:-8} --server torch-ready --zygote > gpurun_out/r3d_zygote/torch_ready_zygote.txt 2>&1 &&
if [ -z "$ZYGOTE_ONLY" ]; then
timeout -k 10 300 python -u -m kubeflow_rm_amd.bench_coldstart --runs 6 --server torch-ready > gpurun_out/r3d_zygote/torch_ready_fresh.txt 2>&1 &&
timeout -k 10 200 python -u -m kubeflow_rm_amd.bench_coldstart --runs 8 --zygote > gpurun_out/r3d_zygote/stub_zygote.txt 2>&1
fi
