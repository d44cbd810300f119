# flash attention: numerics vs fp32 SDPA, then the A/B vs aotriton
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_attention.py > gpurun_out/r5b/pytest_attn.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/r5b/pytest_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r5b/attn_bench.jsonl 2>&1
echo "bench rc=$?"; cat gpurun_out/r5b/attn_bench.jsonl
