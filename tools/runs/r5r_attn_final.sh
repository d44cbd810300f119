#!/bin/bash
# production attention (atomic-free dQ kernel, LDS-DMA backward staging): GPU tests of the attention,
# models and smoke, the bench vs the atomic build and aotriton, the gpt-1b / gpt-small train steps
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5r_attn_final
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_models.py tests/test_gpu_rccl.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for r in 1 2; do
  for v in prod atomics; do
    KFAMD_KERNEL_LIB=$R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$v.so timeout -k 10 200 python -u tools/attn_bench.py > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    echo "== $v round $r"; python3 -c "
import json
for l in open('$OUT/bench_${v}_$r.jsonl'):
    d=json.loads(l); print(d['shape'], d['pass'], d['ours_us'], d['sdpa_us'], d['speedup'], d['ours_tflops'])"
  done
done
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out $OUT/train.jsonl > $OUT/train.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/train_bench.py --model gpt-small --batch 16 --seq 2048 --steps 10 --rounds 3 --out $OUT/train.jsonl >> $OUT/train.log 2>&1 || exit $?
cut -c1-330 $OUT/train.jsonl
