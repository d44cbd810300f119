#!/bin/bash
# LayerNorm forward: DPP/permlane wave reductions (no ds_bpermute) and the gamma/beta prefetch
# variant (KFAMD_LN_PF = largest VPL that prefetches) vs the plain kernel, kbench + kernel trace;
# the same reductions in flash attention (row max across the wave halves) and cross-entropy
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5i_ln
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_layernorm_residual.py tests/test_gpu_attention.py tests/test_gpu_kernels.py -k "norm or layer or attention or attn or cross" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pf in 0 16 8 0; do
  KFAMD_LN_PF=$pf timeout -k 10 200 python -u tools/kbench.py --sizes "" --ln 8192x4096,8192x8192,32768x8192,8192x2048 --rounds 5 --no-torch --out $OUT/kbench_pf$pf.jsonl > $OUT/kbench_pf$pf.log 2>&1 || exit $?
  echo "pf=$pf"; grep layernorm_fwd $OUT/kbench_pf$pf.jsonl | cut -c1-200
done
timeout -k 10 200 python -u tools/attn_bench.py > $OUT/attn_bench.jsonl 2> $OUT/attn_bench.err || exit $?
cat $OUT/attn_bench.jsonl | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o ln -- python3 $R/tools/kbench.py --sizes "" --ln 8192x4096,8192x8192,32768x8192 --rounds 2 --no-torch > $OUT/prof.log 2>&1 || exit $?
grep norm_fwd $OUT/prof/ln_kernel_stats.csv | cut -c1-220
