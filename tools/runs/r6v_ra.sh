#!/bin/bash
# attn_fwd_pp LDS read-ahead (KFATT_FWD_RA) and split softmax chains (KFATT_FWD_SPLIT): numerics of
# every variant, then three rounds in rotating order (causal + non-causal)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6v_ra}
mkdir -p $OUT
cd $R
VARS=${VARS:-prod ra2 ra4 split ra4split}
lib() { echo $R/kubeflow_rm_amd/lib/attnab/libkfamd_kernels_$1.so; }
for v in $VARS; do
  KFAMD_KERNEL_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
set -- $VARS
for r in 1 2 3; do
  for v in "$@"; do
    KFAMD_KERNEL_LIB=$(lib $v) timeout -k 10 200 python -u tools/attn_bench.py --shapes ${SHAPES:-4x16x2048x128,2x32x4096x128} > $OUT/bench_${v}_$r.jsonl 2> $OUT/bench_${v}_$r.err || exit $?
    KFAMD_KERNEL_LIB=$(lib $v) timeout -k 10 200 python -u tools/attn_bench.py --no-causal --shapes ${NCSHAPES:-4x16x2048x128} > $OUT/bench_nc${v}_$r.jsonl 2> $OUT/bench_nc${v}_$r.err || exit $?
  done
  set -- "${@:2}" "$1"   # rotate the order
done
python3 - <<PY
import json, glob, statistics, collections
res = collections.defaultdict(list)
for f in glob.glob("$OUT/bench_*_*.jsonl"):
    v = f.split("bench_")[1].rsplit("_", 1)[0]
    for l in open(f):
        d = json.loads(l); res[(d["shape"], d["pass"], v)].append(d["ours_us"])
for k in sorted(res):
    print(k, [round(x, 1) for x in sorted(res[k])], "median", round(statistics.median(res[k]), 1))
PY
