# round 4: rocprofv3 kernel traces of 6 gpt-1b training steps, framework kernels vs torch ops, grouped by
# role (tools/train_kernel_summary.py); each trace bounded, stop at the first failure
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${PROF_OUT:-r4_proftrain}
mkdir -p $OUT
for b in native torch; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$b -o run -- python3 $R/tools/prof_train.py $b gpt-1b 4 2048 > $OUT/$b.log 2>&1 || exit $?
done
for b in native torch; do
  f=$(ls $OUT/$b/*kernel_stats.csv $OUT/$b/*/*kernel_stats.csv 2>/dev/null | head -1)
  python3 $R/tools/train_kernel_summary.py $f > $OUT/summary_$b.json || exit 1
done
