#!/bin/bash
set -o pipefail
O=gpurun_out/r3pt; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for w in native torch; do
  timeout -k 10 180 rocprofv3 --kernel-trace -d $R/$O/$w -o run -- python3 $R/tools/prof_train.py $w gpt-1b 4 2048 > $R/$O/$w.log 2>&1 || exit $?
  echo "== $w"; python3 $R/tools/rocpd_stats.py $(ls $R/$O/$w/*.db | head -1) --csv $R/$O/$w.csv | head -30 || exit $?
done
