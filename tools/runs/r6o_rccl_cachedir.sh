#!/bin/bash
# what persists between the first and the second RCCL communicator on a box
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6o_rccl_cachedir
mkdir -p $OUT
B=$R/kubeflow_rm_amd/bin/kfamd-readiness
echo "HOME=$HOME TMPDIR=$TMPDIR XDG_CACHE_HOME=$XDG_CACHE_HOME"
(ls -la $HOME/.cache 2>&1; du -sh $HOME/.cache/* 2>&1) > $OUT/before.txt
find / -xdev -newer $OUT/before.txt -type f 2>/dev/null | grep -v "^/proc\|^/sys\|$OUT" | head -50 > /dev/null
touch $OUT/stamp; sleep 1
timeout -k 10 120 $B --rccl-single --skip-ln --no-fast-exit > $OUT/first.json 2> $OUT/first.err || exit $?
python3 -c "
import json
d=json.loads(open('$OUT/first.json').read().strip().splitlines()[-1]); print('first comm_init_ms', round(d['allreduce']['comm_init_ms']))"
(ls -la $HOME/.cache 2>&1; du -sh $HOME/.cache/* 2>&1) > $OUT/after.txt
timeout -k 10 60 find $HOME /tmp /var/tmp -newer $OUT/stamp -type f 2>/dev/null | head -40 > $OUT/new_files.txt
wc -l $OUT/new_files.txt; head -20 $OUT/new_files.txt; cat $OUT/after.txt | head -20
