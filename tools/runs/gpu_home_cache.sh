#!/bin/bash
# Is the readiness op's 150 ms first-launch cost a per-$HOME cache miss? (pods get a fresh HOME)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/homecache; mkdir -p $out
one() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 60 ./kubeflow_rm_amd/bin/kfamd-readiness --skip-allreduce > $out/$label.json 2>$out/$label.err || return $?
  python3 -c "import json; d=json.load(open('$out/$label.json')); print('$label', round(d['hip_init_ms'],1), {k: round(v,1) for k,v in d['gemm'][0]['stages'].items()}, {k: round(v,1) for k,v in d['stages_ms'].items()}, round(d['total_ms'],1))"
}
H=$(mktemp -d)
one warmup HOME=$H && sleep 0.3 &&
one fixed1 HOME=$H && sleep 0.3 && one fixed2 HOME=$H && sleep 0.3 &&
one fresh1 HOME=$(mktemp -d) && sleep 0.3 && one fresh2 HOME=$(mktemp -d) && sleep 0.3 &&
one fresh_xdg1 HOME=$(mktemp -d) XDG_CACHE_HOME=$H/.cache && sleep 0.3 && one fresh_xdg2 HOME=$(mktemp -d) XDG_CACHE_HOME=$H/.cache && sleep 0.3 &&
one fresh_nocache1 HOME=$(mktemp -d) AMD_COMGR_CACHE=0 && sleep 0.3 && one fresh_nocache2 HOME=$(mktemp -d) AMD_COMGR_CACHE=0 &&
echo "== files under the fixed HOME" && (cd $H && find . -type f | head -20 && du -sh . )
