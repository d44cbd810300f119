#!/bin/bash
# Does /dev/kfd open wait for the previous GPU process's teardown? hsa probe after a gap of S s.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
for s in 0 0 0.1 0.25 0.5 1 2 0 4 0; do
  sleep $s
  echo -n "gap=$s " && timeout -k 10 60 ./tools/probe/hipinit_probe hsa || exit $?
done | tee gpurun_out/probe/gap.txt
