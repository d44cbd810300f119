#!/bin/bash
# r3: where the torch-ready notebook server's start goes (import torch / ops / first GEMM), 6 fresh
# processes, plus python -X importtime of torch.
set -o pipefail
O=gpurun_out/r3ti; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python3 -c "
import time; t=time.perf_counter()
from kubeflow_rm_amd.images.notebook_server import warmup_torch
import json; w=warmup_torch(); w['proc_to_ret_ms']=round((time.perf_counter()-t)*1e3,1); print(json.dumps(w))" >> $O/warmup.jsonl 2>>$O/err.log || exit $?
done
cat $O/warmup.jsonl
timeout -k 10 120 python3 -X importtime -c "import torch" 2> $O/importtime.txt || exit $?
sort -t'|' -k2 -n -r $O/importtime.txt | head -40 > $O/importtime_top.txt
timeout -k 10 120 python3 -c "
import time,os; t=time.perf_counter(); import torch; t1=time.perf_counter(); torch.cuda.init(); t2=time.perf_counter()
x=torch.ones(1,device='cuda'); torch.cuda.synchronize(); t3=time.perf_counter()
print('import', round((t1-t)*1e3), 'cuda.init', round((t2-t1)*1e3), 'first tensor', round((t3-t2)*1e3))" | tee $O/split.txt
