#!/bin/bash
# production attention after the attn_fwd_pp change: GPU numerics, the interleaved bench (causal and
# not), then the PMC passes of tools/runs/r5t_attn_pmc.sh (MFMA busy per kernel)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6e_attn}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u tools/attn_bench.py > $OUT/causal.jsonl 2> $OUT/causal.err || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --no-causal > $OUT/noncausal.jsonl 2> $OUT/noncausal.err || exit $?
cat $OUT/causal.jsonl $OUT/noncausal.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['shape'], d['causal'], d['pass'], d['ours_us'], d['sdpa_us'], d['ours_tflops'])"
TAG=${TAG:-r6e_attn}/pmc bash tools/runs/r5t_attn_pmc.sh > /dev/null || exit $?
python3 -c "
import json
d=json.load(open('$OUT/pmc/summary.json'))
for k,v in d.items(): print(k, 'mfma_busy', v.get('mfma_busy_of_gui_active'), 'valu/mfma', round(v.get('SQ_INSTS_VALU',0)/max(1,v.get('SQ_INSTS_MFMA',1)),2))"
