#!/bin/bash
# w4 GEMM schedule knobs vs production vs torch.matmul (hipBLASLt), 7 interleaved rounds, bitwise check first
set -o pipefail
OUT=gpurun_out/${TAG:-r6g_w4_ab}
mkdir -p $OUT
timeout -k 10 600 python -u tools/w4_ab.py --variants ${VARS:-r4,phase3,dma_spread6,rg4,noprio,gm8,prebar2} --sizes 4096,8192,16384 --rounds 7 --diag "" \
  > $OUT/ab.jsonl 2> $OUT/ab.err
rc=$?; echo "ab rc=$rc"; tail -5 $OUT/ab.err
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); t=d['median_tf']; h=t['torch']
    print(d['size'], 'torch', h, ' '.join(f'{k}={v}({v/h:.3f})' for k,v in sorted(t.items(), key=lambda x:-x[1]) if k!='torch'))
    bad=[k for k,v in d['bitwise_equal_to_prod'].items() if not v]
    if bad: print('NOT BITWISE:', bad)"
exit $rc
