#!/bin/bash
# PMC passes over the production attention kernels at the gpt-1b shape (fwd, dK/dV, dQ), each pass
# its own bounded run, then a per-kernel summary (tools/attn_pmc_summary.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r5t_attn_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o run -- python3 $R/tools/attn_prof.py 4x16x2048x128 3 > $OUT/pmc1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAVES --output-format csv -d $OUT/pmc2 -o run -- python3 $R/tools/attn_prof.py 4x16x2048x128 3 > $OUT/pmc2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU --output-format csv -d $OUT/pmc3 -o run -- python3 $R/tools/attn_prof.py 4x16x2048x128 3 > $OUT/pmc3.log 2>&1 || exit $?
python3 $R/tools/attn_pmc_summary.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 | tee $OUT/summary.json
