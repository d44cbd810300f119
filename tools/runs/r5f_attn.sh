# round 5: flash attention backward with 64-row query tiles and the swizzled dS^T image
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5f
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_bench.py > $OUT/attn_bench.jsonl 2>&1 || exit $?
cat $OUT/attn_bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $OUT/pmc3 -o run -- python3 $R/tools/attn_prof.py 4x16x2048x128 3 > $OUT/pmc3.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o run -- python3 $R/tools/attn_prof.py 4x16x2048x128 3 > $OUT/pmc1.log 2>&1 || exit $?
echo done
