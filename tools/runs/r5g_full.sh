# round 5 checkpoint: the whole GPU suite, smoke(), the default bench line, the gpt step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${RUN_TAG:-r5g}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread tests/ > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -c 600 $OUT/bench.json
timeout -k 10 300 python -u tools/train_bench.py --model gpt-1b --batch 4 --seq 2048 --steps 10 --rounds 3 --out $OUT/train.jsonl > $OUT/train.log 2>&1 &&
timeout -k 10 300 python -u tools/train_bench.py --model gpt-small --batch 16 --seq 2048 --steps 10 --rounds 3 --out $OUT/train.jsonl >> $OUT/train.log 2>&1
rc=$?; cat $OUT/train.jsonl; exit $rc
