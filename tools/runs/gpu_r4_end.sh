# round-4 end state on one MI355X after the training-kernel work: smoke, the driver's bench at its
# defaults, then a rocprofv3 kernel summary of a short bench; each step bounded, stop at the first failure
out=gpurun_out/r4_end
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 560 python -u bench.py > $out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python3 bench.py --steps 10 --warmup 3 --coldstart-runs 0 --coldstart-torch-runs 0 --no-compare-torch > $out/prof.log 2>&1
