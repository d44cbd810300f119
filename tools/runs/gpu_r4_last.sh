# round 4, last check of the committed tree: the whole GPU suite and smoke; stop at the first failure
out=gpurun_out/r4_last
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
