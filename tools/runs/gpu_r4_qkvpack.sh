# round 4: QKV gradient pack + parallel LayerNorm dgamma/dbeta finalize: the whole GPU suite, then the
# gpt-1b traces by op and role and the training steps (tools/runs/gpu_r4_proftrain2.sh); stop at the first failure
out=gpurun_out/r4_qkvpack
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
bash tools/runs/gpu_r4_proftrain2.sh
