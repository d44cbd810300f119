# torch-ready fresh-interpreter cold start: A/B of the HIP pre-init placement (after torch._C = new
# default, whole-import overlap = round 3, off), 10 runs each, per-run timings + failure diagnostics
# (profiles/r4_coldstart). rc 1 = runs failed (recorded, keep going); anything else stops the script.
out=gpurun_out/r4_coldstart
mkdir -p $out
step() {  # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m kubeflow_rm_amd.bench_coldstart "$@" > $out/$name.txt 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
step fresh_afterc 200 --runs ${RUNS:-10} --server torch-ready --timeout 30 --max-failures 3 --env KFAMD_HIP_PREINIT=after-c
step fresh_thread 200 --runs ${RUNS:-10} --server torch-ready --timeout 30 --max-failures 3 --env KFAMD_HIP_PREINIT=thread
step fresh_off 200 --runs ${RUNS:-10} --server torch-ready --timeout 30 --max-failures 3 --env KFAMD_HIP_PREINIT=0
step zygote 300 --runs 8 --server torch-ready --zygote --timeout 30
