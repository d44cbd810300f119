#!/bin/bash
# Control-plane sanitizer run: build kflite + the split binaries with
# ThreadSanitizer and with AddressSanitizer+UBSan (ROCm LLVM runtimes, see _build.SANITIZER_CXX),
# then drive the end-to-end suites (real process pods, watches, webhooks, gateway, KFAM, load test)
# against each build. Host code only: GPU sanitizers are not available on the target pool.
#
#   bash tools/sanitize.sh [outdir]       (e.g. profiles/r2_sanitizers)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${1:-profiles/r1_sanitizers}
mkdir -p "$OUT"
# every suite that drives the native control plane concurrently (the prober pool,
# the TokenReview cache, the mesh listener, kubectl create/patch/apply and the split binaries too)
SUITES="tests/test_pod_addresses.py tests/test_comgr_seed.py tests/test_pod_network_isolation.py tests/test_resource_validation.py tests/test_crd_schemas.py tests/test_zygote.py tests/test_kubectl_cli.py tests/test_e2e_controlplane.py tests/test_odh.py tests/test_e2e_tensorboard_pvcviewer.py tests/test_loadtest.py tests/test_kfam.py tests/test_apiserver.py tests/test_e2e_telemetry.py tests/test_e2e_multigpu.py tests/test_resilience.py tests/test_kubelet_probes.py tests/test_gateway_authz.py tests/test_kubectl_mutate.py tests/test_kubectl_apply.py tests/test_split_binaries.py tests/test_tls.py"
rc=0
for san in thread address; do
  python -c "from kubeflow_rm_amd import _build; _build.build_native(sanitize='$san', build_type='RelWithDebInfo')" \
    > "$OUT/build_$san.log" 2>&1 || { echo "build $san failed"; exit 1; }
  logdir=$(mktemp -d /tmp/kfamd-san-XXXX)
  # kflite and every split binary (KFAMD_BIN_DIR) from the instrumented build
  export KFAMD_KFLITE=$PWD/build/native-$san/bin/kflite KFAMD_BIN_DIR=$PWD/build/native-$san/bin KFAMD_TIMEOUT_SCALE=6
  export TSAN_OPTIONS="halt_on_error=0 exitcode=0 log_path=$logdir/report"
  export ASAN_OPTIONS="halt_on_error=0 detect_leaks=1 log_path=$logdir/report"
  export UBSAN_OPTIONS="print_stacktrace=1 log_path=$logdir/report"
  timeout -k 10 2400 python -m pytest $SUITES -q -p no:cacheprovider > "$OUT/pytest_$san.log" 2>&1 || rc=1
  tail -1 "$OUT/pytest_$san.log"
  cat "$logdir"/report* > "$OUT/reports_$san.txt" 2>/dev/null || : > "$OUT/reports_$san.txt"
  n=$(grep -c -E 'WARNING: ThreadSanitizer|ERROR: AddressSanitizer|ERROR: LeakSanitizer|runtime error:' "$OUT/reports_$san.txt")
  echo "$san: $n sanitizer reports"
  grep -E '^SUMMARY' "$OUT/reports_$san.txt" | sort | uniq -c | sort -rn | head -20
  rm -rf "$logdir"
  unset KFAMD_KFLITE KFAMD_BIN_DIR KFAMD_TIMEOUT_SCALE TSAN_OPTIONS ASAN_OPTIONS UBSAN_OPTIONS
done
exit $rc
