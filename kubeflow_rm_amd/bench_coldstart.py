"""Notebook pod cold-start benchmark (BASELINE.json headline, first half).

Brings up the single-binary control plane (``kflite``: API server + notebook/profile
controllers + admission + GPU-aware scheduler + process-pod kubelet + gateway), then for each
run creates a Notebook CR requesting ``gpus_per_notebook`` MI355X GPUs and measures

* ``cold_start_s``   Notebook CREATE -> ``status.readyReplicas == 1`` (wall clock, client side),
* phases from the pod's own (ms-precision) timestamps: reconcile (CR -> StatefulSet),
  schedule (pod -> PodScheduled), init (gpu-readiness op: HIP init + in-pod bf16 MFMA GEMM /
  LayerNorm / RCCL all-reduce on the allocated GPUs), start (container start -> Ready).

The reference publishes no cold-start numbers: the controller path it measures is
notebook_controller.go Reconcile -> StatefulSet -> kubelet; here every hop is native and the
in-pod readiness op is the hand-written gfx950 kernel set (kfamd-readiness).

Usage: ``python -m kubeflow_rm_amd.bench_coldstart --runs 5 --gpus-per-notebook 1``.
"""
from __future__ import annotations

import argparse
import datetime as _dt
import json
import statistics
import time

from .cluster import LocalCluster


def _ts(s: str | None) -> float | None:
    if not s:
        return None
    s = s.rstrip("Z")
    fmt = "%Y-%m-%dT%H:%M:%S.%f" if "." in s else "%Y-%m-%dT%H:%M:%S"
    return _dt.datetime.strptime(s, fmt).replace(tzinfo=_dt.timezone.utc).timestamp()


def _cond(pod: dict, typ: str) -> float | None:
    for c in pod.get("status", {}).get("conditions", []) or []:
        if c.get("type") == typ and c.get("status") == "True":
            return _ts(c.get("lastTransitionTime"))
    return None


def _pct(xs: list[float], q: float) -> float:
    xs = sorted(xs)
    if not xs:
        return float("nan")
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


SERVERS = {
    # stdlib HTTP notebook server (no torch import): the control plane + readiness-op path alone
    "stub": {},
    # jupyter-pytorch-rocm: the server imports torch + kubeflow_rm_amd.ops and runs a GEMM on the
    # allocated GPU before it listens; a readinessProbe makes Ready wait for it
    "torch-ready": {"env": [{"name": "KFAMD_WARMUP", "value": "torch"}], "probe": True},
}


def _diagnose(c, name: str, namespace: str, log_bytes: int = 2048) -> dict:
    """What a failed run leaves behind: the pod's phase, conditions and container states, and the last
    ``log_bytes`` of every container's log (the torch-ready server dumps its threads' stacks there
    every few seconds while it warms up)."""
    out: dict = {"pod": f"{name}-0"}
    try:
        pod = c.get("v1", "Pod", f"{name}-0", namespace)
    except Exception as e:  # noqa: BLE001
        out["pod_error"] = f"{type(e).__name__}: {e}"
        return out
    st = pod.get("status") or {}
    out["phase"] = st.get("phase")
    out["conditions"] = [{k: cnd.get(k) for k in ("type", "status", "reason")} for cnd in st.get("conditions") or []]
    logs = {}
    for cs in (st.get("initContainerStatuses") or []) + (st.get("containerStatuses") or []):
        out.setdefault("containers", []).append({"name": cs.get("name"), "ready": cs.get("ready"),
                                                 "restartCount": cs.get("restartCount"), "state": cs.get("state")})
        try:
            logs[cs.get("name")] = c.pod_logs(f"{name}-0", namespace, container=cs.get("name"))[-log_bytes:]
        except Exception as e:  # noqa: BLE001
            logs[cs.get("name")] = f"<logs unavailable: {type(e).__name__}: {e}>"
    out["logs_tail"] = logs
    return out


class ColdStartFailure(RuntimeError):
    """A run that did not become Ready; ``diag`` is _diagnose()'s record."""

    def __init__(self, msg: str, diag: dict | None = None):
        super().__init__(msg)
        self.diag = diag or {}


def _wait_ready(c, name: str, namespace: str, timeout: float) -> dict:
    """Poll the Notebook every 5 ms until readyReplicas == 1. Every ~100 ms also look at the pod: an
    init container (the GPU readiness op) that terminated non-zero, or a main container that exited,
    fails the run at once with its termination message instead of after the whole timeout. Either
    failure carries the pod's diagnostics (ColdStartFailure.diag)."""
    deadline = time.time() + timeout
    next_pod_check = time.time() + 0.1
    while True:
        try:
            o = c.get("kubeflow.org/v1", "Notebook", name, namespace)
            if (o.get("status") or {}).get("readyReplicas") == 1:
                return o
        except Exception:  # noqa: BLE001 - not created yet / transient
            pass
        now = time.time()
        if now >= next_pod_check:
            next_pod_check = now + 0.1
            try:
                pod = c.get("v1", "Pod", f"{name}-0", namespace)
            except Exception:  # noqa: BLE001
                pod = None
            st = (pod or {}).get("status") or {}
            for cs in (st.get("initContainerStatuses") or []) + (st.get("containerStatuses") or []):
                term = (cs.get("state") or {}).get("terminated") or {}
                if term and term.get("exitCode", 0) != 0:
                    raise ColdStartFailure(f"{name}: container {cs.get('name')} exited {term.get('exitCode')}: "
                                           f"{(term.get('message') or '')[:400]}", _diagnose(c, name, namespace))
        if now > deadline:
            raise ColdStartFailure(f"{name}: not Ready within {timeout:.0f} s", _diagnose(c, name, namespace))
        time.sleep(0.005)


def _teardown(c, name: str, namespace: str, settle_s: float) -> None:
    """Delete the run's Notebook and wait for its pod to go (the GPU is free again), then settle."""
    try:
        c.delete("kubeflow.org/v1", "Notebook", name, namespace)
        c.wait_gone("kubeflow.org/v1", "Notebook", name, namespace, timeout=60)
    except Exception:  # noqa: BLE001 - already gone
        pass
    # the StatefulSet / pod are garbage collected asynchronously; wait for the GPU to free up
    end = time.time() + 60
    while time.time() < end:
        try:
            c.get("v1", "Pod", f"{name}-0", namespace)
        except Exception:  # noqa: BLE001
            break
        time.sleep(0.02)
    time.sleep(settle_s)


def _reconcile_latency(url: str) -> dict:
    """p50 / p99 of controller_runtime_reconcile_time_seconds and workqueue_queue_duration_seconds
    per controller, scraped from the control plane's /metrics (PromQL histogram_quantile)."""
    import urllib.request
    from .loadtest import histogram_quantile, parse_histograms
    with urllib.request.urlopen(url + "/metrics", timeout=10) as r:
        text = r.read().decode()
    out = {}
    for fam, key in (("controller_runtime_reconcile_time_seconds", "reconcile"),
                     ("workqueue_queue_duration_seconds", "queue")):
        for labels, h in parse_histograms(text, fam).items():
            name = dict(labels).get("controller") or dict(labels).get("name") or "?"
            if not h["count"]:
                continue
            out.setdefault(name, {})[key] = {"count": int(h["count"]),
                                             "p50_ms": round(1e3 * histogram_quantile(0.5, h["buckets"]), 3),
                                             "p99_ms": round(1e3 * histogram_quantile(0.99, h["buckets"]), 3)}
    return out


def measure_cold_start(runs: int = 5, gpus_per_notebook: int = 1, gpus: int | None = None, image: str = "kfamd/jupyter-pytorch-rocm:latest",
                       readiness: bool = True, timeout: float = 120.0, namespace: str = "bench",
                       settle_s: float = 0.5, server: str = "stub", odh_oauth: bool = False,
                       zygote: bool = False, env: dict | None = None, deadline: float | None = None,
                       max_failures: int = 2) -> dict:
    """Returns {"p50_s", "p90_s", "runs": [...], "failures": [...], "phases_p50_s": {...}, "readiness": {...},
    "reconcile": {controller: {"reconcile": {p50_ms, p99_ms}, "queue": {...}}}}.

    A run that is not Ready within ``timeout`` (or whose container exits non-zero) is recorded in
    ``failures`` with the pod's phase, container states and log tails (``_diagnose``) and the next
    run goes on; after ``max_failures`` of them the measurement stops. ``deadline`` (wall-clock
    ``time.time()``) stops starting new runs, so a caller with a total budget gets a partial result
    (``"truncated": true``) instead of none. ``env``: extra container env (e.g. an A/B knob).
    p50/p90 are over the runs that became Ready; ``failures`` says how many did not.

    ``server``: "stub" or "torch-ready" (see SERVERS). Both are process pods (no container runtime).
    ``odh_oauth``: the ODH spawn path of SURVEY CS1 with OAuth: the ODH webhook injects the
    oauth-proxy sidecar and the reconciliation lock; the odh-notebook-controller creates the OAuth
    ServiceAccount / Service / Secret / Route and removes the lock once the SA has its image pull
    secret (Q7), and only then does the notebook controller scale the StatefulSet to 1.

    ``zygote``: the kubelet forks the notebook server from a pre-imported interpreter (torch already
    imported, GPU untouched: kubeflow_rm_amd/images/zygote.py) instead of starting a fresh one; the
    runs start once the node's zygote serves (like a node with the image pre-pulled).

    ``settle_s``: pause after the previous run's pod is gone, so runs are independent cold starts.
    The amdgpu KFD tears a GPU process down asynchronously after it exits and the next open of
    /dev/kfd waits for that (100-130 ms right after an exit, 0.1 ms after >= 0.25 s:
    ``profiles/r1_coldstart2/kfd_gap.txt``); back to back, run i+1 would pay run i's teardown.
    """
    out_runs: list[dict] = []
    failures: list[dict] = []
    truncated = False
    with LocalCluster(gpus=gpus, zygote=zygote) as cl:
        if zygote:
            cl.wait_zygotes(timeout=300 if deadline is None else max(1.0, min(300.0, deadline - time.time())))
        c = cl.client
        c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": namespace}})
        for i in range(runs):
            if deadline is not None and time.time() + 1.0 > deadline:
                truncated = True
                break
            if len(failures) >= max_failures:
                truncated = True
                break
            name = f"cs-{i}"
            ann = {} if readiness else {"kfamd.io/gpu-readiness-op": "false"}
            if odh_oauth:
                ann["notebooks.opendatahub.io/inject-oauth"] = "true"
            ctr = {"name": name, "image": image, "resources": {"limits": {"amd.com/gpu": str(gpus_per_notebook)}}}
            srv = SERVERS[server]
            if srv.get("env") or env:
                ctr["env"] = list(srv.get("env") or []) + [{"name": k, "value": str(v)} for k, v in (env or {}).items()]
            if srv.get("probe"):
                ctr["readinessProbe"] = {"httpGet": {"path": f"/notebook/{namespace}/{name}/api/status", "port": 8888},
                                         "periodSeconds": 5}
            nb = {"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
                  "metadata": {"name": name, "namespace": namespace, "annotations": ann},
                  "spec": {"template": {"spec": {"containers": [ctr]}}}}
            t0 = time.time()
            c.create(nb)
            run_timeout = timeout if deadline is None else max(1.0, min(timeout, deadline - time.time()))
            try:
                obj = _wait_ready(c, name, namespace, run_timeout)
            except ColdStartFailure as e:
                failures.append({"run": i, "error": str(e), "after_s": round(time.time() - t0, 3), **e.diag})
                _teardown(c, name, namespace, settle_s)
                continue
            t1 = time.time()
            pod = c.get("v1", "Pod", f"{name}-0", namespace)
            t_sched = _cond(pod, "PodScheduled")
            t_init = _cond(pod, "Initialized")
            t_ready = _cond(pod, "Ready")
            phases = {}
            if t_sched and t_init:
                phases["schedule_to_initialized_s"] = t_init - t_sched
            if t_init and t_ready:
                phases["initialized_to_ready_s"] = t_ready - t_init
            if t_ready:
                phases["create_to_pod_ready_s"] = t_ready - t0
            if t_sched:
                phases["create_to_scheduled_s"] = t_sched - t0
            stages = {}
            # the op's report: the sidecar's (published by the kubelet as a pod annotation) or the
            # init container's termination message (gpu-readiness-mode: init)
            msgs = [((pod.get("metadata") or {}).get("annotations") or {}).get("notebooks.kubeflow.org/gpu-readiness") or ""]
            msgs += [((st.get("state") or {}).get("terminated") or {}).get("message") or ""
                     for st in (pod.get("status") or {}).get("initContainerStatuses") or []]
            for msg in msgs:
                try:
                    rep = json.loads(msg)
                except ValueError:
                    continue
                if not isinstance(rep, dict):
                    continue
                stages = {"hip_init_ms": rep.get("hip_init_ms"), "total_ms": rep.get("total_ms"),
                          "warm_op": 1.0 if rep.get("warm_op_ms") is not None else 0.0,
                          **{f"{k}_ms": v for k, v in (rep.get("stages_ms") or {}).items()},
                          **{f"gemm_{k}": v for k, v in (rep.get("gemm0_stages_ms") or {}).items()}}
            ctl_phases = None
            try:
                ctl_phases = json.loads((c.get("kubeflow.org/v1", "Notebook", name, namespace)["metadata"].get("annotations")
                                         or {}).get("notebooks.kubeflow.org/cold-start-phases", "null"))
            except Exception:
                pass
            warm = None
            if server == "torch-ready":  # the server's own warmup timings (import / first GEMM)
                try:
                    import urllib.request
                    ip = (pod.get("status") or {}).get("podIP")
                    with urllib.request.urlopen(f"http://{ip}:8888/notebook/{namespace}/{name}/api/gpu", timeout=5) as r:
                        warm = json.loads(r.read()).get("warmup")
                    # container start -> server main -> listening -> pod Ready (wall clock, one host)
                    st = next((cs for cs in (pod.get("status") or {}).get("containerStatuses") or []
                               if cs.get("name") == name), {})
                    t_cs = _ts(((st.get("state") or {}).get("running") or {}).get("startedAt"))
                    if warm and t_cs and warm.get("main_ts") and warm.get("listen_ts"):
                        warm["start_to_main_ms"] = round((warm["main_ts"] - t_cs) * 1e3, 1)
                        warm["main_to_listen_ms"] = round((warm["listen_ts"] - warm["main_ts"]) * 1e3, 1)
                        if t_ready:
                            warm["listen_to_pod_ready_ms"] = round((t_ready - warm["listen_ts"]) * 1e3, 1)
                        if t_init:
                            warm["initialized_to_start_ms"] = round((t_cs - t_init) * 1e3, 1)
                except Exception:  # noqa: BLE001 - diagnostics only
                    pass
            warm_child = None
            if zygote:  # did the container take the zygote's warm GPU child? (the kubelet's log line)
                try:
                    warm_child = "# kflite: warm child of zygote" in c.pod_logs(f"{name}-0", namespace, container=name)
                except Exception:  # noqa: BLE001 - diagnostics only
                    pass
            out_runs.append({"cold_start_s": t1 - t0, "phases": phases, "readiness_stages": stages, "server_warmup": warm,
                             "warm_child": warm_child,
                             "controller_phases_ms": ctl_phases,
                             "gpus": (obj.get("status") or {}).get("gpus"),
                             "gpuReadiness": (obj.get("status") or {}).get("gpuReadiness")})
            _teardown(c, name, namespace, settle_s)
        try:
            recon = _reconcile_latency(cl.url)
        except Exception as e:  # noqa: BLE001 - reported, never fatal
            recon = {"error": f"{type(e).__name__}: {e}"}
    xs = [r["cold_start_s"] for r in out_runs]
    phase_keys = sorted({k for r in out_runs for k in r["phases"]})
    res = {"p50_s": _pct(xs, 0.5), "p90_s": _pct(xs, 0.9), "settle_s": settle_s, "runs": out_runs, "server": server,
           "failures": failures, "truncated": truncated, "env": env or None,
           "odh_oauth": odh_oauth, "zygote": zygote, "reconcile": recon,
           "phases_p50_s": {k: _pct([r["phases"][k] for r in out_runs if k in r["phases"]], 0.5) for k in phase_keys}}
    stage_keys = sorted({k for r in out_runs for k, v in r["readiness_stages"].items() if v is not None})
    if stage_keys:
        res["readiness_stages_p50_ms"] = {k: _pct([r["readiness_stages"][k] for r in out_runs
                                                    if r["readiness_stages"].get(k) is not None], 0.5) for k in stage_keys}
    wk = sorted({k for r in out_runs for k, v in (r.get("server_warmup") or {}).items() if isinstance(v, (int, float))
                 and not isinstance(v, bool)})
    if wk:
        res["server_warmup_p50_ms"] = {k: _pct([r["server_warmup"][k] for r in out_runs if (r.get("server_warmup") or {}).get(k)
                                                is not None], 0.5) for k in wk if k.endswith("_ms")}
    if zygote:
        res["warm_children"] = sum(1 for r in out_runs if r.get("warm_child"))
    rd = [r["gpuReadiness"] for r in out_runs if r.get("gpuReadiness")]
    if rd:
        res["readiness"] = rd[-1]
    return res


def measure_control_plane(runs: int = 5, gpus: int | None = None, timeout: float = 30.0) -> dict:
    """BASELINE configs 3 and 5 on the same native control plane (process pods), p50 over ``runs``:

    * profile_ready_s: Profile CREATE (owner + ``amd.com/gpu`` / HBM quota) -> namespace, owner
      RoleBinding, editor/viewer ServiceAccounts, AuthorizationPolicy and ResourceQuota all present.
    * tensorboard_ready_s: Tensorboard CREATE (pvc:// logspath) -> ``status.readyReplicas == 1``.
    * pvcviewer_ready_s: PVCViewer CREATE on the same PVC -> ``status.ready``.
    """
    def p50(xs):
        return _pct(xs, 0.5) if xs else None

    prof, tb, pv = [], [], []
    with LocalCluster(gpus=gpus) as cl:
        c = cl.client
        for i in range(runs):
            name = f"cp-{i}"
            t0 = time.time()
            c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": name},
                      "spec": {"owner": {"kind": "User", "name": f"{name}@example.com"},
                               "resourceQuotaSpec": {"hard": {"amd.com/gpu": "8", "amd.com/gpu-memory": "2304Gi"}}}})
            for av, kind, obj in [("v1", "Namespace", None), ("rbac.authorization.k8s.io/v1", "RoleBinding", "namespaceAdmin"),
                                  ("v1", "ServiceAccount", "default-editor"), ("v1", "ServiceAccount", "default-viewer"),
                                  ("security.istio.io/v1beta1", "AuthorizationPolicy", "ns-owner-access-istio"),
                                  ("v1", "ResourceQuota", "kf-resource-quota")]:
                if obj is None:
                    c.wait_for(av, kind, name, None, lambda o: True, timeout=timeout, interval=0.005)
                else:
                    c.wait_for(av, kind, obj, name, lambda o: True, timeout=timeout, interval=0.005)
            prof.append(time.time() - t0)
            c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "logs", "namespace": name},
                      "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}})
            t0 = time.time()
            c.create({"apiVersion": "tensorboard.kubeflow.org/v1alpha1", "kind": "Tensorboard",
                      "metadata": {"name": "tb", "namespace": name}, "spec": {"logspath": "pvc://logs/"}})
            c.wait_for("tensorboard.kubeflow.org/v1alpha1", "Tensorboard", "tb", name,
                       lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=timeout, interval=0.005)
            tb.append(time.time() - t0)
            t0 = time.time()
            c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PVCViewer", "metadata": {"name": "viewer", "namespace": name},
                      "spec": {"pvc": "logs", "rwoScheduling": True}})
            c.wait_for("kubeflow.org/v1alpha1", "PVCViewer", "viewer", name,
                       lambda o: (o.get("status") or {}).get("ready") is True, timeout=timeout, interval=0.005)
            pv.append(time.time() - t0)
    return {"runs": runs, "profile_ready_p50_s": p50(prof), "tensorboard_ready_p50_s": p50(tb),
            "pvcviewer_ready_p50_s": p50(pv), "note": "process pods (no container runtime)"}


def measure_gpu_notebook_configs(gpus_per_notebook: int = 1, gpus: int | None = None, timeout: float = 120.0,
                                 namespace: str = "bench-cfg") -> dict:
    """BASELINE configs 4 and 5 exactly as stated, on ONE notebook that requests every GPU:

    * config 4 — "Notebook CR requesting 8 GPUs: RCCL all-reduce smoke over xGMI inside the pod": the
      Notebook carries ``kfamd.io/gpu-readiness-args: --rccl`` (``--rccl-single`` when it has one GPU),
      so the pod's readiness op builds an RCCL communicator over the pod's devices and sweeps an
      all-reduce 8 B - 64 MiB before the pod is Ready. Reported: Ready time, ``comm_init_ms``, busbw at
      the largest size, correctness, and the devices the device plugin allocated.
    * config 5 — "TensorBoard + PVCViewer attached to the 8-GPU notebook": a Tensorboard
      (``pvc://<nb>-workspace/logs``) and a PVCViewer on that notebook's ReadWriteOnce workspace PVC
      (the JWA's ``{notebook-name}-workspace``), both co-scheduled onto the notebook's node through the
      RWO affinity (tensorboard_controller.go:207-231 with RWO_PVC_SCHEDULING, pvcviewer_controller.go:372-445).
      Reported: their Ready times and the node affinity they got.
    """
    name = "cfg-nb"
    pvc = f"{name}-workspace"
    out: dict = {"gpus_per_notebook": gpus_per_notebook}
    with LocalCluster(gpus=gpus, env={"RWO_PVC_SCHEDULING": "true"}) as cl:
        c = cl.client
        c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": namespace}})
        c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": pvc, "namespace": namespace},
                  "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "10Gi"}}}})
        rccl = "--rccl-single" if gpus_per_notebook == 1 else "--rccl"
        ctr = {"name": name, "image": "kfamd/jupyter-pytorch-rocm:latest",
               "resources": {"limits": {"amd.com/gpu": str(gpus_per_notebook)}},
               "volumeMounts": [{"name": "workspace", "mountPath": "/home/jovyan"}]}
        nb = {"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
              "metadata": {"name": name, "namespace": namespace, "annotations": {"kfamd.io/gpu-readiness-args": rccl}},
              "spec": {"template": {"spec": {"containers": [ctr],
                                             "volumes": [{"name": "workspace", "persistentVolumeClaim": {"claimName": pvc}}]}}}}
        t0 = time.time()
        c.create(nb)
        obj = _wait_ready(c, name, namespace, timeout)
        out["config4_ready_s"] = time.time() - t0
        st = obj.get("status") or {}
        rep = st.get("gpuReadiness") or {}
        ar = rep.get("allreduce") or {}
        sweep = ar.get("sweep") or []
        ids = str(st.get("gpus") or "")
        out.update({"config4_readiness_args": rccl, "config4_gpu_ids": ids, "config4_gpus": len([i for i in ids.split(",") if i]),
                    "config4_readiness_ok": rep.get("ok"),
                    "config4_rccl_devices": ar.get("devices"), "config4_rccl_comm_init_ms": ar.get("comm_init_ms"),
                    "config4_rccl_correct": ar.get("correct"), "config4_rccl_load_ms": rep.get("rccl_load_ms"),
                    "config4_rccl_busbw_GBps": sweep[-1].get("busbw_GBps") if sweep else None,
                    "config4_rccl_algbw_GBps": sweep[-1].get("algbw_GBps") if sweep else None,
                    "config4_rccl_bytes": sweep[-1].get("bytes") if sweep else None,
                    "config4_rccl_sweep": [{k: s.get(k) for k in ("bytes", "us", "algbw_GBps", "busbw_GBps")} for s in sweep]})
        pod = c.get("v1", "Pod", f"{name}-0", namespace)
        node = (pod.get("spec") or {}).get("nodeName")
        t0 = time.time()
        c.create({"apiVersion": "tensorboard.kubeflow.org/v1alpha1", "kind": "Tensorboard",
                  "metadata": {"name": "tb", "namespace": namespace}, "spec": {"logspath": f"pvc://{pvc}/logs"}})
        c.wait_for("tensorboard.kubeflow.org/v1alpha1", "Tensorboard", "tb", namespace,
                   lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=timeout, interval=0.005)
        out["config5_tensorboard_ready_s"] = time.time() - t0
        t0 = time.time()
        c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PVCViewer", "metadata": {"name": "viewer", "namespace": namespace},
                  "spec": {"pvc": pvc, "rwoScheduling": True}})
        c.wait_for("kubeflow.org/v1alpha1", "PVCViewer", "viewer", namespace,
                   lambda o: (o.get("status") or {}).get("ready") is True, timeout=timeout, interval=0.005)
        out["config5_pvcviewer_ready_s"] = time.time() - t0

        def affinity_nodes(kind_path, dep_name):
            dep = c.get("apps/v1", "Deployment", dep_name, namespace)
            aff = (((dep["spec"]["template"]["spec"].get("affinity") or {}).get("nodeAffinity") or {})
                   .get("preferredDuringSchedulingIgnoredDuringExecution") or [])
            vals = [v for t in aff for e in (t.get("preference") or {}).get("matchExpressions") or [] for v in e.get("values") or []]
            pods = c.list("v1", "Pod", namespace, label_selector=kind_path)["items"]
            return vals, sorted({(p.get("spec") or {}).get("nodeName") for p in pods})

        tb_aff, tb_nodes = affinity_nodes("app=tb", "tb")
        pv_aff, pv_nodes = affinity_nodes("app.kubernetes.io/instance=pvcviewer-viewer", "pvcviewer-viewer")
        out.update({"config5_notebook_node": node, "config5_pvc": pvc,
                    "config5_tensorboard_affinity_nodes": tb_aff, "config5_tensorboard_pod_nodes": tb_nodes,
                    "config5_pvcviewer_affinity_nodes": pv_aff, "config5_pvcviewer_pod_nodes": pv_nodes,
                    "config5_coscheduled": bool(tb_aff == [node] and pv_aff == [node] and tb_nodes == [node] and pv_nodes == [node])})
    return out


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--runs", type=int, default=5)
    p.add_argument("--gpus-per-notebook", type=int, default=1)
    p.add_argument("--gpus", type=int, default=None, help="node GPUs (default: discover; -> synthetic 8 without /dev/kfd)")
    p.add_argument("--no-readiness", action="store_true")
    p.add_argument("--settle", type=float, default=0.5, help="seconds between runs (0: back to back)")
    p.add_argument("--odh-oauth", action="store_true", help="ODH spawn path with the OAuth proxy (CS1)")
    p.add_argument("--zygote", action="store_true", help="kubelet --pod-zygote (pre-imported interpreter)")
    p.add_argument("--server", choices=sorted(SERVERS), default="stub",
                   help="notebook server recipe: stub (no torch) or torch-ready (torch import + GEMM before Ready)")
    p.add_argument("--env", action="append", default=[], metavar="K=V", help="extra notebook container env (repeatable)")
    p.add_argument("--timeout", type=float, default=120.0, help="per-run Ready deadline, seconds")
    p.add_argument("--max-failures", type=int, default=2)
    a = p.parse_args()
    env = dict(kv.split("=", 1) for kv in a.env) or None
    r = measure_cold_start(runs=a.runs, gpus_per_notebook=a.gpus_per_notebook, gpus=a.gpus, readiness=not a.no_readiness,
                           settle_s=a.settle, server=a.server, odh_oauth=a.odh_oauth, zygote=a.zygote, env=env,
                           timeout=a.timeout, max_failures=a.max_failures)
    print(json.dumps({k: v for k, v in r.items() if k not in ("runs", "failures")}))
    for f in r["failures"]:
        print(json.dumps({"failure": f}))
    if r["runs"]:
        print(json.dumps({"median_run": statistics.median(x["cold_start_s"] for x in r["runs"])}))
    for x in r["runs"]:
        print(json.dumps({"run_s": round(x["cold_start_s"], 4), "server_warmup": x.get("server_warmup")}))
    return 1 if r["failures"] else 0


if __name__ == "__main__":
    raise SystemExit(main())
