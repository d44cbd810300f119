"""Notebook-controller load test (parity with the reference's
``components/notebook-controller/loadtest/start_notebooks.py:50-96`` + ``jupyter_test.yaml`` /
``jupyter_pvc.yaml``), extended with the measurements the reference never took.

Reference mode (against a running API server, ``--server`` or ``$KFAMD_API_URL``)::

    python -m kubeflow_rm_amd.loadtest -l 3 -n kubeflow            # apply N Notebook + PVC pairs
    python -m kubeflow_rm_amd.loadtest -l 3 -n kubeflow -p delete  # delete them

Same objects as the reference: Notebook ``jupyter-test-<i>`` (container ``notebook-<i>``,
500m CPU / 1Gi, workspace PVC ``test-vol-<i>`` at /home/jovyan, a Memory emptyDir at /dev/shm,
serviceAccountName default-editor) and PVC ``test-vol-<i>`` (RWO, 2Gi).

Measure mode (BASELINE.md §3 "controller reconcile latency p50/p99" and cold start under load)::

    python -m kubeflow_rm_amd.loadtest --measure -l 50 [--gpus-per-notebook 0] [--concurrency 16]

starts an embedded ``kflite`` control plane, applies N pairs with ``--concurrency`` client threads,
waits until every Notebook reports ``status.readyReplicas == 1`` and then scrapes ``/metrics``:

* ``controller_runtime_reconcile_time_seconds{controller}``  reconcile duration,
* ``workqueue_queue_duration_seconds{name}``                  watch event -> worker pick-up,

reporting p50/p99 (bucket interpolation, as PromQL ``histogram_quantile``), counts, and the
per-notebook create -> Ready distribution. GPU notebooks (``--gpus-per-notebook k``) go through the
xGMI-aware allocator; with no ``/dev/kfd`` the node advertises a synthetic 8x MI355X.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import copy
import json
import math
import re
import sys
import time
import urllib.request

from .client import ApiException, KubeClient

NOTEBOOK_TEMPLATE = {
    "apiVersion": "kubeflow.org/v1",
    "kind": "Notebook",
    "metadata": {"name": "jupyter-test"},
    "spec": {"template": {"spec": {
        "serviceAccountName": "default-editor",
        "volumes": [{"name": "test-vol", "persistentVolumeClaim": {"claimName": "test-pvc"}},
                    {"name": "dshm", "emptyDir": {"medium": "Memory"}}],
        "containers": [{
            "image": "jupyter-scipy:latest",
            "name": "notebook",
            "resources": {"requests": {"cpu": "500m", "memory": "1Gi"}},
            "volumeMounts": [{"mountPath": "/home/jovyan", "name": "test-vol"},
                             {"mountPath": "/dev/shm", "name": "dshm"}],
        }],
    }}},
}

PVC_TEMPLATE = {
    "apiVersion": "v1",
    "kind": "PersistentVolumeClaim",
    "metadata": {"name": "test-pvc"},
    "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "2Gi"}}},
}


def notebook_config(num: int, namespace: str, image: str | None = None, gpus: int = 0,
                    command: list[str] | None = None) -> dict:
    """start_notebooks.py write_notebook_config: name jupyter-test-<n>, container notebook-<n>,
    claim test-vol-<n>."""
    nb = copy.deepcopy(NOTEBOOK_TEMPLATE)
    nb["metadata"]["name"] = f"jupyter-test-{num}"
    nb["metadata"]["namespace"] = namespace
    spec = nb["spec"]["template"]["spec"]
    c = spec["containers"][0]
    c["name"] = f"notebook-{num}"
    if image:
        c["image"] = image
    if gpus:
        c["resources"]["limits"] = {"amd.com/gpu": str(gpus)}
    if command:
        c["command"] = list(command)
    spec["volumes"][0]["persistentVolumeClaim"]["claimName"] = f"test-vol-{num}"
    return nb


def pvc_config(num: int, namespace: str) -> dict:
    pvc = copy.deepcopy(PVC_TEMPLATE)
    pvc["metadata"]["name"] = f"test-vol-{num}"
    pvc["metadata"]["namespace"] = namespace
    return pvc


def apply_pair(client: KubeClient, num: int, namespace: str, image: str | None = None, gpus: int = 0,
               command: list[str] | None = None) -> float:
    """Apply the PVC then the Notebook (the reference applies the Notebook first; the PVC-first
    order avoids a pod briefly pending on a missing claim, which is not what we time). Returns the
    client-side timestamp of the Notebook CREATE."""
    client.apply(pvc_config(num, namespace))
    t0 = time.time()
    client.apply(notebook_config(num, namespace, image, gpus, command))
    return t0


def delete_pair(client: KubeClient, num: int, namespace: str) -> None:
    for av, kind, name in (("kubeflow.org/v1", "Notebook", f"jupyter-test-{num}"),
                           ("v1", "PersistentVolumeClaim", f"test-vol-{num}")):
        try:
            client.delete(av, kind, name, namespace)
        except ApiException as e:
            if e.status != 404:
                raise


# ---- Prometheus text parsing -------------------------------------------------------------------
_SAMPLE = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{[^}]*\})?\s+(\S+)')
_LABEL = re.compile(r'(\w+)="((?:[^"\\]|\\.)*)"')


def parse_histograms(text: str, name: str) -> dict[tuple, dict]:
    """{labels-without-le: {"buckets": [(le, cumulative)], "sum": s, "count": n}} for one family."""
    out: dict[tuple, dict] = {}
    for line in text.splitlines():
        m = _SAMPLE.match(line)
        if not m or not m.group(1).startswith(name):
            continue
        metric, lbl, val = m.group(1), m.group(2) or "", float(m.group(3))
        labels = dict(_LABEL.findall(lbl))
        le = labels.pop("le", None)
        key = tuple(sorted(labels.items()))
        h = out.setdefault(key, {"buckets": [], "sum": 0.0, "count": 0})
        if metric == name + "_bucket" and le is not None:
            h["buckets"].append((math.inf if le == "+Inf" else float(le), val))
        elif metric == name + "_sum":
            h["sum"] = val
        elif metric == name + "_count":
            h["count"] = int(val)
    for h in out.values():
        h["buckets"].sort()
    return out


def histogram_quantile(q: float, buckets: list[tuple[float, float]]) -> float:
    """PromQL histogram_quantile: linear interpolation inside the bucket holding rank q*count."""
    if not buckets or buckets[-1][1] == 0:
        return float("nan")
    total = buckets[-1][1]
    rank = q * total
    prev_le, prev_c = 0.0, 0.0
    for le, c in buckets:
        if c >= rank:
            if math.isinf(le):
                return prev_le
            if c == prev_c:
                return le
            return prev_le + (le - prev_le) * (rank - prev_c) / (c - prev_c)
        prev_le, prev_c = le, c
    return prev_le


def summarize(text: str) -> dict:
    res: dict = {}
    for fam, lab in (("controller_runtime_reconcile_time_seconds", "controller"),
                     ("workqueue_queue_duration_seconds", "name"),
                     ("apiserver_request_duration_seconds", None)):
        for key, h in parse_histograms(text, fam).items():
            who = dict(key).get(lab, "?") if lab else " ".join(v for _, v in key)
            if not h["count"]:
                continue
            res.setdefault(fam, {})[who] = {
                "count": h["count"],
                "mean_ms": 1e3 * h["sum"] / h["count"],
                "p50_ms": 1e3 * histogram_quantile(0.5, h["buckets"]),
                "p99_ms": 1e3 * histogram_quantile(0.99, h["buckets"]),
            }
    return res


def _pct(xs: list[float], q: float) -> float:
    xs = sorted(xs)
    if not xs:
        return float("nan")
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def measure(n: int = 20, namespace: str = "loadtest", concurrency: int = 8, gpus_per_notebook: int = 0,
            image: str | None = None, timeout: float = 180.0, workers: int = 1, node_gpus: int | None = 8,
            command: list[str] | None = None) -> dict:
    """Embedded control plane + N notebook/PVC pairs; returns latency percentiles (see module doc).

    ``command`` overrides the container command (e.g. ``["sleep", "infinity"]``): every pod is then a
    bare process, so on a small host the numbers measure the control plane rather than N Python
    notebook servers competing for the CPUs while they start."""
    from .cluster import LocalCluster

    args = ["--workers", str(workers)] if workers != 1 else []
    # every pair requests 500m CPU (jupyter_test.yaml); advertise a node that fits all of them so
    # the test measures the control plane, not an Insufficient-cpu Pending queue
    args += ["--node-cpus", str(max(8, (n + 1) // 2 + 1)), "--node-memory-gib", str(max(64, n + 8))]
    with LocalCluster(env={"ENABLE_CULLING": "false"}, args=args, gpus=node_gpus) as cl:
        c0 = cl.client
        c0.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": namespace}})
        if image is None and gpus_per_notebook == 0:
            image = "jupyter-scipy:latest"
        t_start = time.time()
        created: dict[int, float] = {}

        def one(i: int) -> tuple[int, float]:
            return i, apply_pair(KubeClient(cl.url), i, namespace, image, gpus_per_notebook, command)

        with cf.ThreadPoolExecutor(max_workers=concurrency) as ex:
            for i, t0 in ex.map(one, range(n)):
                created[i] = t0
        t_applied = time.time()
        ready: dict[int, float] = {}
        deadline = time.time() + timeout
        while len(ready) < n and time.time() < deadline:
            items = c0.list("kubeflow.org/v1", "Notebook", namespace)["items"]
            now = time.time()
            for it in items:
                num = int(it["metadata"]["name"].rsplit("-", 1)[1])
                if num not in ready and (it.get("status") or {}).get("readyReplicas") == 1:
                    ready[num] = now
            time.sleep(0.01)
        with urllib.request.urlopen(cl.url + "/metrics", timeout=10) as r:
            metrics_text = r.read().decode()
        lat = [ready[i] - created[i] for i in ready]
        res = {
            "notebooks": n, "ready": len(ready), "concurrency": concurrency, "workers_per_controller": workers,
            "gpus_per_notebook": gpus_per_notebook, "pod_process": " ".join(command) if command else "image recipe",
            "apply_wall_s": t_applied - t_start,
            "all_ready_wall_s": (max(ready.values()) - t_start) if ready else None,
            "create_to_ready_p50_s": _pct(lat, 0.5), "create_to_ready_p90_s": _pct(lat, 0.9),
            "create_to_ready_p99_s": _pct(lat, 0.99), "create_to_ready_max_s": max(lat) if lat else None,
            "metrics": summarize(metrics_text),
        }
        return res


def main(argv: list[str] | None = None) -> int:
    p = argparse.ArgumentParser(description="Load test the notebook controller (start_notebooks.py parity)")
    p.add_argument("-l", "--load", dest="num_notebooks", type=int, default=3,
                   help="Number of notebooks to start the load test. (Default: %(default)s)")
    p.add_argument("-n", "--namespace", default=None, help="Namespace (default: kubeflow; loadtest with --measure)")
    p.add_argument("-p", "--operation", default="apply", choices=["apply", "delete"])
    p.add_argument("--server", default=None, help="API server URL (default $KFAMD_API_URL)")
    p.add_argument("--image", default=None)
    p.add_argument("--gpus-per-notebook", type=int, default=0)
    p.add_argument("--measure", action="store_true", help="embedded control plane + latency report (JSON)")
    p.add_argument("--concurrency", type=int, default=8)
    p.add_argument("--workers", type=int, default=1, help="reconcile workers per controller (--measure)")
    p.add_argument("--node-gpus", type=int, default=8, help="node GPUs for --measure (0 = discover)")
    p.add_argument("--timeout", type=float, default=180.0)
    p.add_argument("--command", default=None, help="container command override, e.g. 'sleep infinity'")
    a = p.parse_args(argv)
    if a.measure:
        res = measure(a.num_notebooks, a.namespace or "loadtest", a.concurrency, a.gpus_per_notebook, a.image,
                      a.timeout, a.workers, a.node_gpus or None, a.command.split() if a.command else None)
        print(json.dumps(res))
        return 0 if res["ready"] == res["notebooks"] else 1
    client = KubeClient(a.server)
    ns = a.namespace or "kubeflow"
    for i in range(a.num_notebooks):
        if a.operation == "apply":
            print(f"apply jupyter-test-{i} + test-vol-{i} ...")
            apply_pair(client, i, ns, a.image, a.gpus_per_notebook)
        else:
            print(f"delete jupyter-test-{i} + test-vol-{i} ...")
            delete_pair(client, i, ns)
    return 0


if __name__ == "__main__":
    sys.exit(main())
