"""Container probes run off the kubelet's reconcile workers.

The kubelet has 4 reconcile workers. Before the Prober (``native/node/prober.{h,cc}``) an httpGet
probe blocked a worker for up to ``timeoutSeconds`` and a not-Ready pod re-probed every 5 ms, so 8
notebooks whose servers had not started answering could hold every worker and stall every other
pod's sync on the node. Now each probe runs on a prober thread and the pod's key is re-queued when
its verdict lands; a reconcile pass only reads the verdict.

Checked here: 8 pods whose readiness endpoint accepts connections but never answers (each probe hangs
its full ``timeoutSeconds: 5``) do not delay a probe-less pod's Ready by more than 50 ms, and probes
still decide readiness (an exec probe that exits 0 / non-zero / outlives its timeout).
"""
import socket
import time

import pytest

from kubeflow_rm_amd.cluster import LocalCluster


def _ready(p):
    return any(c["type"] == "Ready" and c["status"] == "True" for c in (p.get("status") or {}).get("conditions") or [])


def _pod(name, ns, probe=None):
    c = {"name": "x", "image": "generic"}
    if probe:
        c["readinessProbe"] = probe
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": ns}, "spec": {"containers": [c]}}


@pytest.fixture(scope="module")
def cl():
    from tests.conftest import _ensure_native
    _ensure_native()
    with LocalCluster(gpus=0) as c:
        c.client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "pr"}})
        yield c


def _time_to_ready(c, name, ns="pr"):
    t0 = time.perf_counter()
    c.create(_pod(name, ns))
    c.wait_for("v1", "Pod", name, ns, _ready, timeout=30, interval=0.002)
    return time.perf_counter() - t0


def test_stalled_readiness_probes_do_not_hold_back_other_pods(cl):
    c = cl.client
    # min of 5: the test host's own load (pytest -n 8) only ever adds to a sample
    base = min(_time_to_ready(c, f"base{i}") for i in range(5))
    stall = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    stall.bind(("127.0.0.1", 0))
    stall.listen(256)  # never accept()ed: every HTTP probe connects, then waits out its timeout
    port = stall.getsockname()[1]
    try:
        probe = {"httpGet": {"host": "127.0.0.1", "port": port, "path": "/api"}, "timeoutSeconds": 5, "periodSeconds": 1}
        for i in range(8):
            c.create(_pod(f"stalled{i}", "pr", probe))
        deadline = time.time() + 30
        while True:  # all 8 running, i.e. their first probes are in flight
            pods = [c.get("v1", "Pod", f"stalled{i}", "pr") for i in range(8)]
            if all((p.get("status") or {}).get("phase") == "Running" for p in pods):
                break
            assert time.time() < deadline
            time.sleep(0.05)
        time.sleep(0.5)
        loaded = min(_time_to_ready(c, f"late{i}") for i in range(5))
        assert loaded <= base + 0.05, (base, loaded)
        assert not any(_ready(c.get("v1", "Pod", f"stalled{i}", "pr")) for i in range(8))
    finally:
        stall.close()
        for i in range(8):
            c.delete("v1", "Pod", f"stalled{i}", "pr")


def test_exec_probe_verdicts(cl):
    c = cl.client
    c.create(_pod("ok", "pr", {"exec": {"command": ["true"]}, "periodSeconds": 1}))
    c.create(_pod("bad", "pr", {"exec": {"command": ["false"]}, "periodSeconds": 1}))
    c.create(_pod("slow", "pr", {"exec": {"command": ["sleep", "30"]}, "timeoutSeconds": 1, "periodSeconds": 1}))
    c.wait_for("v1", "Pod", "ok", "pr", _ready, timeout=30)
    time.sleep(2.5)  # two rounds of the failing / timing-out probes
    assert not _ready(c.get("v1", "Pod", "bad", "pr"))
    assert not _ready(c.get("v1", "Pod", "slow", "pr"))
    # the timed-out `sleep 30` was killed and reaped, not left behind
    import subprocess
    ps = subprocess.run(["ps", "-eo", "args"], capture_output=True, text=True).stdout.splitlines()
    assert sum(1 for a in ps if a.strip() == "sleep 30") <= 1
