"""End-to-end control plane on kube-lite + process-pod kubelet (CPU, synthetic 8x MI355X node).

Ports the reference's envtest BDD flow (notebook_controller_bdd_test.go: CR -> StatefulSet) and
extends it through the parts envtest cannot run (no kube-controller-manager, no
kubelet): pods actually start, become Ready, get GPUs from the xGMI-aware allocator, are routed
by the ingress gateway, and are garbage collected.
"""
import json
import time
import urllib.error
import urllib.request

import pytest

from kubeflow_rm_amd.client import ApiException

NB = "kubeflow.org/v1"


def _notebook(name, ns, gpus=0, labels=None, annotations=None, image="jupyter-scipy:latest"):
    c = {"name": name, "image": image}
    if gpus:
        c["resources"] = {"limits": {"amd.com/gpu": str(gpus)}}
    return {"apiVersion": NB, "kind": "Notebook",
            "metadata": {"name": name, "namespace": ns, "labels": labels or {}, "annotations": annotations or {}},
            "spec": {"template": {"spec": {"containers": [c]}}}}


def _ready(o):
    return (o.get("status") or {}).get("readyReplicas") == 1


@pytest.fixture(scope="module")
def c(cluster):
    cl = cluster.client
    # a mesh member, like every Kubeflow profile namespace (profile_controller.go:71): the ODH
    # controller's <nb>-ctrl-np admits only its own namespace on :8888, and the member namespace's
    # mesh policy (istio-mesh) is what admits the ingress gateway
    cl.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "e2e", "labels": {"istio-injection": "enabled"}}})
    return cl


def test_notebook_to_statefulset_service_and_ready(c, cluster):
    c.create(_notebook("nb1", "e2e"))
    sts = c.wait_for("apps/v1", "StatefulSet", "nb1", "e2e", lambda o: True, timeout=10)
    ref = sts["metadata"]["ownerReferences"][0]
    assert ref["kind"] == "Notebook" and ref["name"] == "nb1" and ref["controller"] is True
    # the reconciler creates the StatefulSet, then the Service, then the VirtualService
    svc = c.wait_for("v1", "Service", "nb1", "e2e", lambda o: True, timeout=10)
    assert svc["spec"]["ports"][0]["targetPort"] == 8888
    vs = c.wait_for("networking.istio.io/v1alpha3", "VirtualService", "notebook-e2e-nb1", "e2e", lambda o: True,
                    timeout=10)
    assert vs["spec"]["http"][0]["match"][0]["uri"]["prefix"] == "/notebook/e2e/nb1/"
    nb = c.wait_for(NB, "Notebook", "nb1", "e2e", _ready, timeout=30)
    assert "running" in nb["status"]["containerState"]
    assert any(x["type"] == "Ready" for x in nb["status"]["conditions"])
    # through the ingress gateway, like the browser would (the notebook has no readiness probe, as
    # in the reference's spawner template, so Ready can precede the server listening: poll briefly)
    deadline = time.time() + 15
    while True:
        try:
            with urllib.request.urlopen(cluster.gateway + "/notebook/e2e/nb1/api/status", timeout=5) as r:
                assert r.status == 200
                assert "started" in json.loads(r.read())
                break
        except urllib.error.HTTPError as e:
            if e.code not in (404, 502, 503) or time.time() > deadline:  # route / server not up yet
                raise
            time.sleep(0.1)


def test_stop_and_restart_notebook(c):
    nb = c.wait_for(NB, "Notebook", "nb1", "e2e", _ready, timeout=30)
    c.patch(NB, "Notebook", "nb1", {"metadata": {"annotations": {"kubeflow-resource-stopped": "2024-01-01T00:00:00Z"}}}, "e2e")
    c.wait_for("apps/v1", "StatefulSet", "nb1", "e2e", lambda o: o["spec"]["replicas"] == 0, timeout=10)
    c.wait_gone("v1", "Pod", "nb1-0", "e2e", timeout=30)
    c.patch(NB, "Notebook", "nb1", {"metadata": {"annotations": {"kubeflow-resource-stopped": None}}}, "e2e")
    c.wait_for(NB, "Notebook", "nb1", "e2e", _ready, timeout=30)
    del nb


def test_pod_events_are_reemitted_on_the_notebook(c):
    def has_event(_):
        evs = c.list("v1", "Event", "e2e", field_selector="involvedObject.kind=Notebook")["items"]
        return any(e["involvedObject"]["name"] == "nb1" for e in evs)
    c.wait_for(NB, "Notebook", "nb1", "e2e", has_event, timeout=15)


def test_gpu_notebook_gets_xgmi_placement(c):
    c.create(_notebook("gpu4", "e2e", gpus=4))
    nb = c.wait_for(NB, "Notebook", "gpu4", "e2e", _ready, timeout=30)
    pod = c.get("v1", "Pod", "gpu4-0", "e2e")
    ids = pod["metadata"]["annotations"]["amd.com/gpu-ids"].split(",")
    assert len(ids) == 4 and len(set(ids)) == 4
    assert nb["status"]["gpus"] == pod["metadata"]["annotations"]["amd.com/gpu-ids"]
    # the readiness op ran as an init container and its report is on the Notebook
    assert nb["status"]["gpuReadiness"]["ok"] is True
    env = c.pod_logs("gpu4-0", "e2e")
    assert env is not None


def test_gpu_allocation_metrics(c, cluster):
    """kubelet GPU metrics: which pod holds which MI355X, HBM allocated per namespace."""
    pod = c.get("v1", "Pod", "gpu4-0", "e2e")
    ids = set(pod["metadata"]["annotations"]["amd.com/gpu-ids"].split(","))
    with urllib.request.urlopen(cluster.url + "/metrics", timeout=5) as r:
        text = r.read().decode()
    held = {line.split('gpu="')[1].split('"')[0] for line in text.splitlines()
            if line.startswith("kfamd_gpu_allocated{") and 'pod="gpu4-0"' in line and 'namespace="e2e"' in line}
    assert held == ids
    hbm = [float(line.split()[-1]) for line in text.splitlines()
           if line.startswith('kfamd_gpu_hbm_allocated_bytes{namespace="e2e"}')]
    assert hbm and hbm[0] >= 4 * 288 * 2**30


def test_gpu_readiness_sidecar_overlaps_server_start(c):
    """The readiness op runs as a native sidecar: the notebook container is started while the op is
    still running (Initialized does not wait for it), the sidecar stays running after its verdict,
    its /readyz gates the pod's Ready, and its report reaches the Notebook status."""
    c.create(_notebook("sc1", "e2e", gpus=1, annotations={"kfamd.io/gpu-readiness-args": "--iters 3"}))
    nb = c.wait_for(NB, "Notebook", "sc1", "e2e", _ready, timeout=30)
    assert nb["status"]["gpuReadiness"]["ok"] is True
    pod = c.get("v1", "Pod", "sc1-0", "e2e")
    side = pod["status"]["initContainerStatuses"][0]
    assert side["name"] == "gpu-readiness" and "running" in side["state"] and side["ready"] is True
    assert side["restartCount"] == 0
    main = pod["status"]["containerStatuses"][0]
    # the server was started before the op's verdict (no serial init wait)
    assert main["state"]["running"]["startedAt"] <= pod["metadata"]["annotations"].get(
        "notebooks.kubeflow.org/gpu-readiness-at", "9999")
    c.delete(NB, "Notebook", "sc1", "e2e")


def test_gpu_readiness_failure_surfaces_on_notebook(c):
    """a GPU-side fault in the readiness op -> pod not Ready -> the Notebook status
    carries the op's error (fault injected through kfamd.io/gpu-readiness-args)."""
    c.create(_notebook("faulty", "e2e", gpus=1, annotations={"kfamd.io/gpu-readiness-args": "--inject-fault gemm"}))

    def failed(o):
        g = (o.get("status") or {}).get("gpuReadiness") or {}
        return g.get("ok") is False
    nb = c.wait_for(NB, "Notebook", "faulty", "e2e", failed, timeout=30)
    assert "injected fault at stage gemm" in nb["status"]["gpuReadiness"]["error"]
    assert not (nb["status"] or {}).get("readyReplicas")
    pod = c.get("v1", "Pod", "faulty-0", "e2e")
    ready = [x for x in pod["status"]["conditions"] if x["type"] == "Ready"][0]
    assert ready["status"] == "False"
    c.delete(NB, "Notebook", "faulty", "e2e")


def test_gpu_oversubscription_is_unschedulable(c):
    c.create(_notebook("gpu16", "e2e", gpus=16))

    def unsched(o):
        return any(x.get("reason") == "Unschedulable" for x in (o.get("status") or {}).get("conditions", []))
    nb = c.wait_for(NB, "Notebook", "gpu16", "e2e", unsched, timeout=15)
    msg = [x for x in nb["status"]["conditions"] if x.get("reason") == "Unschedulable"][0]["message"]
    assert "amd.com/gpu" in msg
    c.delete(NB, "Notebook", "gpu16", "e2e")


def test_delete_notebook_garbage_collects(c):
    c.delete(NB, "Notebook", "gpu4", "e2e")
    c.wait_gone("apps/v1", "StatefulSet", "gpu4", "e2e", timeout=15)
    c.wait_gone("v1", "Pod", "gpu4-0", "e2e", timeout=30)
    c.wait_gone("v1", "Service", "gpu4", "e2e", timeout=15)


def test_profile_lifecycle_with_gpu_quota_and_poddefaults(c):
    c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": "alice"},
              "spec": {"owner": {"kind": "User", "name": "alice@example.com"},
                       "resourceQuotaSpec": {"hard": {"amd.com/gpu": "2"}}}})
    ns = c.wait_for("v1", "Namespace", "alice", None, lambda o: True, timeout=10)
    assert ns["metadata"]["annotations"]["owner"] == "alice@example.com"
    assert ns["metadata"]["labels"]["app.kubernetes.io/part-of"] == "kubeflow-profile"
    for av, kind, name in [("security.istio.io/v1beta1", "AuthorizationPolicy", "ns-owner-access-istio"),
                           ("v1", "ServiceAccount", "default-editor"), ("v1", "ServiceAccount", "default-viewer"),
                           ("rbac.authorization.k8s.io/v1", "RoleBinding", "namespaceAdmin"),
                           ("rbac.authorization.k8s.io/v1", "RoleBinding", "default-editor"),
                           ("v1", "ResourceQuota", "kf-resource-quota")]:
        c.wait_for(av, kind, name, "alice", lambda o: True, timeout=10)
    # owner can now create notebooks in the namespace (RBAC via namespaceAdmin -> kubeflow-admin)
    r = c.subject_access_review("alice@example.com", "create", "kubeflow.org", "notebooks", "alice")
    assert r["status"]["allowed"] is True
    # PodDefault injection (webhook gated on the profile namespace label)
    c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PodDefault", "metadata": {"name": "add-env", "namespace": "alice"},
              "spec": {"selector": {"matchLabels": {"add-env": "true"}}, "desc": "env",
                       "env": [{"name": "FOO", "value": "bar"}]}})
    c.create(_notebook("nb", "alice", gpus=2, labels={"add-env": "true"}))
    c.wait_for(NB, "Notebook", "nb", "alice", _ready, timeout=30)
    pod = c.get("v1", "Pod", "nb-0", "alice")
    assert {"name": "FOO", "value": "bar"} in pod["spec"]["containers"][0]["env"]
    assert "poddefault.admission.kubeflow.org/poddefault-add-env" in pod["metadata"]["annotations"]
    q = c.wait_for("v1", "ResourceQuota", "kf-resource-quota", "alice",
                   lambda o: (o.get("status") or {}).get("used", {}).get("amd.com/gpu") == "2", timeout=10)
    assert q["status"]["hard"]["amd.com/gpu"] == "2"
    # the quota is full: a third GPU is rejected at admission (surfaced as a StatefulSet event / no pod)
    with pytest.raises(ApiException) as e:
        c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "extra", "namespace": "alice"},
                  "spec": {"containers": [{"name": "x", "image": "x", "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
    assert e.value.status == 403 and "exceeded quota" in str(e.value.body)
    # deletion: finalizer released, namespace + children garbage collected
    c.delete("kubeflow.org/v1", "Profile", "alice")
    c.wait_gone("kubeflow.org/v1", "Profile", "alice", None, timeout=15)
    c.wait_gone("v1", "Namespace", "alice", None, timeout=30)


def test_profile_rejects_foreign_namespace(c):
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "taken", "annotations": {"owner": "bob@example.com"}}})
    c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": "taken"},
              "spec": {"owner": {"kind": "User", "name": "eve@example.com"}}})
    p = c.wait_for("kubeflow.org/v1", "Profile", "taken", None,
                   lambda o: any(x["type"] == "Failed" for x in (o.get("status") or {}).get("conditions", [])), timeout=10)
    assert "not owned by profile creator" in p["status"]["conditions"][0]["message"]
    assert not c.exists("rbac.authorization.k8s.io/v1", "RoleBinding", "namespaceAdmin", "taken")


@pytest.mark.parametrize("hard_key,hard,per_pod,admitted", [
    ("amd.com/gpu", "2", {"amd.com/gpu": "1"}, 2),
    # HBM quota in GiB: 3 x 288 GiB fits in 900, the 4th does not
    ("amd.com/gpu-memory", "900", {"amd.com/gpu": "1"}, 3),
])
def test_concurrent_pod_creates_never_overcommit_quota(c, cluster, hard_key, hard, per_pod, admitted):
    """K7: 16 concurrent 1-GPU pod creates against one ResourceQuota admit exactly the quota
    (admission reserves under a per-namespace lock until the pod is in the store). Every create
    sleeps 50 ms between admission and commit (``commitdelay`` fault), so without the reservation
    all 16 would pass the check against the same committed pods."""
    import concurrent.futures as cf
    ns = "qrace-" + hard_key.replace("amd.com/", "").replace("-", "")
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    c.create({"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q", "namespace": ns},
              "spec": {"hard": {hard_key: hard}}})

    def create(i):
        pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{i}", "namespace": ns},
               # unschedulable on purpose: the pods stay Pending (and keep counting against the quota)
               "spec": {"nodeSelector": {"kfamd.io/no-such-node": "true"},
                        "containers": [{"name": "x", "image": "x", "resources": {"limits": dict(per_pod)}}]}}
        try:
            c.create(pod)
            return True
        except ApiException as e:
            assert e.status == 403 and "exceeded quota" in str(e.body), (e.status, e.body)
            return False

    req = urllib.request.Request(cluster.url + "/debug/faults", data=json.dumps({"spec": "commitdelay:pods:24:50"}).encode(),
                                 method="POST", headers={"Content-Type": "application/json"})
    urllib.request.urlopen(req, timeout=5).close()
    try:
        with cf.ThreadPoolExecutor(16) as ex:
            results = list(ex.map(create, range(16)))
    finally:
        urllib.request.urlopen(urllib.request.Request(cluster.url + "/debug/faults", method="DELETE"), timeout=5).close()
    assert sum(results) == admitted, results
    assert len(c.list("v1", "Pod", ns)["items"]) == admitted
    # a rejected-then-freed slot: deleting one admitted pod lets exactly one more in
    victim = c.list("v1", "Pod", ns)["items"][0]["metadata"]["name"]
    c.delete("v1", "Pod", victim, ns)
    c.wait_gone("v1", "Pod", victim, ns, timeout=15)
    with cf.ThreadPoolExecutor(8) as ex:
        results = list(ex.map(create, range(100, 108)))
    assert sum(results) == 1, results


def _ws_client_frame(payload: bytes, op: int = 1) -> bytes:
    import os as _os
    import struct
    mask = _os.urandom(4)
    n = len(payload)
    head = struct.pack(">BB", 0x80 | op, 0x80 | n) if n < 126 else struct.pack(">BBH", 0x80 | op, 0x80 | 126, n)
    return head + mask + bytes(b ^ mask[i & 3] for i, b in enumerate(payload))


def _ws_read(sock_file):
    import struct
    h = sock_file.read(2)
    op, n = h[0] & 0x0F, h[1] & 0x7F
    if n == 126:
        n = struct.unpack(">H", sock_file.read(2))[0]
    elif n == 127:
        n = struct.unpack(">Q", sock_file.read(8))[0]
    return op, sock_file.read(n)


def test_gateway_tunnels_kernel_websocket_and_streams_events(c, cluster):
    """JupyterLab's kernel channel WebSocket through the notebook's
    VirtualService route (notebook_controller.go:519-619), and a streamed (chunked) response
    relayed as it is produced instead of buffered."""
    import base64
    import hashlib
    import os as _os
    import socket
    import urllib.parse
    c.create(_notebook("ws1", "e2e"))
    c.wait_for(NB, "Notebook", "ws1", "e2e", _ready, timeout=30)
    base = cluster.gateway + "/notebook/e2e/ws1"
    deadline = time.time() + 15
    while True:
        try:
            req = urllib.request.Request(base + "/api/kernels", data=b'{"name": "python3"}', method="POST",
                                         headers={"Content-Type": "application/json"})
            with urllib.request.urlopen(req, timeout=5) as r:
                kid = json.loads(r.read())["id"]
            break
        except (urllib.error.URLError, ConnectionError):
            if time.time() > deadline:
                raise
            time.sleep(0.2)
    gw = urllib.parse.urlparse(cluster.gateway)
    key = base64.b64encode(_os.urandom(16)).decode()
    s = socket.create_connection((gw.hostname, gw.port), timeout=10)
    try:
        s.sendall((f"GET /notebook/e2e/ws1/api/kernels/{kid}/channels?session_id=abc HTTP/1.1\r\n"
                   f"Host: {gw.hostname}:{gw.port}\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                   f"Sec-WebSocket-Key: {key}\r\nSec-WebSocket-Version: 13\r\n\r\n").encode())
        f = s.makefile("rb")
        status = f.readline()
        assert b" 101 " in status, status
        headers = {}
        while True:
            line = f.readline().strip()
            if not line:
                break
            k, v = line.decode().split(":", 1)
            headers[k.strip().lower()] = v.strip()
        want = base64.b64encode(hashlib.sha1((key + "258EAFA5-E914-47DA-95CA-C5AB0DC85B11").encode()).digest()).decode()
        assert headers["sec-websocket-accept"] == want
        # the open channel is visible to the culler as a connection
        with urllib.request.urlopen(base + f"/api/kernels/{kid}", timeout=5) as r:
            assert json.loads(r.read())["connections"] == 1
        msg = {"header": {"msg_id": "m1", "msg_type": "execute_request", "session": "abc", "version": "5.3"},
               "parent_header": {}, "metadata": {}, "channel": "shell",
               "content": {"code": "print(355)", "silent": False}}
        s.sendall(_ws_client_frame(json.dumps(msg).encode()))
        seen = []
        while "execute_reply" not in seen:
            op, data = _ws_read(f)
            assert op == 1
            m = json.loads(data)
            assert m["parent_header"]["msg_id"] == "m1"
            seen.append(m["header"]["msg_type"])
            if m["header"]["msg_type"] == "stream":
                assert m["content"]["text"] == "print(355)"
        assert seen[:3] == ["status", "execute_input", "stream"]
        s.sendall(_ws_client_frame(b"", op=8))
        ops = []
        while not ops or ops[-1] != 8:
            op, data = _ws_read(f)
            ops.append(op)
            if op == 1:  # the trailing idle status
                assert json.loads(data)["content"] == {"execution_state": "idle"}
        assert ops[-1] == 8
    finally:
        s.close()
    # streamed response: 6 events 250 ms apart; the first must arrive long before the last
    t0 = time.time()
    with urllib.request.urlopen(base + "/api/events/stream?n=6&interval_ms=250", timeout=10) as r:
        assert r.headers["Content-Type"] == "text/event-stream"
        first = r.readline()
        t_first = time.time() - t0
        rest = r.read()
    t_all = time.time() - t0
    assert first.startswith(b"id: 0") and rest.count(b"data: ") == 6
    assert t_all >= 1.2 and t_first < 0.6, (t_first, t_all)
    c.delete(NB, "Notebook", "ws1", "e2e")


def test_cold_start_phases_recorded_on_notebook_and_exported(c, cluster):
    """the first start of a Notebook is broken into phases by the controller
    (annotation notebooks.kubeflow.org/cold-start-phases + notebook_cold_start_seconds histogram)."""
    c.create(_notebook("cs1", "e2e", gpus=1))
    nb = c.wait_for(NB, "Notebook", "cs1", "e2e",
                    lambda o: "notebooks.kubeflow.org/cold-start-phases" in (o["metadata"].get("annotations") or {}),
                    timeout=30)
    ph = json.loads(nb["metadata"]["annotations"]["notebooks.kubeflow.org/cold-start-phases"])
    for k in ("observed_to_statefulset_ms", "statefulset_to_scheduled_ms", "scheduled_to_initialized_ms",
              "initialized_to_ready_ms", "total_ms"):
        assert k in ph and 0 <= ph[k] < 30000, ph
    assert ph["total_ms"] >= ph["scheduled_to_initialized_ms"]
    with urllib.request.urlopen(cluster.url + "/metrics", timeout=5) as r:
        text = r.read().decode()
    count = [ln for ln in text.splitlines() if ln.startswith('notebook_cold_start_seconds_count{phase="total"}')]
    assert count and float(count[0].split()[-1]) >= 1
    # written once: a pod restart does not rewrite it
    c.delete(NB, "Notebook", "cs1", "e2e")


def test_admission_latency_histograms(c, cluster):
    """admission latency per in-process plugin (kube-apiserver's metric names), with the
    operation, admit/validate and rejected labels; GPU pods went through placement/readiness plugins."""
    with urllib.request.urlopen(cluster.url + "/metrics", timeout=5) as r:
        text = r.read().decode()
    name = "apiserver_admission_controller_admission_duration_seconds_count"
    rows = [ln for ln in text.splitlines() if ln.startswith(name + "{")]
    assert rows, "no admission histogram"
    plugins = {ln.split('name="')[1].split('"')[0] for ln in rows}
    assert len(plugins) >= 2, plugins
    creates = [ln for ln in rows if 'operation="CREATE"' in ln and 'type="admit"' in ln and 'rejected="false"' in ln]
    assert creates and max(float(ln.split()[-1]) for ln in creates) >= 1
    assert "# TYPE apiserver_admission_controller_admission_duration_seconds histogram" in text
