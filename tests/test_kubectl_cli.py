"""kfctl's kubectl subset (get / describe / wait / rollout status / logs / apply -f / delete) against
kube-lite, driven as the reference's own acceptance flow drives kubectl:

* ``.github/workflows/odh_notebook_controller_integration_test.yaml:233-289``: apply a Notebook,
  wait for its StatefulSet, ``rollout status``, ``wait --for=jsonpath='{.spec.replicas}'=1``,
  ``wait pods <nb>-0 --for=condition=Ready``, then the ``describe`` / ``logs`` dump;
* ``notebook_controller_integration_test.yaml:106``: ``wait pods -l app=... --for=condition=Ready``.
Every command runs as a subprocess of ``python -m kubeflow_rm_amd.kfctl`` (the user-facing CLI).
"""
import json
import os
import subprocess
import sys
import time

import pytest

from kubeflow_rm_amd.cluster import LocalCluster

NB_YAML = """
apiVersion: kubeflow.org/v1
kind: Notebook
metadata:
  name: minimal-notebook
  annotations:
    notebooks.opendatahub.io/inject-oauth: "false"
spec:
  template:
    spec:
      containers:
        - name: minimal-notebook
          image: quay.io/thoth-station/s2i-minimal-notebook:v0.3.0
          imagePullPolicy: Always
          workingDir: /opt/app-root/src
          env:
            - name: JUPYTER_NOTEBOOK_PORT
              value: "8888"
          ports:
            - name: notebook-port
              containerPort: 8888
              protocol: TCP
          resources:
            requests:
              cpu: "1"
              memory: 1m
            limits:
              cpu: "1"
              memory: 1Gi
          livenessProbe:
            initialDelaySeconds: 10
            periodSeconds: 5
            timeoutSeconds: 1
            successThreshold: 1
            failureThreshold: 3
            httpGet:
              scheme: HTTP
              path: /notebook/ci-ns/minimal-notebook/api
              port: notebook-port
"""


@pytest.fixture(scope="module")
def cl():
    from tests.conftest import _ensure_native
    _ensure_native()
    with LocalCluster() as c:
        c.client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "ci-ns"}})
        yield c


def kfctl(cl, *args, stdin=None, timeout=120):
    env = dict(os.environ, KFAMD_API_URL=cl.url)
    p = subprocess.run([sys.executable, "-m", "kubeflow_rm_amd.kfctl", *args, "--server", cl.url],
                       input=stdin, capture_output=True, text=True, timeout=timeout, env=env)
    return p.returncode, p.stdout, p.stderr


def test_reference_ci_sequence(cl):
    rc, out, err = kfctl(cl, "apply", "-f", "-", "-n", "ci-ns", stdin=NB_YAML)
    assert rc == 0, err
    # timeout 100 bash -c -- 'until kubectl get statefulset minimal-notebook; do sleep 1; done'
    deadline = time.time() + 100
    while True:
        rc, out, err = kfctl(cl, "get", "statefulset", "minimal-notebook", "-n", "ci-ns")
        if rc == 0:
            break
        assert "NotFound" in err, err
        assert time.time() < deadline
        time.sleep(0.2)
    assert out.splitlines()[0].split() == ["NAME", "READY", "AGE"]
    rc, out, err = kfctl(cl, "rollout", "status", "--watch", "statefulset", "minimal-notebook", "-n", "ci-ns")
    assert rc == 0, err
    rc, out, err = kfctl(cl, "wait", "statefulset", "minimal-notebook", "--for=jsonpath={.spec.replicas}=1",
                         "--timeout=100s", "-n", "ci-ns")
    assert rc == 0 and "statefulset.apps/minimal-notebook condition met" in out, (out, err)
    rc, out, err = kfctl(cl, "rollout", "status", "--watch", "statefulset", "minimal-notebook", "--timeout=300s",
                         "-n", "ci-ns")
    assert rc == 0 and "roll out complete" in out, (out, err)
    rc, out, err = kfctl(cl, "wait", "pods", "minimal-notebook-0", "--for=condition=Ready", "--timeout=100s",
                         "-n", "ci-ns")
    assert rc == 0 and "pod/minimal-notebook-0 condition met" in out, (out, err)
    # Print notebook logs (the workflow's failure dump)
    rc, out, err = kfctl(cl, "describe", "notebooks", "-n", "ci-ns")
    assert rc == 0 and "Name:         minimal-notebook" in out and "Kind:         Notebook" in out, err
    rc, out, err = kfctl(cl, "describe", "statefulsets", "-n", "ci-ns")
    assert rc == 0 and "Controlled By:  Notebook/minimal-notebook" in out, out
    rc, out, err = kfctl(cl, "describe", "pods", "-n", "ci-ns")
    assert rc == 0 and "Conditions:" in out and "Ready" in out and "Events:" in out, out
    rc, out, err = kfctl(cl, "logs", "minimal-notebook-0", "-n", "ci-ns")
    assert rc == 0, err
    rc, out, err = kfctl(cl, "describe", "routes", "-n", "ci-ns")
    assert rc == 0, err


def test_get_output_formats(cl):
    rc, out, err = kfctl(cl, "get", "nb", "-n", "ci-ns", "-o", "json")
    assert rc == 0
    doc = json.loads(out)
    assert doc["kind"] == "List" and doc["items"][0]["metadata"]["name"] == "minimal-notebook"
    rc, out, _ = kfctl(cl, "get", "notebooks.kubeflow.org/minimal-notebook", "-n", "ci-ns", "-o", "yaml")
    assert rc == 0 and "kind: Notebook" in out and "readyReplicas: 1" in out
    rc, out, _ = kfctl(cl, "get", "po", "-n", "ci-ns", "-o", "name")
    assert rc == 0 and out.strip() == "pod/minimal-notebook-0"
    rc, out, _ = kfctl(cl, "get", "pods", "-n", "ci-ns", "-o", "jsonpath={.items[*].metadata.name}")
    assert rc == 0 and out == "minimal-notebook-0"
    rc, out, _ = kfctl(cl, "get", "pods", "-A", "-o", "wide")
    hdr = out.splitlines()[0].split()
    assert rc == 0 and hdr[:2] == ["NAMESPACE", "NAME"] and "IP" in hdr
    rc, out, _ = kfctl(cl, "get", "notebook", "minimal-notebook", "-n", "ci-ns")
    assert rc == 0 and out.splitlines()[1].split()[:3] == ["minimal-notebook", "1", "Ready"]
    rc, out, _ = kfctl(cl, "get", "sts,svc", "-n", "ci-ns")
    assert rc == 0 and out.count("NAME") == 2 and "ClusterIP" in out
    rc, _, err = kfctl(cl, "get", "frobnicators")
    assert rc == 1 and "doesn't have a resource type" in err


def test_wait_by_label_timeout_and_delete(cl):
    # notebook_controller_integration_test.yaml:106 form: wait pods -l ... --for=condition=Ready
    rc, out, err = kfctl(cl, "wait", "pods", "-n", "ci-ns", "-l", "notebook-name=minimal-notebook",
                         "--for=condition=Ready", "--timeout=30s")
    assert rc == 0 and "condition met" in out, err
    rc, out, err = kfctl(cl, "wait", "pod/minimal-notebook-0", "-n", "ci-ns", "--for=condition=Bogus",
                         "--timeout=1s")
    assert rc == 1 and "timed out waiting for the condition" in err
    rc, out, err = kfctl(cl, "delete", "notebook", "minimal-notebook", "-n", "ci-ns")
    assert rc == 0 and "deleted" in out, err
    rc, out, err = kfctl(cl, "wait", "pods", "minimal-notebook-0", "-n", "ci-ns", "--for=delete", "--timeout=60s")
    assert rc == 0, err


METRICS = """# HELP kfamd_gpu_allocated 1 for every MI355X allocated to a pod by the device plugin
kfamd_gpu_allocated{gpu="0",namespace="team-a",pod="nb-0"} 1
kfamd_gpu_allocated{gpu="1",namespace="team-a",pod="nb-0"} 1
kfamd_gpu_gfx_activity_percent{gpu="0",namespace="team-a",pod="nb-0"} 90
kfamd_gpu_gfx_activity_percent{gpu="1",namespace="team-a",pod="nb-0"} 70
kfamd_gpu_gfx_activity_percent{gpu="2",namespace="",pod=""} 0
kfamd_gpu_vram_used_bytes{gpu="0"} 10737418240
kfamd_gpu_vram_used_bytes{gpu="1"} 5368709120
kfamd_gpu_vram_total_bytes{gpu="0"} 309237645312
kfamd_gpu_power_watts{gpu="0"} 1320
kfamd_gpu_gfxclk_mhz{gpu="0"} 1850
kfamd_gpu_temperature_celsius{gpu="0",sensor="hotspot"} 81
kfamd_gpu_temperature_celsius{gpu="0",sensor="hbm"} 70
"""


def test_top_tables_from_kubelet_metrics():
    from types import SimpleNamespace
    import io
    from kubeflow_rm_amd import kubectl

    class FakeClient:
        def _req(self, method, path, raw=False, **kw):
            assert (method, path, raw) == ("GET", "/metrics", True)
            return METRICS
    out = io.StringIO()
    assert kubectl.cmd_top(FakeClient(), SimpleNamespace(what="node", namespace=None), out) == 0
    lines = out.getvalue().splitlines()
    assert lines[0].split() == ["GPU", "POD", "GFX%", "HBM%", "VRAM", "POWER", "SCLK", "HOTSPOT"]
    row0 = lines[1].split()
    assert row0[:3] == ["0", "team-a/nb-0", "90%"] and row0[4] == "10.0Gi/288.0Gi" and row0[5:] == ["1320W", "1850MHz", "81C"]
    assert lines[3].split()[:2] == ["2", "<none>"]
    out = io.StringIO()
    assert kubectl.cmd_top(FakeClient(), SimpleNamespace(what="pod", namespace="team-a"), out) == 0
    rows = [r.split() for r in out.getvalue().splitlines()]
    assert rows[1] == ["team-a", "nb-0", "0,1", "80%", "15.0Gi", "1320W"]


def test_top_pod_on_the_cluster(cl):
    """kfctl top against kube-lite: a 2-GPU notebook shows up on its two devices (synthetic node:
    allocation series only, no AMD SMI telemetry)."""
    nb = {"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
          "metadata": {"name": "topnb", "namespace": "ci-ns", "annotations": {"kfamd.io/gpu-readiness-op": "false"}},
          "spec": {"template": {"spec": {"containers": [{"name": "topnb", "image": "jupyter-scipy:latest",
                                                          "resources": {"limits": {"amd.com/gpu": "2"}}}]}}}}
    cl.client.create(nb)
    cl.client.wait_for("v1", "Pod", "topnb-0", "ci-ns", lambda o: (o.get("spec") or {}).get("nodeName"), timeout=30)
    rc, out, err = kfctl(cl, "top", "pod", "-n", "ci-ns")
    assert rc == 0, err
    row = [r.split() for r in out.splitlines() if "topnb-0" in r][0]
    assert row[0] == "ci-ns" and len(row[2].split(",")) == 2
    rc, out, err = kfctl(cl, "top", "node")
    assert rc == 0, err
    assert sum("ci-ns/topnb-0" in r for r in out.splitlines()) == 2
    cl.client.delete("kubeflow.org/v1", "Notebook", "topnb", "ci-ns")


def test_exec_runs_in_the_container_environment(cl):
    """kfctl exec (pods/exec, no TTY): the command runs with the container's env and working directory,
    output comes back, and the exit status is the CLI's."""
    nb = {"apiVersion": "kubeflow.org/v1", "kind": "Notebook", "metadata": {"name": "exnb", "namespace": "ci-ns"},
          "spec": {"template": {"spec": {"containers": [{"name": "exnb", "image": "jupyter-scipy:latest",
                                                          "env": [{"name": "GREETING", "value": "hi from the pod"}]}]}}}}
    cl.client.create(nb)
    cl.client.wait_for("kubeflow.org/v1", "Notebook", "exnb", "ci-ns",
                       lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=60)
    env = dict(os.environ, KFAMD_API_URL=cl.url)

    def run(*args):
        p = subprocess.run([sys.executable, "-m", "kubeflow_rm_amd.kfctl", "exec", *args], capture_output=True, text=True,
                           timeout=60, env=env)
        return p.returncode, p.stdout, p.stderr
    rc, out, err = run("exnb-0", "-n", "ci-ns", "--", "sh", "-c", 'echo "$GREETING"; echo "$POD_NAME"; pwd; exit 3')
    assert rc == 3, err
    lines = out.splitlines()
    assert lines[0] == "hi from the pod" and lines[1] == "exnb-0" and "/pods/ci-ns_exnb-0_" in lines[2]
    assert "command terminated with exit code 3" in err
    rc, out, err = run("exnb-0", "-n", "ci-ns", "-c", "nope", "--", "true")
    assert rc == 1 and "not valid" in err
    rc, out, err = run("exnb-0", "-n", "ci-ns", "--timeout", "1s", "--", "sleep", "30")
    assert rc != 0 and "timeout" in out
    cl.client.delete("kubeflow.org/v1", "Notebook", "exnb", "ci-ns")


def test_exec_sees_the_pods_gpu_allocation(cl):
    """exec in a GPU notebook: the command gets the device plugin's HIP/ROCR visibility and the
    NUMA-local CPU mask the container process got."""
    nb = {"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
          "metadata": {"name": "gpunb", "namespace": "ci-ns", "annotations": {"kfamd.io/gpu-readiness-op": "false"}},
          "spec": {"template": {"spec": {"containers": [{"name": "gpunb", "image": "jupyter-scipy:latest",
                                                          "resources": {"limits": {"amd.com/gpu": "2"}}}]}}}}
    cl.client.create(nb)
    o = cl.client.wait_for("kubeflow.org/v1", "Notebook", "gpunb", "ci-ns",
                           lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=60)
    r = cl.client.pod_exec("gpunb-0", "ci-ns", ["sh", "-c", 'echo "$HIP_VISIBLE_DEVICES|$ROCR_VISIBLE_DEVICES|$WORLD_SIZE"'])
    assert r["exitCode"] == 0
    hip, rocr, world = r["output"].strip().split("|")
    assert len(hip.split(",")) == 2 and len(rocr.split(",")) == 2 and world == "2"
    rc, out, err = kfctl(cl, "describe", "pod", "gpunb-0", "-n", "ci-ns")
    assert rc == 0, err
    gpus_line = [ln for ln in out.splitlines() if ln.startswith("GPUs:")]
    assert gpus_line and "xGMI ring" in gpus_line[0], out
    rc, out, err = kfctl(cl, "get", "pods", "-n", "ci-ns", "-o", "wide")
    assert rc == 0, err
    hdr, row = out.splitlines()[0].split(), [r.split() for r in out.splitlines() if r.startswith("gpunb-0")][0]
    assert hdr[-1] == "GPUS" and len(row[-1].split(",")) == 2
    del o
    cl.client.delete("kubeflow.org/v1", "Notebook", "gpunb", "ci-ns")


def test_top_from_a_separate_node_agent_metrics_url():
    import http.server
    import io
    import threading
    from types import SimpleNamespace
    from kubeflow_rm_amd import kubectl

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            body = METRICS.encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        out = io.StringIO()
        a = SimpleNamespace(what="gpus", namespace=None, metrics_url=f"http://127.0.0.1:{srv.server_address[1]}/metrics")
        assert kubectl.cmd_top(None, a, out) == 0
        assert "team-a/nb-0" in out.getvalue()
    finally:
        srv.shutdown()


def test_exec_output_is_bounded(cl):
    """a command that floods stdout (``yes``) is killed once its output passes 64 MiB and the
    reply carries at most the last 16 MiB, instead of filling the pod directory and the kubelet's RAM."""
    nb = {"apiVersion": "kubeflow.org/v1", "kind": "Notebook", "metadata": {"name": "floodnb", "namespace": "ci-ns"},
          "spec": {"template": {"spec": {"containers": [{"name": "floodnb", "image": "jupyter-scipy:latest"}]}}}}
    cl.client.create(nb)
    cl.client.wait_for("kubeflow.org/v1", "Notebook", "floodnb", "ci-ns",
                       lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=60)
    t0 = time.time()
    r = cl.client.pod_exec("floodnb-0", "ci-ns", ["yes"], timeout=120)
    assert time.time() - t0 < 60
    out = r["output"]
    assert "output exceeded 64 MiB" in out
    assert len(out) <= (16 << 20) + 200
    assert out.startswith("[... output truncated ...]")
    cl.client.delete("kubeflow.org/v1", "Notebook", "floodnb", "ci-ns")


def test_exec_needs_create_on_pods_exec():
    """pods/exec is authorized as ``create``, whatever the HTTP method. A user whose
    role grants get/list on pods and every pods/* subresource gets 403 from exec (GET and POST); with
    ``create pods/exec`` the request gets past authorization (404: no such pod)."""
    from tests.conftest import _ensure_native
    _ensure_native()
    from kubeflow_rm_amd.client import ApiException, KubeClient
    with LocalCluster(args=["--authorization-mode", "RBAC"], controllers="builtin") as c:
        admin = c.client
        admin.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "rb"}})
        admin.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": "reader", "namespace": "rb"},
                      "rules": [{"apiGroups": [""], "resources": ["pods", "pods/*"], "verbs": ["get", "list", "watch"]}]})
        admin.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding", "metadata": {"name": "eve-reads", "namespace": "rb"},
                      "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": "reader"},
                      "subjects": [{"kind": "User", "name": "eve", "apiGroup": "rbac.authorization.k8s.io"}]})
        eve = KubeClient(c.url, impersonate="eve")
        for method in ("GET", "POST"):
            with pytest.raises(ApiException) as e:
                eve._req(method, "/api/v1/namespaces/rb/pods/p-0/exec", params={"command": "id"})
            assert e.value.status == 403, (method, e.value.status)
        with pytest.raises(ApiException) as e:
            eve.get("v1", "Pod", "p-0", "rb")
        assert e.value.status == 404  # get itself is allowed
        admin.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": "execer", "namespace": "rb"},
                      "rules": [{"apiGroups": [""], "resources": ["pods/exec"], "verbs": ["create"]}]})
        admin.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding", "metadata": {"name": "eve-execs", "namespace": "rb"},
                      "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": "execer"},
                      "subjects": [{"kind": "User", "name": "eve", "apiGroup": "rbac.authorization.k8s.io"}]})
        with pytest.raises(ApiException) as e:
            eve._req("POST", "/api/v1/namespaces/rb/pods/p-0/exec", params={"command": "id"})
        assert e.value.status == 404
