"""Tensorboard + PVCViewer CRs end to end (BASELINE config 5's control-plane path, CPU).

Event files written with the framework's own tfevents writer into a PVC are served by the
tensorboard pod through the ingress gateway; the PVCViewer's file browser lists the same PVC.
Webhook cases port pvcviewer_controller_test.go:69-138.
"""
import json
import os
import time
import urllib.error
import urllib.request

import pytest

from kubeflow_rm_amd.client import ApiException
from kubeflow_rm_amd.utils.tfevents import SummaryWriter

NS = "tbpv"


@pytest.fixture(scope="module")
def c(cluster):
    cl = cluster.client
    cl.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": NS}})
    cl.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "logs", "namespace": NS},
               "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}})
    return cl


def _get(url, timeout=15.0):
    """GET through the gateway. The pods carry no readiness probe (as in the reference manifests),
    so Ready can precede the server's bind by a few ms: a 502/503 or refused connection is retried."""
    deadline = time.time() + timeout
    while True:
        try:
            with urllib.request.urlopen(url, timeout=5) as r:
                return json.loads(r.read())
        except urllib.error.HTTPError as e:
            if e.code not in (502, 503) or time.time() > deadline:
                raise
        except urllib.error.URLError:
            if time.time() > deadline:
                raise
        time.sleep(0.1)


def test_tensorboard_serves_pvc_logs(c, cluster):
    pvdir = os.path.join(cluster.data_dir, "kubelet", "pv", NS, "logs", "run1")
    with SummaryWriter(pvdir) as w:
        for step in range(5):
            w.add_scalar("loss", 1.0 / (step + 1), step)
    c.create({"apiVersion": "tensorboard.kubeflow.org/v1alpha1", "kind": "Tensorboard",
              "metadata": {"name": "tb", "namespace": NS}, "spec": {"logspath": "pvc://logs/"}})
    c.wait_for("apps/v1", "Deployment", "tb", NS, lambda o: True, timeout=10)
    tb = c.wait_for("tensorboard.kubeflow.org/v1alpha1", "Tensorboard", "tb", NS,
                    lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=30)
    assert tb["status"]["conditions"]
    vs = c.get("networking.istio.io/v1alpha3", "VirtualService", "tb", NS)
    assert vs["spec"]["http"][0]["match"][0]["uri"]["prefix"] == f"/tensorboard/{NS}/tb/"
    base = cluster.gateway + f"/tensorboard/{NS}/tb"
    assert _get(base + "/data/runs") == ["run1"]
    pts = _get(base + "/data/plugin/scalars/scalars?run=run1&tag=loss")
    assert [p[1] for p in pts] == [0, 1, 2, 3, 4]
    assert abs(pts[-1][2] - 0.2) < 1e-6


def test_pvcviewer_webhooks(c):
    with pytest.raises(ApiException) as e:
        c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PVCViewer", "metadata": {"name": "bad", "namespace": NS},
                  "spec": {"pvc": "", "rwoScheduling": False}})
    assert "denied the request: PVC name must be specified" in str(e.value.body)
    with pytest.raises(ApiException) as e:
        c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PVCViewer", "metadata": {"name": "bad2", "namespace": NS},
                  "spec": {"pvc": "test-pvc", "rwoScheduling": False, "podSpec": {"containers": [{"name": "test", "image": "test"}], "volumes": []}}})
    assert "denied the request: PVC test-pvc must be used in the podSpec" in str(e.value.body)
    v = c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PVCViewer", "metadata": {"name": "dflt", "namespace": NS},
                  "spec": {"pvc": "test-pvc", "rwoScheduling": False}})
    ps = v["spec"]["podSpec"]
    assert len(ps["containers"]) == 1 and ps["containers"][0]["image"]
    assert ps["volumes"] == [{"name": "viewer-volume", "persistentVolumeClaim": {"claimName": "test-pvc"}}]
    c.delete("kubeflow.org/v1alpha1", "PVCViewer", "dflt", NS)


def test_pvcviewer_browses_pvc(c, cluster):
    pvdir = os.path.join(cluster.data_dir, "kubelet", "pv", NS, "logs")
    os.makedirs(pvdir, exist_ok=True)
    with open(os.path.join(pvdir, "hello.txt"), "w") as f:
        f.write("hi")
    c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PVCViewer", "metadata": {"name": "viewer", "namespace": NS},
              "spec": {"pvc": "logs", "rwoScheduling": True, "networking": {"basePrefix": "/pvcviewer", "targetPort": 8080}}})
    v = c.wait_for("kubeflow.org/v1alpha1", "PVCViewer", "viewer", NS, lambda o: (o.get("status") or {}).get("ready") is True,
                   timeout=30)
    assert v["status"]["url"] == f"/pvcviewer/{NS}/viewer/"
    dep = c.get("apps/v1", "Deployment", "pvcviewer-viewer", NS)
    assert dep["spec"]["strategy"]["type"] == "Recreate"
    # the tensorboard pod mounts the RWO pvc on the node -> preferred affinity to it
    aff = dep["spec"]["template"]["spec"].get("affinity", {})
    terms = aff.get("nodeAffinity", {}).get("preferredDuringSchedulingIgnoredDuringExecution", [])
    assert terms and terms[0]["preference"]["matchExpressions"][0]["values"] == ["mi355x-node-0"]
    listing = _get(cluster.gateway + f"/pvcviewer/{NS}/viewer/api/resources/")
    assert "hello.txt" in [i["name"] for i in listing["items"]]
