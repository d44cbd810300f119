"""TensorBoards (TWA) and Volumes (VWA) web apps against kube-lite, as a profile owner.

TWA: create from a pvc:// log path with a PodDefault configuration label, list until the
tensorboard controller reports it ready, delete.
VWA: create PVCs (storage-class sentinels), list with the notebooks mounting them, open a
PVCViewer from viewer-spec.yaml ($VAR expansion), refuse deleting a PVC a notebook pod mounts
(409) but delete one only a viewer mounts (viewer removed first).
"""
import os
import time

import pytest

from kubeflow_rm_amd.webapps import volumes as vwa

USER = "apps-owner@example.com"
NS = "apps-owner"


def _h(token=None):
    h = {"kubeflow-userid": USER}
    if token:
        h["X-XSRF-TOKEN"] = token
    return h


def _client(app):
    app.testing = True
    tc = app.test_client()
    assert tc.get("/", headers=_h()).status_code == 200
    return tc, tc.get_cookie("XSRF-TOKEN").value


@pytest.fixture(scope="module")
def apps(cluster):
    os.environ["APP_SECURE_COOKIES"] = "false"
    from kubeflow_rm_amd.webapps import tensorboards
    from kubeflow_rm_amd.webapps.crud_backend import config, k8s

    c = cluster.client
    c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": NS},
              "spec": {"owner": {"kind": "User", "name": USER}}})
    c.wait_for("rbac.authorization.k8s.io/v1", "RoleBinding", "namespaceAdmin", NS, lambda o: True, timeout=15)
    k8s.set_client(c)
    yield {"twa": _client(tensorboards.create_app(config.Config(mode="prod"))),
           "vwa": _client(vwa.create_app(config.Config(mode="prod"))), "c": c}
    os.environ.pop("APP_SECURE_COOKIES", None)


def _poll(fn, pred, timeout=40):
    deadline = time.time() + timeout
    while True:
        v = fn()
        if pred(v) or time.time() > deadline:
            return v
        time.sleep(0.5)


def test_storage_class_sentinels():
    assert vwa.handle_storage_class({}) is None
    assert vwa.handle_storage_class({"class": "{empty}"}) is None
    assert vwa.handle_storage_class({"class": "{none}"}) == ""
    assert vwa.handle_storage_class({"class": "fast"}) == "fast"
    pvc = vwa.pvc_from_dict({"name": "a", "mode": "ReadWriteOnce", "size": "1Gi", "class": "{none}"}, "ns")
    assert pvc["spec"]["storageClassName"] == "" and pvc["metadata"]["namespace"] == "ns"


def test_viewer_template_substitution(monkeypatch):
    monkeypatch.setenv("VOLUME_VIEWER_IMAGE", "my/filebrowser:1")
    v = vwa.create_viewer_template("data", "team")
    assert v["kind"] == "PVCViewer" and v["spec"]["pvc"] == "data"
    ctr = v["spec"]["podSpec"]["containers"][0]
    assert ctr["image"] == "my/filebrowser:1"
    assert {"name": "FB_BASEURL", "value": "/pvcviewers/team/data/"} in ctr["env"]
    assert v["spec"]["podSpec"]["volumes"][0]["persistentVolumeClaim"]["claimName"] == "data"


def test_viewer_status():
    assert vwa.viewer_status(None) == "uninitialized"
    assert vwa.viewer_status({"metadata": {"deletionTimestamp": "x"}}) == "terminating"
    assert vwa.viewer_status({"metadata": {}, "status": {"ready": True}}) == "ready"
    assert vwa.viewer_status({"metadata": {}, "status": {}}) == "waiting"


def test_twa_lifecycle(apps):
    tc, token = apps["twa"]
    c = apps["c"]
    c.create({"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "logs", "namespace": NS},
              "spec": {"accessModes": ["ReadWriteMany"], "resources": {"requests": {"storage": "1Gi"}}}})
    assert "logs" in tc.get(f"/api/namespaces/{NS}/pvcs", headers=_h()).get_json()["pvcs"]
    assert tc.post(f"/api/namespaces/{NS}/tensorboards", json={"name": "tb"}, headers=_h(token)).status_code == 400
    r = tc.post(f"/api/namespaces/{NS}/tensorboards", headers=_h(token),
                json={"name": "tb", "logspath": "pvc://logs/runs", "configurations": ["add-creds"]})
    assert r.status_code == 200, r.get_json()
    tb = c.get("tensorboard.kubeflow.org/v1alpha1", "Tensorboard", "tb", NS)
    assert tb["metadata"]["labels"] == {"add-creds": "true"} and tb["spec"]["logspath"] == "pvc://logs/runs"
    rows = _poll(lambda: tc.get(f"/api/namespaces/{NS}/tensorboards", headers=_h()).get_json()["tensorboards"],
                 lambda rows: rows and rows[0]["status"]["phase"] == "ready")
    assert rows[0]["name"] == "tb" and rows[0]["status"]["phase"] == "ready", rows
    assert tc.delete(f"/api/namespaces/{NS}/tensorboards/tb", headers=_h(token)).status_code == 200
    c.wait_gone("tensorboard.kubeflow.org/v1alpha1", "Tensorboard", "tb", NS, timeout=20)


def test_vwa_lifecycle(apps):
    tc, token = apps["vwa"]
    c = apps["c"]
    base = f"/api/namespaces/{NS}"
    body = {"name": "data", "mode": "ReadWriteOnce", "class": "{empty}", "size": "2Gi", "type": "empty"}
    assert tc.post(base + "/pvcs", json={"name": "x"}, headers=_h(token)).status_code == 400
    assert tc.post(base + "/pvcs", json=body, headers=_h(token)).status_code == 200
    assert tc.post(base + "/pvcs", json=dict(body, name="shared"), headers=_h(token)).status_code == 200
    rows = _poll(lambda: tc.get(base + "/pvcs", headers=_h()).get_json()["pvcs"],
                 lambda rows: all(r["status"]["phase"] == "ready" for r in rows))
    by = {r["name"]: r for r in rows}
    assert by["data"]["capacity"] == "2Gi" and by["data"]["viewer"]["status"] == "uninitialized"
    assert tc.get(base + "/pvcs/data", headers=_h()).get_json()["pvc"]["metadata"]["name"] == "data"
    assert tc.get(base + "/pvcs/data/events", headers=_h()).status_code == 200

    # a notebook mounting "shared": listed as its user, and the PVC cannot be deleted
    c.create({"apiVersion": "kubeflow.org/v1", "kind": "Notebook", "metadata": {"name": "user", "namespace": NS},
              "spec": {"template": {"spec": {"containers": [{"name": "user", "image": "jupyter-scipy:latest",
                                                             "volumeMounts": [{"name": "shared", "mountPath": "/data"}]}],
                                             "volumes": [{"name": "shared", "persistentVolumeClaim": {"claimName": "shared"}}]}}}})
    c.wait_for("v1", "Pod", "user-0", NS, lambda o: True, timeout=20)
    by = {r["name"]: r for r in tc.get(base + "/pvcs", headers=_h()).get_json()["pvcs"]}
    assert by["shared"]["notebooks"] == ["user"]
    assert [p["metadata"]["name"] for p in tc.get(base + "/pvcs/shared/pods", headers=_h()).get_json()["pods"]] == ["user-0"]
    r = tc.delete(base + "/pvcs/shared", headers=_h(token))
    assert r.status_code == 409 and "user-0" in r.get_json()["log"]

    # a viewer on "data": becomes ready, then deleting the PVC removes the viewer too
    assert tc.post(base + "/viewers", json={"name": "data"}, headers=_h(token)).status_code == 200
    rows = _poll(lambda: tc.get(base + "/pvcs", headers=_h()).get_json()["pvcs"],
                 lambda rows: {r["name"]: r for r in rows}["data"]["viewer"]["status"] == "ready")
    viewer = {r["name"]: r for r in rows}["data"]["viewer"]
    assert viewer["status"] == "ready" and viewer["url"].rstrip("/").endswith(f"/pvcviewers/{NS}/data"), viewer
    assert tc.delete(base + "/pvcs/data", headers=_h(token)).status_code == 200
    c.wait_gone("kubeflow.org/v1alpha1", "PVCViewer", "data", NS, timeout=20)
    c.wait_gone("v1", "PersistentVolumeClaim", "data", NS, timeout=20)
    c.delete("kubeflow.org/v1", "Notebook", "user", NS)
