"""Jupyter web app (JWA) backend.

Unit part: ports of the reference's apps/common/status_test.py and volumes_test.py (same cases,
pytest style; the PVC object is a plain dict since the `kubernetes` package is absent).
Integration part: the Flask app driven with its test client against a kube-lite cluster, as a
profile owner would through the ingress (user header + CSRF double-submit): config, spawn with
MI355X GPUs + workspace PVC, list with status, stop/start, pod/events/logs, delete, and the
authn/authz/CSRF refusals.
"""
import copy
import os
import time

import pytest
from werkzeug import exceptions

from kubeflow_rm_amd.webapps.jupyter import status, volumes

PVC_NAME = "workspace_volume"
NEW_API_VOLUME = {"name": "workspace-volume", "mount": "/home/jovyan",
                  "newPvc": {"metadata": {"name": PVC_NAME},
                             "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "5Gi"}}}}}
EXISTING_API_VOLUME = {"name": "workspace-volume", "mount": "/home/jovyan",
                       "existingSource": {"persistentVolumeClaim": {"claimName": PVC_NAME}}}


# ---- status_test.py ---------------------------------------------------------------------------
@pytest.mark.parametrize("state", [{"terminating": {}}, {"running": {}}])
def test_container_state_not_waiting(state):
    assert status.get_status_from_container_state({"status": {"containerState": state}}) == (None, None)


def test_container_state_waiting_without_message():
    nb = {"status": {"containerState": {"waiting": {"reason": "PodInitializing"}}}}
    assert status.get_status_from_container_state(nb) == (
        "warning", "PodInitializing: No available message for container state.")


# ---- volumes_test.py --------------------------------------------------------------------------
def test_volume_with_both_sources_rejected():
    v = copy.deepcopy(NEW_API_VOLUME)
    v[volumes.EXISTING_SOURCE] = {}
    with pytest.raises(exceptions.BadRequest):
        volumes.check_volume_format(v)


def test_volume_with_no_source_rejected():
    v = copy.deepcopy(NEW_API_VOLUME)
    del v[volumes.NEW_PVC]
    with pytest.raises(exceptions.BadRequest):
        volumes.check_volume_format(v)


def test_volume_without_mount_rejected():
    v = copy.deepcopy(EXISTING_API_VOLUME)
    del v[volumes.MOUNT]
    with pytest.raises(exceptions.BadRequest):
        volumes.check_volume_format(v)


def test_volume_name():
    with pytest.raises(exceptions.BadRequest):
        volumes.get_volume_name(copy.deepcopy(NEW_API_VOLUME))
    assert volumes.get_volume_name(copy.deepcopy(EXISTING_API_VOLUME)) == PVC_NAME
    v = copy.deepcopy(EXISTING_API_VOLUME)
    del v["existingSource"]["persistentVolumeClaim"]
    v["nfs"] = {"address": "127.0.0.1"}
    assert "existing-source-volume" in volumes.get_volume_name(v)


def test_pod_volume_uses_pvc_name():
    pvc = {"metadata": {"name": PVC_NAME}}
    assert volumes.get_pod_volume(copy.deepcopy(EXISTING_API_VOLUME), pvc) == {
        "name": PVC_NAME, "persistentVolumeClaim": {"claimName": PVC_NAME}}


def test_new_pvc_name_template_and_namespace_refused():
    v = copy.deepcopy(NEW_API_VOLUME)
    v["newPvc"]["metadata"]["name"] = "{notebook-name}-ws"
    assert volumes.get_new_pvc(v, "nb")["metadata"]["name"] == "nb-ws"
    v["newPvc"]["metadata"]["namespace"] = "x"
    with pytest.raises(exceptions.BadRequest):
        volumes.get_new_pvc(v, "nb")


def test_stopped_and_ready_status():
    old = "2020-01-01T00:00:00Z"
    nb = {"metadata": {"creationTimestamp": old, "annotations": {status.STOP_ANNOTATION: old}}, "status": {"readyReplicas": 0}}
    assert status.process_status(nb)["phase"] == "stopped"
    nb["status"]["readyReplicas"] = 1
    assert status.process_status(nb)["phase"] == "waiting"
    nb = {"metadata": {"creationTimestamp": old}, "status": {"readyReplicas": 1}}
    assert status.process_status(nb)["phase"] == "ready"


# ---- the app against kube-lite ----------------------------------------------------------------
USER = "jwa-owner@example.com"
NS = "jwa-owner"


@pytest.fixture(scope="module")
def jwa(cluster):
    os.environ["APP_SECURE_COOKIES"] = "false"
    from kubeflow_rm_amd.webapps import jupyter
    from kubeflow_rm_amd.webapps.crud_backend import config, k8s

    c = cluster.client
    c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": NS},
              "spec": {"owner": {"kind": "User", "name": USER}}})
    c.wait_for("rbac.authorization.k8s.io/v1", "RoleBinding", "namespaceAdmin", NS, lambda o: True, timeout=15)
    k8s.set_client(c)
    app = jupyter.create_app(config.Config(mode="prod"))
    app.testing = True
    tc = app.test_client()
    r = tc.get("/", headers={"kubeflow-userid": USER})  # index.html sets the CSRF cookie
    assert r.status_code == 200 and b'<base href="/">' in r.data
    token = tc.get_cookie("XSRF-TOKEN").value
    yield tc, token, c
    os.environ.pop("APP_SECURE_COOKIES", None)


def _h(token=None):
    h = {"kubeflow-userid": USER}
    if token:
        h["X-XSRF-TOKEN"] = token
    return h


def _spawn_body(name, gpus="2"):
    return {"name": name, "namespace": NS, "image": "kfamd/jupyter-pytorch-rocm:latest", "imagePullPolicy": "IfNotPresent",
            "serverType": "jupyter", "cpu": "1", "memory": "2Gi",
            "gpus": {"num": gpus, "vendor": "amd.com/gpu"} if gpus != "none" else {"num": "none"},
            "tolerationGroup": "none", "affinityConfig": "none", "configurations": [], "shm": True, "datavols": [],
            "workspace": {"mount": "/home/jovyan",
                          "newPvc": {"metadata": {"name": "{notebook-name}-workspace"},
                                     "spec": {"resources": {"requests": {"storage": "1Gi"}},
                                              "accessModes": ["ReadWriteOnce"]}}}}


def test_health_and_auth(jwa):
    tc, token, _ = jwa
    assert tc.get("/healthz/liveness").status_code == 200
    r = tc.get("/api/config")
    assert r.status_code == 401 and r.get_json()["success"] is False
    assert tc.get("/common/kf.js").status_code == 200
    assert tc.get("/assets/app.js", headers=_h()).status_code == 200


def test_config_and_gpu_vendors(jwa):
    tc, _, _ = jwa
    cfg = tc.get("/api/config", headers=_h()).get_json()["config"]
    assert cfg["gpus"]["value"]["vendors"][0]["limitsKey"] == "amd.com/gpu"
    assert tc.get("/api/gpus", headers=_h()).get_json()["vendors"] == ["amd.com/gpu"]
    # namespaces are cluster scoped: a plain profile owner gets them from the dashboard, not here
    assert tc.get("/api/namespaces", headers=_h()).status_code == 403


def test_csrf_required_for_mutations(jwa):
    tc, _, _ = jwa
    r = tc.post(f"/api/namespaces/{NS}/notebooks", json=_spawn_body("nocsrf"), headers=_h())
    assert r.status_code == 403 and "CSRF" in r.get_json()["log"]
    r = tc.post(f"/api/namespaces/{NS}/notebooks", json=_spawn_body("nocsrf"), headers=_h("wrong"))
    assert r.status_code == 403


def test_foreign_namespace_forbidden(jwa):
    tc, _, _ = jwa
    r = tc.get("/api/namespaces/kube-system/notebooks", headers=_h())
    assert r.status_code == 403 and "not authorized" in r.get_json()["log"]


def test_spawn_list_stop_start_delete(jwa):
    tc, token, c = jwa
    r = tc.post(f"/api/namespaces/{NS}/notebooks", json=_spawn_body("gpunb"), headers=_h(token))
    assert r.status_code == 200, r.get_json()
    nb = c.get("kubeflow.org/v1beta1", "Notebook", "gpunb", NS)
    ctr = nb["spec"]["template"]["spec"]["containers"][0]
    assert ctr["resources"]["limits"]["amd.com/gpu"] == "2"
    assert ctr["resources"]["limits"]["cpu"] == "1.2" and ctr["resources"]["limits"]["memory"] == "2.4Gi"
    assert {"name": "gpunb-workspace", "mountPath": "/home/jovyan"} in ctr["volumeMounts"]
    assert {"mountPath": "/dev/shm", "name": "dshm"} in ctr["volumeMounts"]
    assert nb["metadata"]["annotations"]["notebooks.kubeflow.org/creator"] == USER
    assert c.get("v1", "PersistentVolumeClaim", "gpunb-workspace", NS)["spec"]["resources"]["requests"]["storage"] == "1Gi"
    # duplicate name: the dry-run fails first and no second PVC is attempted
    r = tc.post(f"/api/namespaces/{NS}/notebooks", json=_spawn_body("gpunb"), headers=_h(token))
    assert r.status_code == 409

    deadline = time.time() + 40
    while True:
        rows = tc.get(f"/api/namespaces/{NS}/notebooks", headers=_h()).get_json()["notebooks"]
        row = [x for x in rows if x["name"] == "gpunb"][0]
        if row["status"]["phase"] == "ready" or time.time() > deadline:
            break
        time.sleep(0.5)
    assert row["status"]["phase"] == "ready", row["status"]
    assert row["gpus"] == {"count": 2, "message": "2 AMD Instinct MI355X"}
    assert row["shortImage"] == "jupyter-pytorch-rocm:latest"

    pod = tc.get(f"/api/namespaces/{NS}/notebooks/gpunb/pod", headers=_h()).get_json()["pod"]
    assert pod["metadata"]["name"] == "gpunb-0"
    r = tc.get(f"/api/namespaces/{NS}/notebooks/gpunb/pod/gpunb-0/logs", headers=_h())
    assert r.status_code == 200 and isinstance(r.get_json()["logs"], list)
    assert tc.get(f"/api/namespaces/{NS}/notebooks/gpunb/events", headers=_h()).status_code == 200
    assert tc.get(f"/api/namespaces/{NS}/notebooks/gpunb", headers=_h()).get_json()["notebook"]["processed_status"]["phase"] == "ready"

    assert tc.patch(f"/api/namespaces/{NS}/notebooks/gpunb", json={"stopped": True}, headers=_h(token)).status_code == 200
    assert tc.patch(f"/api/namespaces/{NS}/notebooks/gpunb", json={"stopped": True}, headers=_h(token)).status_code == 409
    c.wait_for("apps/v1", "StatefulSet", "gpunb", NS, lambda o: o["spec"]["replicas"] == 0, timeout=10)
    deadline = time.time() + 30
    while time.time() < deadline:
        row = [x for x in tc.get(f"/api/namespaces/{NS}/notebooks", headers=_h()).get_json()["notebooks"]
               if x["name"] == "gpunb"][0]
        if row["status"]["phase"] == "stopped":
            break
        time.sleep(0.5)
    assert row["status"]["phase"] == "stopped"
    assert tc.patch(f"/api/namespaces/{NS}/notebooks/gpunb", json={"stopped": False}, headers=_h(token)).status_code == 200
    c.wait_for("apps/v1", "StatefulSet", "gpunb", NS, lambda o: o["spec"]["replicas"] == 1, timeout=10)

    r = tc.delete(f"/api/namespaces/{NS}/notebooks/gpunb", headers=_h(token))
    assert r.status_code == 200
    c.wait_gone("kubeflow.org/v1beta1", "Notebook", "gpunb", NS, timeout=30)


def test_form_validation(jwa):
    tc, token, _ = jwa
    body = _spawn_body("badgpu")
    body["gpus"] = {"num": "two", "vendor": "amd.com/gpu"}
    r = tc.post(f"/api/namespaces/{NS}/notebooks", json=body, headers=_h(token))
    assert r.status_code == 400
    body = _spawn_body("badtype")
    body["serverType"] = "emacs"
    assert tc.post(f"/api/namespaces/{NS}/notebooks", json=body, headers=_h(token)).status_code == 400
    body = _spawn_body("nocpu")
    del body["cpu"]
    assert tc.post(f"/api/namespaces/{NS}/notebooks", json=body, headers=_h(token)).status_code == 400
    r = tc.post(f"/api/namespaces/{NS}/notebooks", data="x", headers=_h(token))
    assert r.status_code == 400
