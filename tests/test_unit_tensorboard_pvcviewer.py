"""Tensorboard + PVCViewer pure functions (native).

Reference: tensorboard-controller/controllers/tensorboard_controller.go:167-486,
pvcviewer-controller/api/v1alpha1/pvcviewer_webhook.go:53-199,
pvcviewer-controller/controllers/pvcviewer_controller.go:149-445 and the envtest cases of
pvcviewer_controller_test.go (webhook defaulting/validation, RWO affinity).
"""
from pathlib import Path

import pytest
import yaml

FIX = Path(__file__).parent / "fixtures"


def _tb(logs, name="tb", ns="ns", labels=None):
    return {"metadata": {"name": name, "namespace": ns, "labels": labels or {}}, "spec": {"logspath": logs}}


@pytest.mark.parametrize("path,cloud,gcs,pvc,name,sub", [
    ("pvc://my-pvc/logs/run1", False, False, True, "my-pvc", "logs/run1"),
    ("pvc://my-pvc", False, False, True, "my-pvc", ""),
    ("pvc://my-pvc/", False, False, True, "my-pvc", ""),
    ("gs://bucket/x", True, True, False, "gs:", "bucket/x"),
    ("s3://bucket/x", True, False, False, "s3:", "bucket/x"),
    ("/cns/x", True, False, False, "", "cns/x"),
    ("/local/logs", False, False, False, "", "local/logs"),
])
def test_logspath_forms(native, path, cloud, gcs, pvc, name, sub):
    r = native.call("tb_paths", path=path)
    assert (r["cloud"], r["gcs"], r["pvc"]) == (cloud, gcs, pvc)
    if pvc:
        assert (r["pvc_name"], r["pvc_subpath"]) == (name, sub)


def test_tb_deployment_pvc(native):
    d = native.call("tb_generate_deployment", tensorboard=_tb("pvc://logs-pvc/run1", labels={"x": "y"}), image="tb:1")
    c = d["spec"]["template"]["spec"]["containers"][0]
    assert c["args"] == ["--logdir=/tensorboard_logs/", "--bind_all"]
    assert c["command"] == ["/usr/local/bin/tensorboard"] and c["image"] == "tb:1"
    assert c["ports"] == [{"containerPort": 6006}]
    assert c["volumeMounts"] == [{"name": "tbpd", "readOnly": True, "mountPath": "/tensorboard_logs/", "subPath": "run1"}]
    assert d["spec"]["template"]["spec"]["volumes"] == [{"name": "tbpd", "persistentVolumeClaim": {"claimName": "logs-pvc"}}]
    assert d["spec"]["template"]["metadata"]["labels"] == {"x": "y", "app": "tb"}
    assert d["spec"]["selector"]["matchLabels"] == {"app": "tb"}


def test_tb_deployment_gcs_and_legacy(native):
    d = native.call("tb_generate_deployment", tensorboard=_tb("gs://b/logs"), image="i")
    ps = d["spec"]["template"]["spec"]
    assert ps["volumes"] == [{"name": "gcp-creds", "secret": {"secretName": "user-gcp-sa"}}]
    assert ps["containers"][0]["args"][0] == "--logdir=gs://b/logs"
    d = native.call("tb_generate_deployment", tensorboard=_tb("/data/logs"), image="i")
    ps = d["spec"]["template"]["spec"]
    assert ps["volumes"][0]["persistentVolumeClaim"]["claimName"] == "tb-volume"
    assert ps["containers"][0]["volumeMounts"][0]["mountPath"] == "/data/logs"
    d = native.call("tb_generate_deployment", tensorboard=_tb("s3://b/logs"), image="i")
    assert "volumes" not in d["spec"]["template"]["spec"]


def test_tb_rwo_affinity(native):
    d = native.call("tb_generate_deployment", tensorboard=_tb("pvc://p"), image="i", node="node-7")
    term = d["spec"]["template"]["spec"]["affinity"]["nodeAffinity"]["preferredDuringSchedulingIgnoredDuringExecution"][0]
    assert term["weight"] == 100
    assert term["preference"]["matchExpressions"][0] == {"key": "kubernetes.io/hostname", "operator": "In", "values": ["node-7"]}


def test_tb_service_and_vs(native):
    s = native.call("tb_generate_service", tensorboard=_tb("x"))
    assert s["spec"]["ports"] == [{"name": "http-tb", "port": 80, "targetPort": 6006}]
    vs = native.call("tb_generate_virtual_service", tensorboard=_tb("x"), gateway="kubeflow/kubeflow-gateway", host="*")
    h = vs["spec"]["http"][0]
    assert h["match"][0]["uri"]["prefix"] == "/tensorboard/ns/tb/"
    assert h["rewrite"]["uri"] == "/" and h["timeout"] == "300s"
    assert h["route"][0]["destination"] == {"host": "tb.ns.svc.cluster.local", "port": {"number": 80}}


def test_tb_copy_fields_only_labels_replicas_affinity(native):
    a = native.call("tb_generate_deployment", tensorboard=_tb("pvc://p"), image="i")
    b = native.call("tb_generate_deployment", tensorboard=_tb("pvc://other"), image="j")
    r = native.call("tb_copy_deployment_fields", **{"from": a, "to": b})
    assert r["changed"] is False  # the reference ignores template changes (quirk kept)
    a2 = native.call("tb_generate_deployment", tensorboard=_tb("pvc://p"), image="i", node="n1")
    assert native.call("tb_copy_deployment_fields", **{"from": a2, "to": b})["changed"] is True


def test_tb_status_appends_on_change(native):
    tb = {"status": {"conditions": [{"deploymentState": "Progressing"}], "readyReplicas": 0}}
    dep = {"status": {"readyReplicas": 1, "conditions": [{"type": "Available", "lastUpdateTime": "2024-01-01T00:00:00Z"}]}}
    st = native.call("tb_status", tensorboard=tb, deployment=dep)
    assert [c["deploymentState"] for c in st["conditions"]] == ["Progressing", "Available"]
    assert st["readyReplicas"] == 1
    tb["status"] = st
    assert len(native.call("tb_status", tensorboard=tb, deployment=dep)["conditions"]) == 2


def _viewer(pvc="test-pvc", pod_spec=None, networking=None, name="v", ns="ns"):
    spec = {"pvc": pvc}
    if pod_spec is not None:
        spec["podSpec"] = pod_spec
    if networking is not None:
        spec["networking"] = networking
    return {"metadata": {"name": name, "namespace": ns}, "spec": spec}


def test_pvcviewer_should_create_a_podspec(native):
    v = native.call("pvcviewer_default", viewer=_viewer(networking={"basePrefix": "/pvcviewer", "targetPort": 8080}))
    ps = v["spec"]["podSpec"]
    assert len(ps["containers"]) == 1 and ps["containers"][0]["image"]
    assert ps["volumes"] == [{"name": "viewer-volume", "persistentVolumeClaim": {"claimName": "test-pvc"}}]
    env = {e["name"]: e["value"] for e in ps["containers"][0]["env"]}
    assert env["FB_BASEURL"] == "/pvcviewer/ns/v/" and env["FB_PORT"] == "8080"


def test_pvcviewer_uses_default_file(native):
    default = yaml.safe_load((FIX / "podspec_default.yaml").read_text())
    v = native.call("pvcviewer_default", viewer=_viewer(), default_pod_spec=default)
    ps = v["spec"]["podSpec"]
    assert ps["containers"][0]["name"] == "test"
    assert ps["securityContext"]["runAsUser"] == 1234


def test_pvcviewer_validation(native):
    assert native.call("pvcviewer_validate", viewer=_viewer(pvc="")) == "PVC name must be specified"
    assert native.call("pvcviewer_validate", viewer=_viewer(pod_spec={})) == "PodSpec must be specified"
    bad = _viewer(pod_spec={"containers": [{"name": "test", "image": "test"}], "volumes": []})
    assert native.call("pvcviewer_validate", viewer=bad) == "PVC test-pvc must be used in the podSpec"
    good = native.call("pvcviewer_default", viewer=_viewer())
    assert native.call("pvcviewer_validate", viewer=good) == ""


def test_pvcviewer_generation(native):
    v = native.call("pvcviewer_default", viewer=_viewer(networking={"basePrefix": "/pvcviewer", "targetPort": 8080,
                                                                    "rewrite": "/", "timeout": "30s"}))
    d = native.call("pvcviewer_generate_deployment", viewer=v)
    labels = {"app.kubernetes.io/name": "v", "app.kubernetes.io/instance": "pvcviewer-v", "app.kubernetes.io/part-of": "pvc-viewer"}
    assert d["metadata"]["name"] == "pvcviewer-v" and d["spec"]["strategy"] == {"type": "Recreate"}
    assert d["spec"]["selector"]["matchLabels"] == labels
    s = native.call("pvcviewer_generate_service", viewer=v)
    assert s["spec"]["ports"] == [{"name": "http", "port": 80, "targetPort": 8080}]
    vs = native.call("pvcviewer_generate_virtual_service", viewer=v, gateway="kubeflow/kubeflow-gateway")
    h = vs["spec"]["http"][0]
    assert h["match"][0]["uri"]["prefix"] == "/pvcviewer/ns/v/" and h["rewrite"]["uri"] == "/" and h["timeout"] == "30s"
    assert h["route"][0]["destination"]["host"] == "pvcviewer-v.ns.svc.cluster.local"


def _pod(name, node, pvc, part_of=None):
    labels = {"app.kubernetes.io/part-of": part_of} if part_of else {}
    return {"metadata": {"name": name, "labels": labels},
            "spec": {"nodeName": node, "volumes": [{"name": "pvc", "persistentVolumeClaim": {"claimName": pvc}}]}}


@pytest.mark.parametrize("modes,pods,want", [
    (["ReadWriteMany"], [_pod("a", "n1", "p")], ""),
    (["ReadWriteOnce"], [_pod("a", "n1", "p")], "n1"),
    (["ReadWriteOnce"], [_pod("a", "n1", "p"), _pod("b", "n2", "p")], ""),
    (["ReadWriteOnce"], [_pod("a", "n1", "p"), _pod("b", "n1", "p")], "n1"),  # conscious fix: same node is fine
    (["ReadWriteOnce"], [_pod("a", "", "p")], ""),
    (["ReadWriteOnce"], [_pod("viewer", "n9", "p", part_of="pvc-viewer")], ""),
    (["ReadWriteOnce"], [_pod("a", "n1", "other")], ""),
])
def test_pvcviewer_rwo_node(native, modes, pods, want):
    pvc = {"metadata": {"name": "p"}, "spec": {"accessModes": modes}}
    assert native.call("pvcviewer_rwo_node", pvc=pvc, pods=pods) == want
