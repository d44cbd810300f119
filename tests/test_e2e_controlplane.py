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
    cl.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "e2e"}})
    return cl


def test_notebook_to_statefulset_service_and_ready(c, cluster):
    c.create(_notebook("nb1", "e2e"))
    sts = c.wait_for("apps/v1", "StatefulSet", "nb1", "e2e", lambda o: True, timeout=10)
    ref = sts["metadata"]["ownerReferences"][0]
    assert ref["kind"] == "Notebook" and ref["name"] == "nb1" and ref["controller"] is True
    svc = c.get("v1", "Service", "nb1", "e2e")
    assert svc["spec"]["ports"][0]["targetPort"] == 8888
    vs = c.get("networking.istio.io/v1alpha3", "VirtualService", "notebook-e2e-nb1", "e2e")
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
            if e.code != 503 or time.time() > deadline:
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
