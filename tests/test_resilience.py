"""Failure detection / recovery / persistence on the embedded control plane.

* fault injection through the API server's ``/debug/faults`` switchboard: injected 500s and 409s
  on the objects a reconciler writes are absorbed by level-triggered requeue with backoff
  (reference: any error -> requeue; RetryOnConflict for Route / NetworkPolicy updates);
* persistence: the WAL replays every object (uid, resourceVersion, status) into a restarted API
  server, so controllers rebuild from list+watch (reference: state lives in etcd);
* idle culling end to end (reference e2e ``notebook_creation_test.go:243-287``: idle notebook ->
  ``kubeflow-resource-stopped`` -> StatefulSet scaled to 0), with a 1 s check period.
"""
import json
import tempfile
import urllib.request

import pytest

from kubeflow_rm_amd.cluster import LocalCluster

NB = "kubeflow.org/v1"


def _notebook(name, ns, annotations=None):
    return {"apiVersion": NB, "kind": "Notebook",
            "metadata": {"name": name, "namespace": ns, "annotations": annotations or {}},
            "spec": {"template": {"spec": {"containers": [{"name": name, "image": "jupyter-scipy:latest"}]}}}}


def _post(url, body):
    req = urllib.request.Request(url, data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=5) as r:
        return r.status


def _metric(url, prefix):
    with urllib.request.urlopen(url + "/metrics", timeout=5) as r:
        return sum(float(line.split()[-1]) for line in r.read().decode().splitlines() if line.startswith(prefix))


def _ready(o):
    return (o.get("status") or {}).get("readyReplicas") == 1


@pytest.fixture(scope="module")
def cluster():
    cl = LocalCluster(env={"ENABLE_CULLING": "false", "USE_ISTIO": "true"})
    cl.start()
    cl.client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "faults"}})
    yield cl
    cl.stop()


def test_injected_server_errors_are_retried_until_the_notebook_is_ready(cluster):
    c = cluster.client
    errors0 = _metric(cluster.url, 'controller_runtime_reconcile_errors_total{controller="notebook-controller"}')
    assert _post(cluster.url + "/debug/faults", {"spec": "error:statefulsets:3"}) == 200
    c.create(_notebook("flaky", "faults"))
    c.wait_for("apps/v1", "StatefulSet", "flaky", "faults", lambda o: True, timeout=20)
    c.wait_for(NB, "Notebook", "flaky", "faults", _ready, timeout=30)
    errors1 = _metric(cluster.url, 'controller_runtime_reconcile_errors_total{controller="notebook-controller"}')
    assert errors1 >= errors0 + 3  # every injected 500 surfaced as a reconcile error, then requeued


def test_injected_conflicts_on_status_updates_are_absorbed(cluster):
    c = cluster.client
    assert _post(cluster.url + "/debug/faults", {"spec": "conflict:notebooks:4"}) == 200
    c.create(_notebook("contended", "faults"))
    nb = c.wait_for(NB, "Notebook", "contended", "faults", _ready, timeout=30)
    assert any(x["type"] == "Ready" for x in nb["status"]["conditions"])


def test_bad_fault_spec_is_rejected(cluster):
    with pytest.raises(urllib.error.HTTPError) as ei:
        _post(cluster.url + "/debug/faults", {"spec": "explode:pods:1"})
    assert ei.value.code == 400


def test_state_survives_an_api_server_restart():
    with tempfile.TemporaryDirectory(prefix="kflite-wal-") as d:
        cl = LocalCluster(data_dir=d, controllers="builtin")
        cl.start()
        c = cl.client
        c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "persist"}})
        cm = c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cfg", "namespace": "persist"},
                       "data": {"k": "v1"}})
        cm["data"]["k"] = "v2"
        cm = c.update(cm)
        c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile",
                  "metadata": {"name": "alice"}, "spec": {"owner": {"kind": "User", "name": "alice@example.com"}}})
        cl.stop()
        cl2 = LocalCluster(data_dir=d, controllers="builtin")
        cl2.start()
        try:
            c2 = cl2.client
            back = c2.get("v1", "ConfigMap", "cfg", "persist")
            assert back["data"] == {"k": "v2"}
            assert back["metadata"]["uid"] == cm["metadata"]["uid"]
            assert back["metadata"]["resourceVersion"] == cm["metadata"]["resourceVersion"]
            assert c2.get("kubeflow.org/v1", "Profile", "alice")["spec"]["owner"]["name"] == "alice@example.com"
            # resourceVersions keep increasing across the restart (watchers resume, no reuse)
            nxt = c2.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "after", "namespace": "persist"}})
            assert int(nxt["metadata"]["resourceVersion"]) > int(cm["metadata"]["resourceVersion"])
        finally:
            cl2.stop()


def test_idle_notebook_is_culled():
    env = {"ENABLE_CULLING": "true", "CULL_IDLE_TIME": "0", "IDLENESS_CHECK_PERIOD_SECONDS": "1", "USE_ISTIO": "true"}
    with LocalCluster(env=env) as cl:
        c = cl.client
        c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "cull"}})
        c.create(_notebook("sleepy", "cull"))

        def stopped(o):
            return "kubeflow-resource-stopped" in ((o.get("metadata") or {}).get("annotations") or {})
        # CULL_IDLE_TIME=0: idle as soon as its pod exists and a check ran (the reference gates on the
        # pod's existence, not readiness: culling_controller.go:112-125)
        nb = c.wait_for(NB, "Notebook", "sleepy", "cull", stopped, timeout=40)
        # once stopping, the culler drops its activity annotations (culling_controller.go:99-111)
        nb = c.wait_for(NB, "Notebook", "sleepy", "cull",
                        lambda o: "notebooks.kubeflow.org/last-activity" not in o["metadata"].get("annotations", {}),
                        timeout=15)
        assert "notebooks.kubeflow.org/last_activity_check_timestamp" not in nb["metadata"]["annotations"]
        c.wait_for("apps/v1", "StatefulSet", "sleepy", "cull", lambda o: o["spec"]["replicas"] == 0, timeout=15)
        c.wait_gone("v1", "Pod", "sleepy-0", "cull", timeout=30)
