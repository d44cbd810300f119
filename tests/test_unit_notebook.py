"""Notebook controller + culler pure functions (native, via libkfcore_capi).

Ported table cases:
  reference components/notebook-controller/controllers/notebook_controller_test.go:22-299
  reference components/notebook-controller/controllers/culling_controller_test.go:14-263
plus generation checks of the StatefulSet / Service / VirtualService shapes
(notebook_controller.go:409-620).
"""
import datetime as dt

import pytest

STOP = "kubeflow-resource-stopped"
LAST = "notebooks.kubeflow.org/last-activity"


def _nb(name="test", ns="kubeflow-user", **extra):
    nb = {"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
          "metadata": {"name": name, "namespace": ns, "uid": "u-1"},
          "spec": {"template": {"spec": {"containers": [{"name": name, "image": "jupyter-scipy:v1"}]}}}}
    nb.update(extra)
    return nb


# ---- createNotebookStatus -------------------------------------------------------------------
def _cond(t, **kw):
    c = {"type": t}
    c.update(kw)
    return c


STATUS_CASES = [
    ("NotebookStatusInitialization", {}, {}, {"conditions": [], "readyReplicas": 0, "containerState": {}}),
    ("NotebookStatusReadyReplicas", {}, {"status": {"readyReplicas": 1}},
     {"conditions": [], "readyReplicas": 1, "containerState": {}}),
    ("NotebookContainerState",
     {"status": {"containerStatuses": [{"name": "test", "state": {"running": {"startedAt": "2022-08-30T01:10:30Z"}}}]}},
     {}, {"conditions": [], "readyReplicas": 0, "containerState": {"running": {"startedAt": "2022-08-30T01:10:30Z"}}}),
    ("mirroringPodConditions",
     {"status": {"conditions": [
         _cond("Running", lastProbeTime="2022-08-30T01:10:30Z", lastTransitionTime="2022-08-30T01:10:30Z"),
         _cond("Waiting", lastProbeTime="2022-08-30T01:10:30Z", lastTransitionTime="2022-08-30T01:10:30Z",
               reason="PodInitializing")]}},
     {"status": {"readyReplicas": 1}},
     {"conditions": [
         _cond("Running", lastProbeTime="2022-08-30T01:10:30Z", lastTransitionTime="2022-08-30T01:10:30Z"),
         _cond("Waiting", lastProbeTime="2022-08-30T01:10:30Z", lastTransitionTime="2022-08-30T01:10:30Z",
               reason="PodInitializing")],
      "readyReplicas": 1, "containerState": {}}),
    ("unschedulablePod",
     {"status": {"conditions": [_cond("PodScheduled", lastProbeTime="2022-04-21T01:10:30Z",
                                      lastTransitionTime="2022-04-21T01:10:30Z",
                                      message="0/1 nodes are available: 1 Insufficient cpu.", status="false",
                                      reason="Unschedulable")]}},
     {"status": {}},
     {"conditions": [_cond("PodScheduled", lastProbeTime="2022-04-21T01:10:30Z",
                           lastTransitionTime="2022-04-21T01:10:30Z",
                           message="0/1 nodes are available: 1 Insufficient cpu.", status="false",
                           reason="Unschedulable")],
      "readyReplicas": 0, "containerState": {}}),
]


@pytest.mark.parametrize("name,pod,sts,want", STATUS_CASES, ids=[c[0] for c in STATUS_CASES])
def test_create_notebook_status(native, name, pod, sts, want):
    got = native.call("create_notebook_status", notebook=_nb(), statefulset=sts, pod=pod)
    for c in got["conditions"]:  # empty optional fields are omitted like Go's omitempty
        for k in [k for k, v in c.items() if v in ("", None)]:
            del c[k]
    assert got == want


# ---- culling --------------------------------------------------------------------------------
def test_set_stop_annotation(native):
    for ann in (None, {}, {STOP: "2024-01-01T00:00:00Z"}):
        obj = {"metadata": {} if ann is None else {"annotations": ann}}
        out = native.call("set_stop_annotation", object=obj)
        assert STOP in out["metadata"]["annotations"]


@pytest.mark.parametrize("meta,want", [({}, False), ({"annotations": {}}, False),
                                       ({"annotations": {STOP: "2024-01-01T00:00:00Z"}}, True)])
def test_stop_annotation_is_set(native, meta, want):
    assert native.call("stop_annotation_is_set", object={"metadata": meta}) is want


@pytest.mark.parametrize("states,want", [([], True), (["idle", "idle"], True), (["idle", "busy"], False)])
def test_all_kernels_are_idle(native, states, want):
    kernels = [{"id": str(i), "execution_state": s, "last_activity": "2024-01-01T00:00:00Z"} for i, s in enumerate(states)]
    assert native.call("all_kernels_are_idle", kernels=kernels) is want


def _rfc(delta_min=0.0):
    return (dt.datetime.now(dt.timezone.utc) + dt.timedelta(minutes=delta_min)).strftime("%Y-%m-%dT%H:%M:%SZ")


class _Now:
    """A timestamp `minutes` from now, taken when the test runs (not at collection: in a long serial
    run the gap between the two pushed the 3-minutes-ago case past the 5-minute deadline)."""

    def __init__(self, minutes=0.0):
        self.minutes = minutes


IDLE_CASES = [
    ("No existing Annotations", {}, 1440, False),
    ("Basic case", {"annotations": {}}, 1440, False),
    ("Stop Annotation already set", {"annotations": {STOP: _Now()}}, 1440, False),
    ("LAST_ACTIVITY_ANNOTATION is not set", {"annotations": {}}, 1440, False),
    ("LAST_ACTIVITY_ANNOTATION is not RF3339", {"annotations": {LAST: "should-fail"}}, 1440, False),
    ("LAST_ACTIVITY_ANNOTATION is old", {"annotations": {LAST: "2021-08-30T15:37:36.990063Z"}}, 1440, True),
    ("LAST_ACTIVITY_ANNOTATION is too old", {"annotations": {LAST: "1900-08-30T15:37:36.990063Z"}}, 1440, True),
    ("LAST_ACTIVITY_ANNOTATION is the current time", {"annotations": {LAST: _Now()}}, 5, False),
    ("1 minute MORE than the deadline", {"annotations": {LAST: _Now(-6)}}, 5, True),
    ("1 minute LESS than the deadline", {"annotations": {LAST: _Now(-3)}}, 5, False),
]


@pytest.mark.parametrize("name,meta,minutes,want", IDLE_CASES, ids=[c[0] for c in IDLE_CASES])
def test_notebook_is_idle(native, name, meta, minutes, want):
    ann = {k: _rfc(v.minutes) if isinstance(v, _Now) else v for k, v in meta.get("annotations", {}).items()}
    nb = {"metadata": {**meta, "annotations": ann}} if "annotations" in meta else {"metadata": meta}
    assert native.call("notebook_is_idle", notebook=nb, cull_idle_minutes=minutes) is want


def test_notebook_recent_time(native):
    assert native.call("notebook_recent_time", times=["2024-01-01T00:00:00Z", "2024-03-01T00:00:00Z",
                                                      "2024-02-01T00:00:00Z"]) == "2024-03-01T00:00:00Z"
    assert native.call("notebook_recent_time", times=["garbage"]) == ""


def test_update_last_activity_from_kernels(native):
    kernels = [{"execution_state": "idle", "last_activity": "2024-01-01T00:00:00Z"},
               {"execution_state": "idle", "last_activity": "2024-05-01T00:00:00Z"}]
    # compareAnnotationTimeToResource: an unparsable / missing annotation is never advanced
    r = native.call("update_timestamp_from_kernels_activity", annotations={}, kernels=kernels)
    assert r["changed"] is False and LAST not in r["annotations"]
    r = native.call("update_timestamp_from_kernels_activity", annotations={LAST: "2024-02-01T00:00:00Z"}, kernels=kernels)
    assert r["changed"] is True and r["annotations"][LAST] == "2024-05-01T00:00:00Z"
    # never go backwards in time
    r = native.call("update_timestamp_from_kernels_activity", annotations={LAST: "2024-06-01T00:00:00Z"}, kernels=kernels)
    assert r["changed"] is False and r["annotations"][LAST] == "2024-06-01T00:00:00Z"
    # a busy kernel means "active now" (annotation set, reported as not-updated like the reference)
    kernels[0]["execution_state"] = "busy"
    r = native.call("update_timestamp_from_kernels_activity", annotations={LAST: "2020-01-01T00:00:00Z"}, kernels=kernels)
    assert r["changed"] is False and r["annotations"][LAST] > "2024-05-01"
    assert native.call("update_timestamp_from_kernels_activity", annotations={}, kernels=[])["changed"] is False


def test_culling_check_period(native):
    now_ms = int(dt.datetime(2024, 1, 1, 0, 10, tzinfo=dt.timezone.utc).timestamp() * 1000)
    nb = {"metadata": {"annotations": {"notebooks.kubeflow.org/last_activity_check_timestamp": "2024-01-01T00:00:00Z"}}}
    assert native.call("culling_check_period_has_passed", notebook=nb, period_s=60, now_ms=now_ms) is True
    assert native.call("culling_check_period_has_passed", notebook=nb, period_s=3600, now_ms=now_ms) is False


# ---- generation -----------------------------------------------------------------------------
def test_generate_statefulset_defaults(native):
    nb = _nb(metadata={"name": "nb1", "namespace": "ns", "uid": "u", "labels": {"a": "b"},
                       "annotations": {"x": "1", "kubectl.kubernetes.io/last-applied-configuration": "{}",
                                       "notebooks.kubeflow.org/foo": "bar"}})
    nb["spec"]["template"]["spec"]["containers"][0]["name"] = "nb1"
    sts = native.call("generate_statefulset", notebook=nb)
    tmpl = sts["spec"]["template"]
    assert sts["metadata"]["name"] == "nb1" and sts["spec"]["replicas"] == 1
    assert sts["spec"]["selector"]["matchLabels"] == {"statefulset": "nb1"}
    # ODH fork: the pod also carries the workbench label (notebook_controller.go:54)
    assert tmpl["metadata"]["labels"] == {"statefulset": "nb1", "notebook-name": "nb1", "a": "b",
                                          "opendatahub.io/workbenches": "true"}
    # Q1: kubectl / notebook annotations are not copied to the pod
    assert tmpl["metadata"]["annotations"] == {"x": "1"}
    c = tmpl["spec"]["containers"][0]
    assert c["workingDir"] == "/home/jovyan"
    assert c["ports"] == [{"containerPort": 8888, "name": "notebook-port", "protocol": "TCP"}]
    assert {"name": "NB_PREFIX", "value": "/notebook/ns/nb1"} in c["env"]
    assert tmpl["spec"]["securityContext"]["fsGroup"] == 100


def test_generate_statefulset_stopped_and_fsgroup(native):
    nb = _nb(metadata={"name": "s", "namespace": "ns", "uid": "u", "annotations": {STOP: "2024-01-01T00:00:00Z"}})
    sts = native.call("generate_statefulset", notebook=nb, options={"add_fsgroup": False})
    assert sts["spec"]["replicas"] == 0
    assert "fsGroup" not in (sts["spec"]["template"]["spec"].get("securityContext") or {})


def test_generate_service(native):
    svc = native.call("generate_service", notebook=_nb(name="nb2", ns="ns"))
    assert svc["metadata"]["name"] == "nb2"
    assert svc["spec"]["type"] == "ClusterIP"
    assert svc["spec"]["selector"] == {"statefulset": "nb2"}
    p = svc["spec"]["ports"][0]
    assert p["port"] == 80 and p["targetPort"] == 8888 and p["name"] == "http-nb2"


def test_generate_virtual_service(native):
    nb = _nb(name="nb3", ns="ns")
    vs = native.call("generate_virtual_service", notebook=nb,
                     options={"use_istio": True, "istio_gateway": "kubeflow/kubeflow-gateway", "cluster_domain": "cluster.local"})
    assert vs["metadata"]["name"] == native.call("virtual_service_name", name="nb3", namespace="ns") == "notebook-ns-nb3"
    http = vs["spec"]["http"][0]
    assert http["match"][0]["uri"]["prefix"] == "/notebook/ns/nb3/"
    assert http["rewrite"]["uri"] == "/notebook/ns/nb3/"
    assert http["route"][0]["destination"]["host"] == "nb3.ns.svc.cluster.local"
    assert vs["spec"]["gateways"] == ["kubeflow/kubeflow-gateway"]


def test_generate_virtual_service_rewrite_and_headers(native):
    nb = _nb(name="nb4", ns="ns", metadata={"name": "nb4", "namespace": "ns", "uid": "u", "annotations": {
        "notebooks.kubeflow.org/http-rewrite-uri": "/", "notebooks.kubeflow.org/http-headers-request-set": '{"X-RStudio-Root-Path": "/notebook/ns/nb4/"}'}})
    vs = native.call("generate_virtual_service", notebook=nb, options={"use_istio": True})
    http = vs["spec"]["http"][0]
    assert http["rewrite"]["uri"] == "/"
    assert http["headers"]["request"]["set"] == {"X-RStudio-Root-Path": "/notebook/ns/nb4/"}


def test_copy_statefulset_fields(native):
    a = native.call("generate_statefulset", notebook=_nb())
    b = {k: v for k, v in a.items()}
    r = native.call("copy_statefulset_fields", **{"from": a, "to": b})
    assert r["changed"] is False
    b2 = dict(a, spec=dict(a["spec"], replicas=0))
    r = native.call("copy_statefulset_fields", **{"from": a, "to": b2})
    assert r["changed"] is True and r["to"]["spec"]["replicas"] == 1
