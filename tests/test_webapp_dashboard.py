"""Central dashboard backend.

Ports the reference's app tests (api_test.ts: metrics 405 / series / intervals; k8s_service_test.ts:
namespaces / events / nodes, empty on error, platform info known / other / unknown / defaults;
attach_user_middleware_test.ts; api_workgroup_test.ts: env-info, exists, create, contributors,
KFAM failure surfacing) with a fake KFAM + metrics service, then runs the whole workgroup flow
against the real native KFAM and kube-lite (registration -> owner namespace -> contributor add /
remove -> nuke-self).
"""
import json
import time

import pytest

from kubeflow_rm_amd.webapps import dashboard
from kubeflow_rm_amd.webapps.dashboard.services import KfamError, LocalMetricsService


class FakeKfam:
    def __init__(self):
        self.bindings = []
        self.admins = set()
        self.calls = []
        self.fail = None

    def _check(self):
        if self.fail:
            raise KfamError(*self.fail)

    def read_bindings(self, user=None, namespace=None, role=None):
        self._check()
        return [b for b in self.bindings if (not user or b["user"]["name"] == user)
                and (not namespace or b["referredNamespace"] == namespace)]

    def is_cluster_admin(self, user):
        self._check()
        return user in self.admins

    def create_binding(self, b, headers):
        self._check()
        self.calls.append(("create_binding", b, headers))
        self.bindings.append(b)

    def delete_binding(self, b, headers):
        self._check()
        self.calls.append(("delete_binding", b, headers))
        self.bindings = [x for x in self.bindings if x != b]

    def create_profile(self, p, headers=None):
        self._check()
        self.calls.append(("create_profile", p))

    def delete_profile(self, name, headers):
        self._check()
        self.calls.append(("delete_profile", name, headers))
        return ""


class FakeMetrics:
    def __init__(self):
        self.asked = []

    def series(self, kind, interval):
        self.asked.append((kind, interval))
        return [{"timestamp": 1.0, "label": kind, "value": 0.5}]

    def charts_link(self):
        return {"resourceChartsLink": "http://grafana/d/x", "resourceChartsLinkText": "View in dashboard"}


class FakeK8s:
    def list(self, av, kind, ns=None, **kw):
        if kind == "Node":
            return {"items": [{"metadata": {"name": "n0"}, "spec": {"providerID": "kfamd://mi355x/n0"}}]}
        if kind == "Namespace":
            return {"items": [{"metadata": {"name": "a"}}, {"metadata": {"name": "b"}}]}
        if kind == "Event":
            return {"items": [{"metadata": {"name": "e", "namespace": ns}, "message": "hi"}]}
        if kind == "Application":
            return {"items": [{"spec": {"descriptor": {"type": "Kubeflow", "version": "1.9-mi355x"}}}]}
        return {"items": []}

    def get(self, av, kind, name, ns=None):
        return {"data": {"links": json.dumps({"menuLinks": [{"type": "item", "link": "/jupyter/", "text": "Notebooks"}]}),
                         "settings": json.dumps({"DASHBOARD_FORCE_IFRAME": True})}}


def _binding(user, ns, role):
    return {"user": {"kind": "User", "name": user}, "referredNamespace": ns, "roleRef": {"kind": "ClusterRole", "name": role}}


@pytest.fixture
def fake_app(monkeypatch):
    monkeypatch.setenv("USERID_HEADER", "kubeflow-userid")
    monkeypatch.setenv("USERID_PREFIX", "")
    kfam, metrics = FakeKfam(), FakeMetrics()
    monkeypatch.setattr(dashboard, "KfamClient", lambda url: kfam)
    app = dashboard.create_app(k8s_client=FakeK8s(), kfam_url="http://unused/kfam", metrics=metrics)
    return app.test_client(), kfam, metrics


U = {"kubeflow-userid": "alice@example.com"}


def test_attach_user(fake_app):
    tc, _, _ = fake_app
    d = tc.get("/debug", headers=U).get_json()["user"]
    assert d == {"email": "alice@example.com", "username": "alice", "domain": "example.com", "hasAuth": True,
                 "auth": {"kubeflow-userid": "alice@example.com"}}
    d = tc.get("/debug").get_json()["user"]
    assert d["email"] == "anonymous@kubeflow.org" and d["hasAuth"] is False and d["auth"] is None


def test_metrics_routes(fake_app):
    tc, _, metrics = fake_app
    assert tc.get("/api/metrics").get_json()["resourceChartsLink"] == "http://grafana/d/x"
    assert tc.get("/api/metrics/node").get_json()[0]["label"] == "node"
    tc.get("/api/metrics/podcpu")
    tc.get("/api/metrics/podmem?interval=Last180m")
    tc.get("/api/metrics/gpu?interval=bogus")
    assert metrics.asked == [("node", "Last15m"), ("podcpu", "Last15m"), ("podmem", "Last180m"), ("gpu", "Last15m")]
    assert tc.get("/api/metrics/disk").status_code == 404


def test_metrics_without_service(monkeypatch):
    monkeypatch.delenv("PROMETHEUS_URL", raising=False)
    monkeypatch.delenv("METRICS_PROVIDER", raising=False)
    tc = dashboard.create_app(k8s_client=FakeK8s(), kfam_url="http://unused/kfam").test_client()
    for p in ("/api/metrics", "/api/metrics/node", "/api/metrics/podmem"):
        r = tc.get(p)
        assert r.status_code == 405 and r.get_json() == {"error": "Operation not supported"}


def test_namespaces_activities_links_settings(fake_app):
    tc, _, _ = fake_app
    assert [n["metadata"]["name"] for n in tc.get("/api/namespaces").get_json()] == ["a", "b"]
    assert tc.get("/api/activities/a").get_json()[0]["message"] == "hi"
    assert tc.get("/api/dashboard-links").get_json()["menuLinks"][0]["link"] == "/jupyter/"
    assert tc.get("/api/dashboard-settings").get_json() == {"DASHBOARD_FORCE_IFRAME": True}
    assert tc.get("/api/nothing").status_code == 404
    assert b"<html" in tc.get("/_/jupyter/").data and b"CentralDashboardEventHandler" in tc.get("/library.js").data


def test_env_info_identity_and_basic(fake_app):
    tc, kfam, _ = fake_app
    kfam.bindings = [_binding("alice@example.com", "alice", "admin"), _binding("alice@example.com", "team", "edit"),
                     _binding("bob@example.com", "bob", "admin")]
    kfam.admins = {"alice@example.com"}
    d = tc.get("/api/workgroup/env-info", headers=U).get_json()
    assert d["user"] == "alice@example.com" and d["isClusterAdmin"] is True
    assert d["namespaces"] == [{"user": "alice@example.com", "namespace": "alice", "role": "owner"},
                               {"user": "alice@example.com", "namespace": "team", "role": "contributor"}]
    assert d["platform"] == {"kubeflowVersion": "1.9-mi355x", "provider": "kfamd://mi355x/n0",
                             "providerName": "kfamd", "logoutUrl": "/logout"}
    d = tc.get("/api/workgroup/env-info").get_json()
    assert d["isClusterAdmin"] is True and d["user"] == "anonymous@kubeflow.org"
    assert [n["namespace"] for n in d["namespaces"]] == ["alice", "bob", "team"]
    assert all(n["role"] == "contributor" for n in d["namespaces"])
    kfam.fail = (500, "kfam down")
    r = tc.get("/api/workgroup/env-info", headers=U)
    assert r.status_code == 500 and r.get_json() == {"error": "kfam down"}


def test_exists(fake_app):
    tc, kfam, _ = fake_app
    assert tc.get("/api/workgroup/exists").get_json() == {"hasAuth": False, "user": "anonymous", "hasWorkgroup": False,
                                                          "registrationFlowAllowed": True}
    kfam.bindings = [_binding("alice@example.com", "team", "edit")]
    assert tc.get("/api/workgroup/exists", headers=U).get_json()["hasWorkgroup"] is False
    kfam.bindings.append(_binding("alice@example.com", "alice", "admin"))
    d = tc.get("/api/workgroup/exists", headers=U).get_json()
    assert d == {"hasAuth": True, "user": "alice", "hasWorkgroup": True, "registrationFlowAllowed": True}


def test_create_workgroup(fake_app):
    tc, kfam, _ = fake_app
    assert tc.post("/api/workgroup/create", headers=U).get_json() == {"message": "Created namespace alice"}
    assert kfam.calls[-1] == ("create_profile", {"metadata": {"name": "alice"},
                                                 "spec": {"owner": {"kind": "User", "name": "alice@example.com"}}})
    tc.post("/api/workgroup/create", headers=U, json={"namespace": "ml", "user": "bob@example.com"})
    assert kfam.calls[-1][1]["metadata"]["name"] == "ml" and kfam.calls[-1][1]["spec"]["owner"]["name"] == "bob@example.com"
    kfam.fail = (409, "already exists")
    r = tc.post("/api/workgroup/create", headers=U)
    assert r.status_code == 409 and r.get_json()["error"] == "already exists"


def test_contributors(fake_app):
    tc, kfam, _ = fake_app
    assert tc.post("/api/workgroup/add-contributor/alice", json={"contributor": "x@y.z"}).status_code == 405
    r = tc.post("/api/workgroup/add-contributor/alice", headers=U, json={})
    assert r.status_code == 400 and r.get_json()["error"] == "Missing contributor field."
    r = tc.post("/api/workgroup/add-contributor/alice", headers=U, json={"contributor": "not-an-email"})
    assert r.get_json()["error"] == "Contributor doesn't look like a valid email address"
    r = tc.post("/api/workgroup/add-contributor/alice", headers={**U, "X-Other": "drop", "Authorization": "Bearer t"},
                json={"contributor": "bob@example.com"})
    assert r.status_code == 200 and r.get_json() == ["bob@example.com"]
    name, binding, headers = kfam.calls[-1]
    assert name == "create_binding" and binding == _binding("bob@example.com", "alice", "edit")
    assert {k.lower() for k in headers} == {"kubeflow-userid", "authorization"}
    r = tc.delete("/api/workgroup/remove-contributor/alice", headers=U, json={"contributor": "bob@example.com"})
    assert r.get_json() == [] and kfam.calls[-1][0] == "delete_binding"
    kfam.bindings = [_binding("alice@example.com", "alice", "admin"), _binding("bob@example.com", "alice", "edit")]
    assert tc.get("/api/workgroup/get-all-namespaces", headers=U).get_json() == [["alice", "alice@example.com", "bob@example.com"]]
    assert tc.get("/api/workgroup/get-contributors/alice", headers=U).get_json() == ["bob@example.com"]
    assert tc.delete("/api/workgroup/nuke-self", headers=U).get_json()["message"] == "Removed namespace/profile alice"


def test_local_metrics_sampler():
    svc = LocalMetricsService(dashboard.KubernetesService(FakeK8s()), period=3600)
    svc.sample_once()
    svc.stop()
    assert svc.series("node", "Last5m") and svc.series("podmem", "Last5m")


# ---- against the native KFAM + kube-lite ------------------------------------------------------
def test_workgroup_flow_against_kfam(cluster, monkeypatch):
    monkeypatch.setenv("USERID_HEADER", "kubeflow-userid")
    monkeypatch.setenv("USERID_PREFIX", "")
    monkeypatch.setenv("METRICS_PROVIDER", "local")
    app = dashboard.create_app(k8s_client=cluster.client, kfam_url=cluster.kfam + "/kfam")
    tc = app.test_client()
    carol = {"kubeflow-userid": "carol@example.com"}
    assert tc.get("/api/workgroup/exists", headers=carol).get_json()["hasWorkgroup"] is False
    assert tc.post("/api/workgroup/create", headers=carol).status_code == 200
    cluster.client.wait_for("rbac.authorization.k8s.io/v1", "RoleBinding", "namespaceAdmin", "carol", lambda o: True, timeout=15)
    deadline = time.time() + 15
    while not tc.get("/api/workgroup/exists", headers=carol).get_json()["hasWorkgroup"] and time.time() < deadline:
        time.sleep(0.2)
    env = tc.get("/api/workgroup/env-info", headers=carol).get_json()
    assert {"user": "carol@example.com", "namespace": "carol", "role": "owner"} in env["namespaces"]
    assert env["isClusterAdmin"] is False
    r = tc.post("/api/workgroup/add-contributor/carol", headers=carol, json={"contributor": "dave@example.com"})
    assert r.status_code == 200 and r.get_json() == ["dave@example.com"], r.get_json()
    # dave now sees carol's namespace as a contributor and may create notebooks there
    dave = tc.get("/api/workgroup/env-info", headers={"kubeflow-userid": "dave@example.com"}).get_json()
    assert {"user": "dave@example.com", "namespace": "carol", "role": "contributor"} in dave["namespaces"]
    sar = cluster.client.subject_access_review("dave@example.com", "create", "kubeflow.org", "notebooks", "carol")
    assert sar["status"]["allowed"] is True
    # a non-owner cannot add contributors (KFAM 403 surfaced)
    r = tc.post("/api/workgroup/add-contributor/carol", headers={"kubeflow-userid": "dave@example.com"},
                json={"contributor": "eve@example.com"})
    assert r.status_code == 403
    r = tc.delete("/api/workgroup/remove-contributor/carol", headers=carol, json={"contributor": "dave@example.com"})
    assert r.status_code == 200 and r.get_json() == []
    # metrics from the in-process sampler: MI355X allocation on the synthetic 8-GPU node
    svc = app.extensions["kfamd-dashboard"]["metrics"]
    svc.sample_once()
    gpu = tc.get("/api/metrics/gpu").get_json()
    assert gpu and all(0.0 <= p["value"] <= 1.0 for p in gpu)
    svc.stop()
    assert tc.delete("/api/workgroup/nuke-self", headers=carol).status_code == 200
    cluster.client.wait_gone("kubeflow.org/v1", "Profile", "carol", None, timeout=20)


# ---- KubernetesService (ports of k8s_service_test.ts) ------------------------------------------
class ScriptedK8s:
    """list() answers from a {kind: items | exception} table (the reference's mocked CoreV1Api)."""

    def __init__(self, table):
        self.table = table

    def list(self, av, kind, ns=None, **kw):
        v = self.table.get(kind, [])
        if isinstance(v, Exception):
            raise v
        return {"items": v}


def _node(provider=None):
    spec = {"podCIDR": "10.44.1.0/24"}
    if provider:
        spec["providerID"] = provider
    return {"apiVersion": "v1", "kind": "Node", "spec": spec}


GCE = "gce://kubeflow-dev/us-east1-d/gke-kubeflow-default-pool-59885f2c-08tm"
KF_APP = {"apiVersion": "app.k8s.io/v1beta1", "kind": "Application", "spec": {"descriptor": {"type": "kubeflow", "version": "1.0.0"}}}


def test_k8s_service_namespaces_events_nodes_and_errors():
    from kubeflow_rm_amd.client import ApiException
    ok = dashboard.KubernetesService(ScriptedK8s({
        "Namespace": [{"metadata": {"name": "default"}}, {"metadata": {"name": "kubeflow"}}],
        "Event": [{"metadata": {"name": "e1"}, "reason": "Scheduled"}],
        "Node": [_node(GCE), _node(GCE.replace("08tm", "r72s"))]}))
    assert [n["metadata"]["name"] for n in ok.get_namespaces()] == ["default", "kubeflow"]   # Returns all namespaces
    assert ok.get_events("kubeflow")[0]["reason"] == "Scheduled"                             # Returns events
    assert len(ok.get_nodes()) == 2                                                          # Returns all Nodes
    err = ApiException(500, "testing-error", None)
    bad = dashboard.KubernetesService(ScriptedK8s({"Namespace": err, "Event": err, "Node": err}))
    assert bad.get_namespaces() == [] and bad.get_events("kubeflow") == [] and bad.get_nodes() == []  # empty on error


@pytest.mark.parametrize("nodes,apps,want", [
    ([_node(GCE), _node(GCE)], [KF_APP], {"provider": GCE, "providerName": "gce", "kubeflowVersion": "1.0.0"}),
    ([_node(), _node()], [KF_APP], {"provider": "other://", "providerName": "other", "kubeflowVersion": "1.0.0"}),
    ([_node(GCE)], [], {"provider": GCE, "providerName": "gce", "kubeflowVersion": "unknown"}),
    ("error", "error", {"provider": "other://", "providerName": "other", "kubeflowVersion": "unknown"}),
], ids=["known provider and version", "no providerID -> other", "no Application -> unknown", "defaults on error"])
def test_k8s_service_platform_info(nodes, apps, want, monkeypatch):
    from kubeflow_rm_amd.client import ApiException
    monkeypatch.delenv("LOGOUT_URL", raising=False)
    err = ApiException(500, "testing-error", None)
    svc = dashboard.KubernetesService(ScriptedK8s({"Node": err if nodes == "error" else nodes,
                                                  "Application": err if apps == "error" else apps}))
    assert svc.get_platform_info() == {**want, "logoutUrl": "/logout"}
