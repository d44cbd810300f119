"""KFAM access-management REST service (native).

Ports access-management/kfam/bindings_test.go:25-61 (binding names) and drives the REST API
(api_default.go) against kube-lite: owner/admin gating, RoleBinding + AuthorizationPolicy pairs,
listing with filters, profile create/delete, cluster-admin query, metrics.
"""
import json
import urllib.request

import pytest


@pytest.mark.parametrize("user,out", [
    ("lalith.vaka@zq.msds.kp.org", "user-lalith-vaka-zq-msds-kp-org-clusterrole-edit"),
    ("397401@zq.msds.kp.org", "user-397401-zq-msds-kp-org-clusterrole-edit"),
    ("lalith.397401@zq.msds.kp.org", "user-lalith-397401-zq-msds-kp-org-clusterrole-edit"),
    ("397401.vaka@zq.msds.kp.org", "user-397401-vaka-zq-msds-kp-org-clusterrole-edit"),
    ("i397401@zq.msds.kp.org", "user-i397401-zq-msds-kp-org-clusterrole-edit"),
])
def test_get_binding_name(native, user, out):
    b = {"user": {"kind": "User", "name": user}, "RoleRef": {"kind": "clusterrole", "name": "edit"}}
    assert native.call("kfam_binding_name", binding=b) == out


def test_role_map(native):
    for a, b in [("admin", "kubeflow-admin"), ("edit", "kubeflow-edit"), ("view", "kubeflow-view")]:
        assert native.call("kfam_role_map", role=a) == b and native.call("kfam_role_map", role=b) == a


def _req(base, method, path, body=None, user=None):
    data = json.dumps(body).encode() if body is not None else None
    r = urllib.request.Request(base + path, data=data, method=method)
    if user:
        r.add_header("kubeflow-userid", user)
    try:
        with urllib.request.urlopen(r, timeout=5) as resp:
            return resp.status, resp.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


@pytest.fixture(scope="module")
def kfam(cluster):
    assert cluster.kfam, "kflite did not start KFAM"
    return cluster.kfam


def test_kfam_flow(kfam, cluster):
    c = cluster.client
    assert _req(kfam, "GET", "/kfam/") == (200, "Hello World!")
    prof = {"metadata": {"name": "team-a"}, "spec": {"owner": {"kind": "User", "name": "owner@example.com"}}}
    assert _req(kfam, "POST", "/kfam/v1/profiles", prof)[0] == 200
    c.wait_for("v1", "Namespace", "team-a", None, lambda o: True, timeout=10)
    c.wait_for("rbac.authorization.k8s.io/v1", "RoleBinding", "namespaceAdmin", "team-a", lambda o: True, timeout=10)
    binding = {"user": {"kind": "User", "name": "bob@example.com"}, "referredNamespace": "team-a",
               "RoleRef": {"kind": "ClusterRole", "name": "edit"}}
    # non-owner cannot share
    assert _req(kfam, "POST", "/kfam/v1/bindings", binding, user="mallory@example.com")[0] == 403
    assert _req(kfam, "POST", "/kfam/v1/bindings", binding, user="owner@example.com")[0] == 200
    name = "user-bob-example-com-clusterrole-edit"
    rb = c.get("rbac.authorization.k8s.io/v1", "RoleBinding", name, "team-a")
    assert rb["roleRef"]["name"] == "kubeflow-edit" and rb["metadata"]["annotations"] == {"user": "bob@example.com", "role": "edit"}
    ap = c.get("security.istio.io/v1beta1", "AuthorizationPolicy", name, "team-a")
    assert ap["spec"]["rules"][0]["when"][0] == {"key": "request.headers[kubeflow-userid]", "values": ["bob@example.com"]}
    # RBAC now lets bob edit notebooks in team-a
    assert c.subject_access_review("bob@example.com", "create", "kubeflow.org", "notebooks", "team-a")["status"]["allowed"]
    # list: all profile namespaces, filtered by user / role
    code, body = _req(kfam, "GET", "/kfam/v1/bindings?user=bob@example.com")
    assert code == 200
    got = json.loads(body)["bindings"]
    assert got == [{"user": {"kind": "User", "name": "bob@example.com"}, "referredNamespace": "team-a",
                    "RoleRef": {"kind": "ClusterRole", "name": "edit"}}]
    code, body = _req(kfam, "GET", "/kfam/v1/bindings?namespace=team-a&role=admin")
    owners = [b["user"]["name"] for b in json.loads(body)["bindings"]]
    assert owners == ["owner@example.com"]
    # delete binding
    assert _req(kfam, "DELETE", "/kfam/v1/bindings", binding, user="owner@example.com")[0] == 200
    assert not c.exists("rbac.authorization.k8s.io/v1", "RoleBinding", name, "team-a")
    assert not c.exists("security.istio.io/v1beta1", "AuthorizationPolicy", name, "team-a")
    # cluster admin query + profile deletion gating
    assert _req(kfam, "GET", "/kfam/v1/role/clusteradmin?user=nobody@example.com") == (200, "false")
    assert _req(kfam, "DELETE", "/kfam/v1/profiles/team-a", user="mallory@example.com")[0] == 401
    assert _req(kfam, "DELETE", "/kfam/v1/profiles/team-a", user="owner@example.com")[0] == 200
    c.wait_gone("kubeflow.org/v1", "Profile", "team-a", None, timeout=15)
    code, metrics = _req(kfam, "GET", "/metrics")
    assert code == 200 and 'request_kf{component="kfam"' in metrics and "service_heartbeat" in metrics
