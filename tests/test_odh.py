"""ODH platform extension: OpenshiftNotebookReconciler (N8) + Notebook webhook (N9).

Unit cases port notebook_webhook_utils_test.go (first-difference reporter); the envtest suite
odh-notebook-controller/controllers/notebook_controller_test.go:46-958 is ported as end-to-end
cases against kube-lite (routes, network policies, CA bundle, OAuth objects, service mesh,
reconciliation lock, update-pending). Runs with SET_PIPELINE_RBAC=true like the reference's
RoleBinding cases.
"""
import copy
import time
from pathlib import Path

import pytest

from kubeflow_rm_amd.client import ApiException

FIX = Path(__file__).parent / "fixtures"
NB = "kubeflow.org/v1"
LOCK = "odh-notebook-controller-lock"


# ---- unit -------------------------------------------------------------------------------------
def test_first_difference(native):
    assert native.call("json_first_difference", a=42, b=42, type="int") == ""
    d = native.call("json_first_difference", a={"spec": {"nodeName": "node1"}}, b={"spec": {"nodeName": "node2"}}, type="v1.Pod")
    assert d == "{v1.Pod}.Spec.NodeName: node1 != node2"
    d = native.call("json_first_difference", a={"containers": [{"image": "a"}]}, b={"containers": [{"image": "b"}]},
                    type="v1.PodSpec")
    assert d == "{v1.PodSpec}.Containers[0].Image: a != b"


def test_pem_validation(native):
    pem = (FIX / "test-ca.crt").read_text()
    assert native.call("pem_certificate_valid", pem=pem) is True
    assert native.call("pem_certificate_valid", pem="-----BEGIN CERTIFICATE-----\nbm90IGEgY2VydA==\n-----END CERTIFICATE-----") is False
    assert native.call("pem_certificate_valid", pem="garbage") is False


def test_pem_validation_parses_the_whole_certificate(native):
    """a well-framed DER (SEQUENCE { SEQUENCE, SEQUENCE, BIT STRING }) with garbage
    inside tbsCertificate is rejected, as x509.ParseCertificate rejects it
    (odh-notebook-controller/controllers/notebook_controller.go:301-307); so is a first block of
    another type."""
    import base64
    import textwrap

    def der(tag, body):
        n = len(body)
        ln = bytes([n]) if n < 128 else bytes([0x81, n]) if n < 256 else bytes([0x82, n >> 8, n & 255])
        return bytes([tag]) + ln + body
    tbs = der(0x30, b"\x02\x01\x05" + b"\xde\xad\xbe\xef" * 20)  # not a TBSCertificate
    alg = der(0x30, der(0x06, b"\x2a\x86\x48\x86\xf7\x0d\x01\x01\x0b") + b"\x05\x00")
    sig = der(0x03, b"\x00" + b"\x11" * 64)
    cert = der(0x30, tbs + alg + sig)
    body = "\n".join(textwrap.wrap(base64.b64encode(cert).decode(), 64))
    framed = f"-----BEGIN CERTIFICATE-----\n{body}\n-----END CERTIFICATE-----\n"
    assert native.call("pem_certificate_valid", pem=framed) is False
    good = (FIX / "test-ca.crt").read_text()
    key_first = "-----BEGIN PRIVATE KEY-----\nAAAA\n-----END PRIVATE KEY-----\n" + good
    assert native.call("pem_certificate_valid", pem=key_first) is False
    assert native.call("pem_certificate_valid", pem=good + framed) is True  # the first block decides


def _nb(name="nb", ns="ns", annotations=None, containers=None):
    return {"apiVersion": NB, "kind": "Notebook",
            "metadata": {"name": name, "namespace": ns, "annotations": annotations or {}},
            "spec": {"template": {"spec": {"containers": containers or [{"name": name, "image": "jupyter:1"}]}}}}


@pytest.mark.parametrize("value,want", [("true", True), ("True", True), ("1", True), ("t", True),
                                        ("false", False), ("yes", False), ("", False)])
def test_bool_annotations(native, value, want):
    nb = _nb(annotations={"notebooks.opendatahub.io/inject-oauth": value})
    assert native.call("odh_flags", notebook=nb)["oauth"] is want


def test_inject_oauth_proxy(native):
    nb = native.call("odh_inject_oauth_proxy", notebook=_nb(annotations={"notebooks.opendatahub.io/oauth-logout-url": "https://x/logout"}),
                     image="proxy:1")
    spec = nb["spec"]["template"]["spec"]
    proxy = [c for c in spec["containers"] if c["name"] == "oauth-proxy"][0]
    assert proxy["image"] == "proxy:1" and proxy["ports"][0]["containerPort"] == 8443
    assert "--openshift-service-account=nb" in proxy["args"] and "--logout-url=https://x/logout" in proxy["args"]
    assert proxy["readinessProbe"]["httpGet"]["path"] == "/oauth/healthz"
    assert proxy["resources"]["limits"] == {"cpu": "100m", "memory": "64Mi"}
    assert {v["name"] for v in spec["volumes"]} == {"oauth-config", "tls-certificates"}
    assert spec["serviceAccountName"] == "nb"
    # idempotent
    again = native.call("odh_inject_oauth_proxy", notebook=nb, image="proxy:1")
    assert again == nb


def test_inject_and_unset_cert_config(native):
    nb = native.call("odh_inject_cert_config", notebook=_nb(), configmap="workbench-trusted-ca-bundle")
    c = nb["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e["value"] for e in c["env"]}
    assert set(env) == {"PIP_CERT", "REQUESTS_CA_BUNDLE", "SSL_CERT_FILE", "PIPELINES_SSL_SA_CERTS", "GIT_SSL_CAINFO"}
    assert c["volumeMounts"] == [{"name": "trusted-ca", "readOnly": True, "mountPath": "/etc/pki/tls/custom-certs/ca-bundle.crt",
                                  "subPath": "ca-bundle.crt"}]
    vol = nb["spec"]["template"]["spec"]["volumes"][0]
    assert vol["configMap"]["name"] == "workbench-trusted-ca-bundle" and vol["configMap"]["optional"] is True
    r = native.call("odh_unset_cert_config", notebook=nb)
    assert r["changed"]
    c = r["notebook"]["spec"]["template"]["spec"]["containers"][0]
    assert c.get("env") == [] and c.get("volumeMounts") == []
    assert r["notebook"]["spec"]["template"]["spec"]["volumes"] == []


def test_image_from_imagestream(native):
    streams = [{"metadata": {"name": "jupyter-pytorch"}, "status": {"tags": [{"tag": "2024.1", "items": [
        {"created": "2024-01-01T00:00:00Z", "dockerImageReference": "quay.io/x@sha256:old"},
        {"created": "2024-06-01T00:00:00Z", "dockerImageReference": "quay.io/x@sha256:new"}]}]}}]
    nb = _nb(annotations={"notebooks.opendatahub.io/last-image-selection": "jupyter-pytorch:2024.1"},
             containers=[{"name": "nb", "image": "placeholder", "env": [{"name": "JUPYTER_IMAGE", "value": "old"}]}])
    r = native.call("odh_set_image_from_imagestreams", notebook=nb, imagestreams=streams)
    c = r["notebook"]["spec"]["template"]["spec"]["containers"][0]
    assert c["image"] == "quay.io/x@sha256:new" and c["env"][0]["value"] == "jupyter-pytorch:2024.1"
    bad = _nb(annotations={"notebooks.opendatahub.io/last-image-selection": "nocolon"})
    assert native.call("odh_set_image_from_imagestreams", notebook=bad, imagestreams=streams)["error"]
    internal = _nb(annotations={"notebooks.opendatahub.io/last-image-selection": "jupyter-pytorch:2024.1"},
                   containers=[{"name": "nb", "image": "image-registry.openshift-image-registry.svc:5000/ns/x:1"}])
    out = native.call("odh_set_image_from_imagestreams", notebook=internal, imagestreams=streams)
    assert out["notebook"]["spec"]["template"]["spec"]["containers"][0]["image"].startswith("image-registry")


def test_generated_objects(native):
    o = native.call("odh_objects", notebook=_nb(), controller_namespace="opendatahub")
    np = o["network_policy"]
    assert np["metadata"]["name"] == "nb-ctrl-np"
    assert np["spec"]["ingress"][0]["ports"] == [{"protocol": "TCP", "port": 8888}]
    assert np["spec"]["ingress"][0]["from"][0]["namespaceSelector"]["matchLabels"] == {"kubernetes.io/metadata.name": "opendatahub"}
    assert o["oauth_network_policy"]["spec"]["ingress"][0]["ports"][0]["port"] == 8443
    assert o["route"]["spec"]["tls"] == {"termination": "edge", "insecureEdgeTerminationPolicy": "Redirect"}
    assert o["route"]["spec"]["port"]["targetPort"] == "http-nb"
    assert o["oauth_route"]["spec"]["to"]["name"] == "nb-tls" and o["oauth_route"]["spec"]["tls"]["termination"] == "reencrypt"
    assert o["oauth_service"]["metadata"]["annotations"]["service.beta.openshift.io/serving-cert-secret-name"] == "nb-tls"
    assert len(o["oauth_secret"]["stringData"]["cookie_secret"]) > 20


# ---- end to end -----------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def cluster():
    from kubeflow_rm_amd.cluster import LocalCluster
    from tests.conftest import _ensure_native
    _ensure_native()
    cl = LocalCluster(env={"ENABLE_CULLING": "false", "USE_ISTIO": "false", "SET_PIPELINE_RBAC": "true"})
    cl.start()
    yield cl
    cl.stop()


@pytest.fixture(scope="module")
def c(cluster):
    cl = cluster.client
    cl.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "odh"}})
    return cl


def _exists(c, av, kind, name, ns="odh", timeout=10):
    return c.wait_for(av, kind, name, ns, lambda o: True, timeout=timeout)


def test_lock_injected_and_removed_route_created(c):
    created = c.create(_nb("plain", "odh"))
    assert created["metadata"]["annotations"]["kubeflow-resource-stopped"] == LOCK
    c.wait_for(NB, "Notebook", "plain", "odh",
               lambda o: "kubeflow-resource-stopped" not in (o["metadata"].get("annotations") or {}), timeout=10)
    route = _exists(c, "route.openshift.io/v1", "Route", "plain")
    assert route["spec"]["to"]["name"] == "plain" and route["metadata"]["ownerReferences"][0]["kind"] == "Notebook"
    c.wait_for(NB, "Notebook", "plain", "odh", lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=30)


def test_route_reconciled_when_modified_and_recreated(c):
    r = c.get("route.openshift.io/v1", "Route", "plain", "odh")
    r["spec"]["to"]["name"] = "hijacked"
    c.update(r)
    c.wait_for("route.openshift.io/v1", "Route", "plain", "odh", lambda o: o["spec"]["to"]["name"] == "plain", timeout=10)
    c.delete("route.openshift.io/v1", "Route", "plain", "odh")
    c.wait_for("route.openshift.io/v1", "Route", "plain", "odh",
               lambda o: o["spec"]["to"]["name"] == "plain" and not o["metadata"].get("deletionTimestamp"), timeout=10)


def test_network_policies(c):
    np = _exists(c, "networking.k8s.io/v1", "NetworkPolicy", "plain-ctrl-np")
    assert np["spec"]["podSelector"]["matchLabels"] == {"notebook-name": "plain"}
    _exists(c, "networking.k8s.io/v1", "NetworkPolicy", "plain-oauth-np")
    np["spec"]["ingress"][0]["ports"][0]["port"] = 9999
    c.update(np)
    c.wait_for("networking.k8s.io/v1", "NetworkPolicy", "plain-ctrl-np", "odh",
               lambda o: o["spec"]["ingress"][0]["ports"][0]["port"] == 8888, timeout=10)
    c.delete("networking.k8s.io/v1", "NetworkPolicy", "plain-oauth-np", "odh")
    _exists(c, "networking.k8s.io/v1", "NetworkPolicy", "plain-oauth-np")


def test_pipeline_rolebinding_only_when_role_exists(c):
    assert not c.exists("rbac.authorization.k8s.io/v1", "RoleBinding", "elyra-pipelines-plain", "odh")
    c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
              "metadata": {"name": "ds-pipeline-user-access-dspa", "namespace": "odh"},
              "rules": [{"apiGroups": [""], "resources": ["configmaps"], "verbs": ["get"]}]})
    c.create(_nb("rbac", "odh"))
    rb = _exists(c, "rbac.authorization.k8s.io/v1", "RoleBinding", "elyra-pipelines-rbac")
    assert rb["subjects"] == [{"kind": "ServiceAccount", "name": "rbac", "namespace": "odh"}]
    assert rb["roleRef"]["name"] == "ds-pipeline-user-access-dspa"
    c.delete(NB, "Notebook", "rbac", "odh")
    c.wait_gone("rbac.authorization.k8s.io/v1", "RoleBinding", "elyra-pipelines-rbac", "odh", timeout=15)


def test_trusted_ca_bundle_mounted(c):
    pem = (FIX / "test-ca.crt").read_text()
    c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "odh-trusted-ca-bundle", "namespace": "odh"},
              "data": {"ca-bundle.crt": pem, "odh-ca-bundle.crt": pem}})
    nb = c.create(_nb("withca", "odh"))
    spec = nb["spec"]["template"]["spec"]
    assert any(v["name"] == "trusted-ca" for v in spec["volumes"])
    env = {e["name"] for e in spec["containers"][0]["env"]}
    assert "REQUESTS_CA_BUNDLE" in env and "GIT_SSL_CAINFO" in env
    cm = _exists(c, "v1", "ConfigMap", "workbench-trusted-ca-bundle")
    assert cm["metadata"]["labels"] == {"opendatahub.io/managed-by": "workbenches"}
    assert "BEGIN CERTIFICATE" in cm["data"]["ca-bundle.crt"]


def test_update_pending_blocks_webhook_restart(c):
    # "plain" was created before the CA bundle existed: an unrelated update of the running
    # notebook must not silently mount it (that would restart the pod)
    c.wait_for(NB, "Notebook", "plain", "odh", lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=30)
    nb = c.patch(NB, "Notebook", "plain", {"metadata": {"labels": {"touched": "yes"}}}, "odh")
    pending = nb["metadata"]["annotations"].get("notebooks.opendatahub.io/update-pending", "")
    assert pending.startswith("{v1.PodSpec}")
    assert not any(v["name"] == "trusted-ca" for v in nb["spec"]["template"]["spec"].get("volumes", []))


def test_workbench_bundle_deleted_unmounts(c):
    def delete_if_there(name):
        try:
            c.delete("v1", "ConfigMap", name, "odh")
        except ApiException as e:
            assert e.status == 404, e
    delete_if_there("odh-trusted-ca-bundle")
    # the reconciler may already have removed the workbench bundle derived from it, or (one pass
    # still working from the old source) re-create it once more: delete until the source is gone
    # from its view too

    def unmounted(o):
        return not any(v.get("configMap", {}).get("name") == "workbench-trusted-ca-bundle"
                       for v in o["spec"]["template"]["spec"].get("volumes", []))
    deadline = time.time() + 30
    while True:
        delete_if_there("workbench-trusted-ca-bundle")
        nb = c.get(NB, "Notebook", "withca", "odh")
        if unmounted(nb):
            break
        assert time.time() < deadline, "workbench bundle still mounted"
        time.sleep(0.2)
    env = {e["name"] for e in nb["spec"]["template"]["spec"]["containers"][0].get("env", [])}
    assert "REQUESTS_CA_BUNDLE" not in env


def test_oauth_notebook(c):
    nb = c.create(_nb("secure", "odh", annotations={"notebooks.opendatahub.io/inject-oauth": "true"}))
    names = [x["name"] for x in nb["spec"]["template"]["spec"]["containers"]]
    assert names == ["secure", "oauth-proxy"]
    sa = _exists(c, "v1", "ServiceAccount", "secure")
    assert "serviceaccounts.openshift.io/oauth-redirectreference.first" in sa["metadata"]["annotations"]
    svc = _exists(c, "v1", "Service", "secure-tls")
    assert svc["spec"]["ports"][0]["port"] == 443
    sec = _exists(c, "v1", "Secret", "secure-oauth-config")
    assert sec["data"]["cookie_secret"]
    route = _exists(c, "route.openshift.io/v1", "Route", "secure")
    assert route["spec"]["tls"]["termination"] == "reencrypt" and route["spec"]["to"]["name"] == "secure-tls"
    # the SA receives a pull secret -> the reconciliation lock is released
    c.wait_for(NB, "Notebook", "secure", "odh",
               lambda o: "kubeflow-resource-stopped" not in (o["metadata"].get("annotations") or {}), timeout=10)
    # recreated when deleted
    for av, kind, name in [("v1", "Secret", "secure-oauth-config"), ("v1", "Service", "secure-tls"),
                           ("v1", "ServiceAccount", "secure")]:
        uid = c.get(av, kind, name, "odh")["metadata"]["uid"]
        c.delete(av, kind, name, "odh")
        c.wait_for(av, kind, name, "odh", lambda o, uid=uid: o["metadata"]["uid"] != uid, timeout=10)
    # deleting the notebook garbage-collects the OAuth objects
    c.delete(NB, "Notebook", "secure", "odh")
    for av, kind, name in [("v1", "Secret", "secure-oauth-config"), ("v1", "Service", "secure-tls"),
                           ("route.openshift.io/v1", "Route", "secure"), ("networking.k8s.io/v1", "NetworkPolicy", "secure-ctrl-np")]:
        c.wait_gone(av, kind, name, "odh", timeout=15)


# ---- OAuth-mode envtest cases, one named test each (notebook_controller_test.go:575-898) ----------
def _oauth_nb():
    nb = _nb("oauth-env", "odh", annotations={"notebooks.opendatahub.io/inject-oauth": "true",
                                              "notebooks.opendatahub.io/foo": "bar"})
    nb["metadata"]["labels"] = {"app.kubernetes.io/instance": "oauth-env"}
    spec = nb["spec"]["template"]["spec"]
    spec["containers"][0]["image"] = "registry.redhat.io/ubi8/ubi:latest"
    spec["volumes"] = [{"name": "notebook-data", "persistentVolumeClaim": {"claimName": "oauth-env-data"}}]
    return nb


def _oauth_spec_as_injected(nb):
    spec = nb["spec"]["template"]["spec"]
    proxy = [x for x in spec["containers"] if x["name"] == "oauth-proxy"][0]
    vols = {v["name"]: v for v in spec["volumes"]}
    return spec["serviceAccountName"], proxy["image"], vols["oauth-config"], vols["tls-certificates"]


def test_oauth_envtest_inject_sidecar_and_remove_lock(c):
    """It("Should inject the OAuth proxy as a sidecar container") / ("Should remove the
    reconciliation lock annotation"): notebook_controller_test.go:660-681."""
    nb = c.create(_oauth_nb())
    spec = nb["spec"]["template"]["spec"]
    assert [x["name"] for x in spec["containers"]] == ["oauth-env", "oauth-proxy"]
    assert spec["serviceAccountName"] == "oauth-env"
    vols = {v["name"]: v for v in spec["volumes"]}
    assert vols["oauth-config"]["secret"] == {"secretName": "oauth-env-oauth-config", "defaultMode": 420}
    assert vols["tls-certificates"]["secret"] == {"secretName": "oauth-env-tls", "defaultMode": 420}
    assert nb["metadata"]["annotations"]["kubeflow-resource-stopped"] == LOCK
    c.wait_for(NB, "Notebook", "oauth-env", "odh",
               lambda o: "kubeflow-resource-stopped" not in (o["metadata"].get("annotations") or {}), timeout=10)


def test_oauth_envtest_reconcile_notebook_when_modified(c):
    """It("Should reconcile the Notebook when modified"), notebook_controller_test.go:684-698: a
    hand edit of the SA name, the OAuth sidecar image and the oauth-config volume is undone by the
    webhook on UPDATE — the spec comes back exactly as injected."""
    for _ in range(50):  # the controllers write the Notebook too: retry the edit on a conflict
        nb = c.get(NB, "Notebook", "oauth-env", "odh")
        want = copy.deepcopy(_oauth_spec_as_injected(nb))
        spec = nb["spec"]["template"]["spec"]
        spec["serviceAccountName"] = "foo"
        [x for x in spec["containers"] if x["name"] == "oauth-proxy"][0]["image"] = "bar"
        for v in spec["volumes"]:
            if v["name"] == "oauth-config":
                v.pop("secret", None)
        try:
            out = c.update(nb)
            break
        except ApiException as e:
            if e.status != 409:
                raise
            time.sleep(0.05)
    assert _oauth_spec_as_injected(out) == want
    time.sleep(0.2)
    assert _oauth_spec_as_injected(c.get(NB, "Notebook", "oauth-env", "odh")) == want


def test_oauth_envtest_route_recreated_when_deleted(c):
    """It("Should recreate the Route when deleted"), notebook_controller_test.go:834-845."""
    r = _exists(c, "route.openshift.io/v1", "Route", "oauth-env")
    assert r["spec"]["to"] == {"kind": "Service", "name": "oauth-env-tls", "weight": 100}
    assert r["spec"]["tls"] == {"termination": "reencrypt", "insecureEdgeTerminationPolicy": "Redirect"}
    assert r["spec"]["port"]["targetPort"] == "oauth-proxy" and r["spec"]["wildcardPolicy"] == "None"
    c.delete("route.openshift.io/v1", "Route", "oauth-env", "odh")
    r2 = c.wait_for("route.openshift.io/v1", "Route", "oauth-env", "odh",
                    lambda o: o["metadata"]["uid"] != r["metadata"]["uid"] and not o["metadata"].get("deletionTimestamp"),
                    timeout=10)
    assert r2["spec"]["to"]["name"] == "oauth-env-tls" and r2["spec"]["tls"]["termination"] == "reencrypt"


def test_oauth_envtest_route_reconciled_when_modified(c):
    """It("Should reconcile the Route when modified"), notebook_controller_test.go:847-863: a merge
    patch of spec.to.name is reverted to the OAuth service."""
    c.patch("route.openshift.io/v1", "Route", "oauth-env", {"spec": {"to": {"name": "foo"}}}, "odh", "merge")
    r = c.wait_for("route.openshift.io/v1", "Route", "oauth-env", "odh",
                   lambda o: o["spec"]["to"]["name"] == "oauth-env-tls", timeout=10)
    assert r["spec"]["tls"]["termination"] == "reencrypt"


def test_oauth_envtest_delete_oauth_proxy_objects(c):
    """It("Should delete the OAuth proxy objects"), notebook_controller_test.go:865-898: the
    Notebook controller-owns the ServiceAccount, Service, Secret and Route (controller +
    blockOwnerDeletion); deleting it removes them (kube-lite runs the garbage collector that envtest
    lacks, so existence is asserted too)."""
    nb = c.get(NB, "Notebook", "oauth-env", "odh")
    want = {"apiVersion": "kubeflow.org/v1", "kind": "Notebook", "name": "oauth-env", "uid": nb["metadata"]["uid"],
            "controller": True, "blockOwnerDeletion": True}
    objs = [("v1", "ServiceAccount", "oauth-env"), ("v1", "Service", "oauth-env-tls"),
            ("v1", "Secret", "oauth-env-oauth-config"), ("route.openshift.io/v1", "Route", "oauth-env")]
    for av, kind, name in objs:
        o = _exists(c, av, kind, name)
        assert want in o["metadata"].get("ownerReferences", []), (kind, o["metadata"].get("ownerReferences"))
    c.delete(NB, "Notebook", "oauth-env", "odh")
    c.wait_gone(NB, "Notebook", "oauth-env", "odh", timeout=15)
    for av, kind, name in objs:
        c.wait_gone(av, kind, name, "odh", timeout=15)


def test_service_mesh_notebook(c):
    nb = c.create(_nb("mesh", "odh", annotations={"opendatahub.io/service-mesh": "true"}))
    assert [x["name"] for x in nb["spec"]["template"]["spec"]["containers"]] == ["mesh"]
    _exists(c, "networking.k8s.io/v1", "NetworkPolicy", "mesh-ctrl-np")
    time.sleep(0.5)
    assert not c.exists("networking.k8s.io/v1", "NetworkPolicy", "mesh-oauth-np", "odh")
    assert not c.exists("route.openshift.io/v1", "Route", "mesh", "odh")
    assert not c.exists("v1", "ServiceAccount", "mesh", "odh")
    assert not c.exists("v1", "Secret", "mesh-oauth-config", "odh")
    with pytest.raises(ApiException) as e:
        c.create(_nb("both", "odh", annotations={"opendatahub.io/service-mesh": "true",
                                                 "notebooks.opendatahub.io/inject-oauth": "true"}))
    assert "Pick one" in str(e.value.body)


# ---- e2e lifecycle (ports of odh-notebook-controller/e2e: creation, traffic, update, deletion) -----
def _via_route(cluster, host, path):
    import urllib.request
    req = urllib.request.Request(cluster.gateway + path, headers={"Host": host})
    with urllib.request.urlopen(req, timeout=5) as r:
        return r.status, r.read()


def test_e2e_lifecycle_creation_traffic_update_deletion(cluster, c):
    # creation (notebook_creation_test.go): instance, Route, NetworkPolicies, StatefulSet
    c.create(_nb("life", "odh"))
    c.wait_for(NB, "Notebook", "life", "odh", lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=30)
    route = _exists(c, "route.openshift.io/v1", "Route", "life")
    for np in ("life-ctrl-np", "life-oauth-np"):
        _exists(c, "networking.k8s.io/v1", "NetworkPolicy", np)
    sts = _exists(c, "apps/v1", "StatefulSet", "life")
    assert sts["spec"]["template"]["spec"]["containers"][0]["image"] == "jupyter:1"
    # traffic (testNotebookTraffic): the Route's host reaches the notebook server through the gateway
    # a Route without spec.host gets the router's default host <name>-<namespace>.<domain>
    host = route["spec"].get("host") or "life-odh.apps.kube-lite"
    deadline = time.time() + 15
    while True:
        try:
            status, _ = _via_route(cluster, host, "/notebook/odh/life/api/status")
            break
        except Exception:
            if time.time() > deadline:
                raise
            time.sleep(0.2)
    assert status == 200
    # update (notebook_update_test.go): a new image reaches the StatefulSet and its pod
    nb = c.get(NB, "Notebook", "life", "odh")
    nb["spec"]["template"]["spec"]["containers"][0]["image"] = "jupyter-minimal:2"
    c.update(nb)
    c.wait_for("apps/v1", "StatefulSet", "life", "odh",
               lambda o: o["spec"]["template"]["spec"]["containers"][0]["image"] == "jupyter-minimal:2", timeout=15)
    c.wait_for("v1", "Pod", "life-0", "odh",
               lambda o: o["spec"]["containers"][0]["image"] == "jupyter-minimal:2"
               and any(cd["type"] == "Ready" and cd["status"] == "True" for cd in (o.get("status") or {}).get("conditions", [])),
               timeout=30)
    assert _exists(c, "route.openshift.io/v1", "Route", "life")["spec"]["to"]["name"] == "life"
    # deletion (notebook_deletion_test.go): the owned StatefulSet, NetworkPolicies and Route go with it
    c.delete(NB, "Notebook", "life", "odh")
    c.wait_gone(NB, "Notebook", "life", "odh", timeout=20)
    for av, kind, name in (("apps/v1", "StatefulSet", "life"), ("networking.k8s.io/v1", "NetworkPolicy", "life-ctrl-np"),
                           ("networking.k8s.io/v1", "NetworkPolicy", "life-oauth-np"), ("route.openshift.io/v1", "Route", "life")):
        c.wait_gone(av, kind, name, "odh", timeout=20)
