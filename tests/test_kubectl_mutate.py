"""kfctl's writing verbs (create / patch / annotate / label / scale) against kube-lite, replaying the
reference CI's kubectl sequence:

* ``.github/workflows/odh_notebook_controller_integration_test.yaml:132,168`` ``kubectl create ns``;
* ``:195,198`` ``kubectl create secret tls [-n NS] NAME --cert=... --key=...`` with an openssl CA and
  serving certificate made the way the workflow makes them (``:189-192``);
* ``:212`` ``kubectl patch MutatingWebhookConfiguration/... --type=json -p=<caBundle replace>``;
* ``:233-280`` the Notebook apply / rollout / wait, then the SURVEY §2.9.3 annotation protocol from
  the CLI: ``kubeflow-resource-stopped`` scales the StatefulSet to 0, ``KEY-`` brings it back, and an
  existing annotation with a different value is an error unless ``--overwrite`` (kubectl's rule).
"""
import base64
import json
import os
import subprocess
import time

import pytest

from kubeflow_rm_amd.cluster import LocalCluster
from tests.test_kubectl_cli import NB_YAML, kfctl

OPENSSL = "/usr/bin/openssl"

MWC = """
apiVersion: admissionregistration.k8s.io/v1
kind: MutatingWebhookConfiguration
metadata:
  name: odh-notebook-controller-mutating-webhook-configuration
webhooks:
- name: notebooks.opendatahub.io
  admissionReviewVersions: [v1]
  sideEffects: None
  failurePolicy: Ignore
  clientConfig:
    service: {name: odh-notebook-controller-webhook-service, namespace: opendatahub, path: /mutate-notebook-v1}
  rules:
  - apiGroups: [kubeflow.org]
    apiVersions: [v1]
    operations: [CONNECT]
    resources: [notebooks]
"""

DEPLOY = """
apiVersion: apps/v1
kind: Deployment
metadata: {name: web, namespace: opendatahub}
spec:
  replicas: 1
  selector: {matchLabels: {app: web}}
  template:
    metadata: {labels: {app: web}}
    spec:
      containers: [{name: web, image: busybox, command: [sleep, "3600"]}]
"""


@pytest.fixture(scope="module")
def cl():
    from tests.conftest import _ensure_native
    _ensure_native()
    with LocalCluster() as c:
        yield c


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    if not os.path.exists(OPENSSL):
        pytest.skip("openssl CLI not installed")
    d = str(tmp_path_factory.mktemp("pki"))

    def run(*a):
        subprocess.run([OPENSSL, *a], cwd=d, check=True, capture_output=True)
    # odh_notebook_controller_integration_test.yaml:189-192 (rsa:2048 instead of 4096 to keep it quick)
    run("req", "-nodes", "-x509", "-newkey", "rsa:2048", "-sha256", "-days", "2", "-keyout", "ca-key.pem",
        "-out", "ca-cert.pem", "-subj", "/CN=TestCA")
    run("req", "-nodes", "-newkey", "rsa:2048", "-keyout", "server-key.pem", "-out", "server-csr.pem",
        "-subj", "/CN=ServerC", "-addext",
        "subjectAltName = DNS:odh-notebook-controller-webhook-service.opendatahub.svc")
    run("x509", "-req", "-in", "server-csr.pem", "-CA", "ca-cert.pem", "-CAkey", "ca-key.pem",
        "-out", "server-cert.pem", "-days", "2", "-CAcreateserial")
    return d


def test_create_namespaces_and_tls_secrets(cl, pki):
    rc, out, err = kfctl(cl, "create", "ns", "opendatahub")
    assert rc == 0 and out.strip() == "namespace/opendatahub created", (out, err)
    # kube-lite's platform bootstrap already made `kubeflow` (the workflow's :132 runs on a bare kind cluster)
    rc, out, err = kfctl(cl, "create", "namespace", "kubeflow")
    assert rc == 1 and ("AlreadyExists" in err or "already exists" in err), err
    cert, key = os.path.join(pki, "server-cert.pem"), os.path.join(pki, "server-key.pem")
    rc, out, err = kfctl(cl, "create", "secret", "tls", "-n", "opendatahub", "odh-notebook-controller-webhook-cert",
                         f"--cert={cert}", f"--key={key}")
    assert rc == 0 and out.strip() == "secret/odh-notebook-controller-webhook-cert created", (out, err)
    rc, out, err = kfctl(cl, "create", "secret", "tls", "minimal-notebook-tls", f"--cert={cert}", f"--key={key}")
    assert rc == 0, err
    s = cl.client.get("v1", "Secret", "odh-notebook-controller-webhook-cert", "opendatahub")
    assert s["type"] == "kubernetes.io/tls"
    with open(cert, "rb") as f:
        assert base64.b64decode(s["data"]["tls.crt"]) == f.read()
    assert "tls.key" in cl.client.get("v1", "Secret", "minimal-notebook-tls", "default")["data"]
    # not PEM -> refused before anything is sent
    notpem = os.path.join(pki, "not.pem")
    with open(notpem, "w") as f:
        f.write("just text\n")
    rc, _, err = kfctl(cl, "create", "secret", "tls", "bad", f"--cert={notpem}", f"--key={key}")
    assert rc == 1 and "not PEM" in err, err
    rc, _, err = kfctl(cl, "create", "secret", "tls", "bad", f"--cert={notpem}.missing", f"--key={key}")
    assert rc == 1 and err.startswith("error: open ") and "no such file" in err, err
    rc, out, err = kfctl(cl, "create", "secret", "generic", "creds", "--from-literal=user=alice", "-n", "opendatahub")
    assert rc == 0, err
    assert base64.b64decode(cl.client.get("v1", "Secret", "creds", "opendatahub")["data"]["user"]) == b"alice"
    rc, out, err = kfctl(cl, "create", "configmap", "cfg", "--from-literal=ENABLE_CULLING=true", "-n", "opendatahub")
    assert rc == 0 and cl.client.get("v1", "ConfigMap", "cfg", "opendatahub")["data"] == {"ENABLE_CULLING": "true"}


def test_patch_webhook_ca_bundle_json(cl, pki):
    rc, out, err = kfctl(cl, "apply", "-f", "-", stdin=MWC)
    assert rc == 0, err
    with open(os.path.join(pki, "ca-cert.pem"), "rb") as f:
        ca_b64 = base64.b64encode(f.read()).decode()
    # odh_notebook_controller_integration_test.yaml:207-212, verbatim form
    bundle_patch = json.dumps([{"op": "replace", "path": "/webhooks/0/clientConfig/caBundle", "value": ca_b64}])
    rc, out, err = kfctl(cl, "patch",
                         "MutatingWebhookConfiguration/odh-notebook-controller-mutating-webhook-configuration",
                         "--type=json", f"-p={bundle_patch}")
    assert rc == 0, err
    assert out.strip() == ("mutatingwebhookconfiguration.admissionregistration.k8s.io/"
                           "odh-notebook-controller-mutating-webhook-configuration patched")
    got = cl.client.get("admissionregistration.k8s.io/v1", "MutatingWebhookConfiguration",
                        "odh-notebook-controller-mutating-webhook-configuration")
    assert got["webhooks"][0]["clientConfig"]["caBundle"] == ca_b64
    # the same patch again: kubectl prints "(no change)"
    rc, out, err = kfctl(cl, "patch", "mutatingwebhookconfiguration",
                         "odh-notebook-controller-mutating-webhook-configuration", "--type", "json", "-p", bundle_patch)
    assert rc == 0 and out.strip().endswith("patched (no change)"), (out, err)
    # a json patch against a missing path is a server-side error, not a silent success
    rc, _, err = kfctl(cl, "patch", "mutatingwebhookconfiguration/odh-notebook-controller-mutating-webhook-configuration",
                       "--type=json", "-p", '[{"op":"replace","path":"/webhooks/7/name","value":"x"}]')
    assert rc == 1, err
    rc, _, err = kfctl(cl, "patch", "ns/kubeflow", "--type=bogus", "-p", "{}")
    assert rc != 0 and "--type must be one of" in err


def test_notebook_stop_restart_by_annotation(cl):
    rc, out, err = kfctl(cl, "apply", "-f", "-", "-n", "default", stdin=NB_YAML)
    assert rc == 0, err
    deadline = time.time() + 100
    while kfctl(cl, "get", "statefulset", "minimal-notebook")[0] != 0:
        assert time.time() < deadline
        time.sleep(0.2)
    rc, out, err = kfctl(cl, "rollout", "status", "--watch", "statefulset", "minimal-notebook", "--timeout=300s")
    assert rc == 0, err
    rc, out, err = kfctl(cl, "wait", "pods", "minimal-notebook-0", "--for=condition=Ready", "--timeout=100s")
    assert rc == 0, (out, err)

    ts = "2026-10-17T00:00:00Z"
    rc, out, err = kfctl(cl, "annotate", "notebook", "minimal-notebook", f"kubeflow-resource-stopped={ts}")
    assert rc == 0 and out.strip() == "notebook.kubeflow.org/minimal-notebook annotated", (out, err)
    rc, out, err = kfctl(cl, "wait", "statefulset", "minimal-notebook", "--for=jsonpath={.spec.replicas}=0",
                         "--timeout=60s")
    assert rc == 0, (out, err)
    rc, out, err = kfctl(cl, "wait", "pods", "minimal-notebook-0", "--for=delete", "--timeout=60s")
    assert rc == 0, err
    # kubectl: a different value for an existing key needs --overwrite; the same value is a no-op
    rc, out, err = kfctl(cl, "annotate", "notebooks/minimal-notebook", "kubeflow-resource-stopped=later")
    assert rc == 1 and "--overwrite is false" in err and "kubeflow-resource-stopped" in err, err
    rc, out, err = kfctl(cl, "annotate", "notebooks/minimal-notebook", f"kubeflow-resource-stopped={ts}")
    assert rc == 0, err
    rc, out, err = kfctl(cl, "annotate", "--overwrite", "notebooks/minimal-notebook", "kubeflow-resource-stopped=later")
    assert rc == 0, err
    ann = cl.client.get("kubeflow.org/v1", "Notebook", "minimal-notebook", "default")["metadata"]["annotations"]
    assert ann["kubeflow-resource-stopped"] == "later"
    # KEY- removes it: the notebook restarts
    rc, out, err = kfctl(cl, "annotate", "notebook", "minimal-notebook", "kubeflow-resource-stopped-")
    assert rc == 0, err
    assert "kubeflow-resource-stopped" not in (cl.client.get("kubeflow.org/v1", "Notebook", "minimal-notebook",
                                                             "default")["metadata"].get("annotations") or {})
    rc, out, err = kfctl(cl, "wait", "statefulset", "minimal-notebook", "--for=jsonpath={.spec.replicas}=1",
                         "--timeout=60s")
    assert rc == 0, (out, err)
    rc, out, err = kfctl(cl, "wait", "pods", "minimal-notebook-0", "--for=condition=Ready", "--timeout=100s")
    assert rc == 0, (out, err)


def test_label_and_selector(cl):
    rc, out, err = kfctl(cl, "label", "ns", "opendatahub", "tier=gpu")
    assert rc == 0 and out.strip() == "namespace/opendatahub labeled", (out, err)
    assert cl.client.get("v1", "Namespace", "opendatahub")["metadata"]["labels"]["tier"] == "gpu"
    rc, out, err = kfctl(cl, "label", "ns", "opendatahub", "tier=cpu")
    assert rc == 1 and "--overwrite is false" in err
    rc, out, err = kfctl(cl, "label", "ns", "opendatahub", "tier=gpu")
    assert rc == 0 and out.strip() == "namespace/opendatahub not labeled", out
    rc, out, err = kfctl(cl, "label", "configmaps", "-n", "opendatahub", "--all", "owner=odh")
    assert rc == 0 and "configmap/cfg labeled" in out, (out, err)
    rc, out, err = kfctl(cl, "annotate", "configmaps", "-n", "opendatahub", "-l", "owner=odh", "note=x")
    assert rc == 0 and "configmap/cfg annotated" in out, (out, err)
    rc, out, err = kfctl(cl, "label", "ns", "opendatahub", "tier-")
    assert rc == 0 and "tier" not in (cl.client.get("v1", "Namespace", "opendatahub")["metadata"].get("labels") or {})
    rc, _, err = kfctl(cl, "label", "ns", "opendatahub")
    assert rc != 0


def test_scale_deployment(cl):
    rc, out, err = kfctl(cl, "apply", "-f", "-", stdin=DEPLOY)
    assert rc == 0, err
    rc, out, err = kfctl(cl, "scale", "deployment", "web", "-n", "opendatahub", "--replicas=3")
    assert rc == 0 and out.strip() == "deployment.apps/web scaled", (out, err)
    assert cl.client.get("apps/v1", "Deployment", "web", "opendatahub")["spec"]["replicas"] == 3
    rc, out, err = kfctl(cl, "scale", "deploy/web", "-n", "opendatahub", "--replicas=0", "--current-replicas=2")
    assert rc == 1 and "Expected replicas to be 2, was 3" in err, err
    rc, out, err = kfctl(cl, "scale", "deploy/web", "-n", "opendatahub", "--replicas=0", "--current-replicas=3")
    assert rc == 0, err
    assert cl.client.get("apps/v1", "Deployment", "web", "opendatahub")["spec"]["replicas"] == 0
    rc, out, err = kfctl(cl, "scale", "deploy/web", "-n", "opendatahub")
    assert rc == 1 and "--replicas=COUNT" in err
