"""TLS on every wire.

Certificates are generated with /usr/bin/openssl the way the reference CI does it
(.github/workflows/odh_notebook_controller_integration_test.yaml:105-295: a self-signed CA, then
a serving certificate signed by it). Covered:

* kube-lite serves the API over HTTPS (kube-apiserver's --tls-cert-file / --tls-private-key-file);
  clients verify it against the CA and refuse it without the CA;
* the split admission-webhook binary talks to that API server over HTTPS (--certificate-authority),
  serves its hooks over HTTPS (--tlsCertFile / --tlsKeyFile, the reference's flags) and registers
  them with a caBundle; the API server calls them over HTTPS and verifies the bundle — a webhook
  presenting a certificate from another CA fails the request (failurePolicy Fail);
* certificate rotation: a replaced pair is served from the next connection on (certwatcher).
"""
import os
import signal
import socket
import ssl
import subprocess
import time

import pytest
import requests

from kubeflow_rm_amd.client import ApiException, KubeClient
from kubeflow_rm_amd.cluster import BIN, LocalCluster

OPENSSL = "/usr/bin/openssl"
pytestmark = pytest.mark.skipif(not os.path.exists(OPENSSL), reason="openssl CLI not installed")


def _run(*args, cwd):
    subprocess.run([OPENSSL, *args], cwd=cwd, check=True, capture_output=True)


def _make_ca(d, name):
    _run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "2", "-subj", f"/CN={name}",
         "-keyout", f"{name}.key", "-out", f"{name}.crt",
         "-addext", "basicConstraints=critical,CA:TRUE", "-addext", "keyUsage=critical,keyCertSign,cRLSign", cwd=d)


def _make_leaf(d, ca, name, cn="127.0.0.1"):
    _run("req", "-new", "-newkey", "rsa:2048", "-nodes", "-subj", f"/CN={cn}", "-keyout", f"{name}.key",
         "-out", f"{name}.csr", cwd=d)
    with open(os.path.join(d, f"{name}.ext"), "w") as f:
        f.write("subjectAltName=IP:127.0.0.1,DNS:localhost\nextendedKeyUsage=serverAuth\n")
    _run("x509", "-req", "-in", f"{name}.csr", "-CA", f"{ca}.crt", "-CAkey", f"{ca}.key", "-CAcreateserial",
         "-days", "2", "-extfile", f"{name}.ext", "-out", f"{name}.crt", cwd=d)


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("pki"))
    _make_ca(d, "ca")
    _make_ca(d, "rogue")
    _make_leaf(d, "ca", "api")
    _make_leaf(d, "ca", "hook")
    _make_leaf(d, "ca", "hook2")
    _make_leaf(d, "rogue", "evil")
    return d


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _peer_cert(port):
    ctx = ssl.create_default_context()
    ctx.check_hostname = False
    ctx.verify_mode = ssl.CERT_NONE
    with socket.create_connection(("127.0.0.1", port), timeout=5) as s:
        with ctx.wrap_socket(s) as t:
            der = t.getpeercert(binary_form=True)
    return der


@pytest.fixture(scope="module")
def tls_cluster(pki):
    from tests.conftest import _ensure_native
    _ensure_native()
    cl = LocalCluster(controllers="builtin,scheduler", gpus=8, ca_file=os.path.join(pki, "ca.crt"),
                      args=["--tls-cert-file", os.path.join(pki, "api.crt"),
                            "--tls-private-key-file", os.path.join(pki, "api.key")])
    cl.start()
    yield cl
    cl.stop()


def test_api_server_serves_https_and_clients_verify_it(tls_cluster, pki):
    assert tls_cluster.url.startswith("https://127.0.0.1:")
    ns = tls_cluster.client.list("v1", "Namespace")
    assert any(n["metadata"]["name"] == "default" for n in ns["items"])
    # without the CA (system trust store only) the handshake is refused
    with pytest.raises(requests.exceptions.SSLError):
        KubeClient(tls_cluster.url).list("v1", "Namespace")
    # a CA that did not sign the server certificate is refused too
    with pytest.raises(requests.exceptions.SSLError):
        KubeClient(tls_cluster.url, ca_file=os.path.join(pki, "rogue.crt")).list("v1", "Namespace")
    # plain HTTP on the HTTPS port gets no API response
    with pytest.raises(requests.exceptions.RequestException):
        requests.get(tls_cluster.url.replace("https://", "http://") + "/api/v1/namespaces", timeout=3).json()


def _start_webhook(pki, cl, cert, key, log_name, extra=()):
    port = _free_port()
    log = open(os.path.join(cl.data_dir, log_name), "wb")
    p = subprocess.Popen([str(BIN / "admission-webhook"), "--server", cl.url, "--certificate-authority",
                          os.path.join(pki, "ca.crt"), "--token-file", "/nonexistent", "--metrics-addr", "0",
                          "--probe-addr", "0", "--webhookPort", str(port), "--tlsCertFile", os.path.join(pki, cert),
                          "--tlsKeyFile", os.path.join(pki, key), "--webhook-ca-file", os.path.join(pki, "ca.crt"),
                          *extra], stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    return p, log, port


def _stop(p, log):
    try:
        os.killpg(p.pid, signal.SIGTERM)
    except ProcessLookupError:
        pass
    try:
        p.wait(timeout=10)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
    log.close()


def _wait_hooks(c, url_prefix, timeout=20):
    deadline = time.time() + timeout
    while time.time() < deadline:
        for m in c.list("admissionregistration.k8s.io/v1", "MutatingWebhookConfiguration")["items"]:
            ws = m.get("webhooks", [])
            if ws and all(w["clientConfig"]["url"].startswith(url_prefix) for w in ws):
                return m
        time.sleep(0.1)
    raise TimeoutError("webhooks not registered")


def _profile_ns(c, name):
    c.create({"apiVersion": "v1", "kind": "Namespace",
              "metadata": {"name": name, "labels": {"app.kubernetes.io/part-of": "kubeflow-profile"}}})
    c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PodDefault", "metadata": {"name": "env", "namespace": name},
              "spec": {"selector": {"matchLabels": {"inject": "yes"}}, "desc": "env",
                       "env": [{"name": "FROM_TLS_HOOK", "value": "1"}]}})


def _pod(name, ns):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": ns, "labels": {"inject": "yes"}},
            "spec": {"nodeSelector": {"kfamd.io/no-such-node": "true"}, "containers": [{"name": "c", "image": "x"}]}}


def test_split_webhook_over_https_with_ca_bundle(tls_cluster, pki):
    c = tls_cluster.client
    p, log, port = _start_webhook(pki, tls_cluster, "hook.crt", "hook.key", "hook.log")
    try:
        cfg = _wait_hooks(c, f"https://127.0.0.1:{port}/")
        import base64
        bundle = base64.b64decode(cfg["webhooks"][0]["clientConfig"]["caBundle"]).decode()
        assert bundle == open(os.path.join(pki, "ca.crt")).read()
        _profile_ns(c, "tls-a")
        c.create(_pod("p1", "tls-a"))
        pod = c.get("v1", "Pod", "p1", "tls-a")
        assert {"name": "FROM_TLS_HOOK", "value": "1"} in pod["spec"]["containers"][0]["env"]

        # rotation: the served certificate follows the files (next connection)
        before = _peer_cert(port)
        with open(os.path.join(pki, "hook2.crt"), "rb") as f:
            crt2 = f.read()
        with open(os.path.join(pki, "hook2.key"), "rb") as f:
            key2 = f.read()
        # key first, then certificate: the pair is only consistent once both are in place
        with open(os.path.join(pki, "hook.key"), "wb") as f:
            f.write(key2)
        with open(os.path.join(pki, "hook.crt"), "wb") as f:
            f.write(crt2)
        deadline = time.time() + 10
        while _peer_cert(port) == before and time.time() < deadline:
            time.sleep(0.3)
        assert _peer_cert(port) != before
        c.create(_pod("p2", "tls-a"))  # still trusted: hook2 is signed by the same CA
        assert {"name": "FROM_TLS_HOOK", "value": "1"} in c.get("v1", "Pod", "p2", "tls-a")["spec"]["containers"][0]["env"]
    finally:
        _stop(p, log)
        for m in c.list("admissionregistration.k8s.io/v1", "MutatingWebhookConfiguration")["items"]:
            c.delete("admissionregistration.k8s.io/v1", "MutatingWebhookConfiguration", m["metadata"]["name"])
        for m in c.list("admissionregistration.k8s.io/v1", "ValidatingWebhookConfiguration")["items"]:
            c.delete("admissionregistration.k8s.io/v1", "ValidatingWebhookConfiguration", m["metadata"]["name"])


def test_webhook_with_untrusted_certificate_fails_closed(tls_cluster, pki):
    c = tls_cluster.client
    # serves a rogue-CA certificate but registers the real CA as its caBundle
    p, log, port = _start_webhook(pki, tls_cluster, "evil.crt", "evil.key", "evil.log")
    try:
        _wait_hooks(c, f"https://127.0.0.1:{port}/")
        _profile_ns(c, "tls-b")
        with pytest.raises(ApiException) as e:
            c.create(_pod("p1", "tls-b"))
        assert e.value.status == 500 and "certificate verify failed" in str(e.value.body)
        assert not c.exists("v1", "Pod", "p1", "tls-b")
    finally:
        _stop(p, log)
        for kind in ("MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"):
            for m in c.list("admissionregistration.k8s.io/v1", kind)["items"]:
                c.delete("admissionregistration.k8s.io/v1", kind, m["metadata"]["name"])
