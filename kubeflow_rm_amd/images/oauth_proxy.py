"""oauth-proxy sidecar for ODH notebooks (the ose-oauth-proxy image's role, kube-lite flavour).

Accepts the reference's flags (--https-address=:8443, --upstream=http://localhost:8888,
--openshift-sar={...}, --openshift-service-account, --cookie-secret-file, --tls-cert/--tls-key,
--logout-url, ...). Each request is authorised with a SubjectAccessReview built from
--openshift-sar (`get notebooks/<name>` in the namespace) for the user named by the
kubeflow-userid header (or a bearer token's user), then proxied to the notebook container.
TLS is served when the serving-cert secret is mounted; otherwise plain HTTP on the same port.
`/oauth/healthz` answers the probes.
"""
from __future__ import annotations

import argparse
import json
import os
import ssl
import sys
import urllib.request
from http.client import HTTPConnection

from kubeflow_rm_amd.images._http import JsonHandler, bind_host, resolve_path, serve

HOP = {"connection", "keep-alive", "proxy-authenticate", "proxy-authorization", "te", "trailers",
       "transfer-encoding", "upgrade", "host", "content-length"}


def sar_allowed(api: str, user: str, sar: dict) -> bool:
    body = {"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview",
            "spec": {"user": user, "resourceAttributes": {
                "verb": sar.get("verb", "get"), "group": sar.get("resourceAPIGroup", ""), "resource": sar.get("resource", ""),
                "name": sar.get("resourceName", ""), "namespace": sar.get("namespace", "")}}}
    req = urllib.request.Request(api + "/apis/authorization.k8s.io/v1/subjectaccessreviews", data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json"}, method="POST")
    try:
        with urllib.request.urlopen(req, timeout=5) as r:
            return bool(json.loads(r.read())["status"]["allowed"])
    except Exception:
        return False


def make_handler(upstream: tuple[str, int], sar: dict, api: str, user_header: str, logout: str | None):
    class H(JsonHandler):
        def _proxy(self):
            if self.path.startswith("/oauth/healthz"):
                return self.send_text(200, "OK")
            if self.path.startswith("/oauth/sign_out"):
                self.send_response(302)
                self.send_header("Location", logout or "/")
                self.send_header("Content-Length", "0")
                self.end_headers()
                return
            user = self.headers.get(user_header, "")
            if not user or not sar_allowed(api, user, sar):
                return self.send_json(403, {"error": "forbidden", "user": user})
            n = int(self.headers.get("Content-Length") or 0)
            body = self.rfile.read(n) if n else None
            conn = HTTPConnection(*upstream, timeout=30)
            hdrs = {k: v for k, v in self.headers.items() if k.lower() not in HOP}
            hdrs["X-Forwarded-User"] = user
            conn.request(self.command, self.path, body=body, headers=hdrs)
            resp = conn.getresponse()
            data = resp.read()
            self.send_response(resp.status)
            for k, v in resp.getheaders():
                if k.lower() not in HOP:
                    self.send_header(k, v)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)
            conn.close()

        do_GET = do_POST = do_PUT = do_DELETE = do_PATCH = _proxy
    return H


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--https-address", default=":8443")
    ap.add_argument("--http-address", default="")
    ap.add_argument("--upstream", default="http://localhost:8888")
    ap.add_argument("--openshift-sar", default="{}")
    ap.add_argument("--tls-cert", default="")
    ap.add_argument("--tls-key", default="")
    ap.add_argument("--logout-url", default=None)
    ap.add_argument("--user-header", default=os.environ.get("KFAMD_USERID_HEADER", "kubeflow-userid"))
    a, _ = ap.parse_known_args(argv)
    ns = os.environ.get("NAMESPACE", "")
    sar = json.loads(a.openshift_sar.replace("$(NAMESPACE)", ns) or "{}")
    up = a.upstream.split("://", 1)[-1]
    host, _, port = up.partition(":")
    if host in ("localhost", "127.0.0.1"):
        host = bind_host()  # the pod's loopback IP: containers of a process pod share it
    port_n = int(a.https_address.rsplit(":", 1)[-1] or 8443)
    api = os.environ.get("KFAMD_API_URL", "http://127.0.0.1:6443")
    srv = serve(make_handler((host, int(port or 80)), sar, api, a.user_header, a.logout_url), port_n)
    cert, key = resolve_path(a.tls_cert) if a.tls_cert else "", resolve_path(a.tls_key) if a.tls_key else ""
    scheme = "http"
    if cert and key and os.path.exists(cert) and os.path.exists(key):
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(cert, key)
        srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
        scheme = "https"
    print(f"oauth-proxy {scheme}://{srv.server_address[0]}:{port_n} -> {host}:{port} sar={sar}", flush=True)
    srv.serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())
