"""Thin Kubernetes REST client (replaces the `kubernetes` Python package, absent here — SURVEY §2.2 P1).

Speaks the Kubernetes API conventions against kube-lite (native/apiserver) or any real
kube-apiserver: discovery-cached kind->plural resolution, CRUD, merge/JSON/strategic patches,
status subresource, dry-run, propagation policies, list/watch with selectors, pod logs, and
SubjectAccessReview. Errors raise :class:`ApiException` carrying the HTTP status and the
Kubernetes ``Status`` body, like the official client's ``ApiException``.
"""
from __future__ import annotations

import json
import os
import re
import sys
import threading
import time
import urllib.parse
from typing import Any, Callable, Iterator

import requests

PATCH_TYPES = {
    "merge": "application/merge-patch+json",
    "json": "application/json-patch+json",
    "strategic": "application/strategic-merge-patch+json",
    "apply": "application/apply-patch+yaml",
}


class ApiException(Exception):
    def __init__(self, status: int, reason: str = "", body: Any = None):
        self.status = status
        self.reason = reason
        self.body = body if body is not None else {}
        msg = self.body.get("message") if isinstance(self.body, dict) else str(self.body)
        super().__init__(f"({status}) {reason}: {msg}")

    @property
    def message(self) -> str:
        return self.body.get("message", "") if isinstance(self.body, dict) else str(self.body)


def _split_api_version(api_version: str) -> tuple[str, str]:
    if "/" in api_version:
        g, v = api_version.split("/", 1)
        return g, v
    return "", api_version


# Sanitizer builds of the control plane (tools/sanitize.sh) run 5-15x slower: every wait scales.
_TIMEOUT_SCALE = float(os.environ.get("KFAMD_TIMEOUT_SCALE", "1"))
_WARN_VALUE = re.compile(r'\d{3} [^ ]+ "((?:[^"\\]|\\.)*)"')


def parse_warning_header(value: str) -> list[str]:
    """RFC 7234 Warning header values (``299 - "unknown field \"spec.x\""``, comma-joined when the
    server sent several) -> the warning texts, in order."""
    return [json.loads(f'"{m.group(1)}"') for m in _WARN_VALUE.finditer(value or "")]


def print_warning(text: str) -> None:
    """kubectl's default warning handler: one ``Warning: <text>`` line on stderr."""
    print(f"Warning: {text}", file=sys.stderr)


_SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class KubeClient:
    """REST client. ``base_url`` defaults to $KFAMD_API_URL / in-cluster KUBERNETES_SERVICE_HOST.

    https servers are verified against ``ca_file`` (default $KFAMD_CA_FILE, else the service
    account's ca.crt in-cluster, else the system trust store); ``verify=False`` skips it."""

    def __init__(self, base_url: str | None = None, token: str | None = None, impersonate: str | None = None,
                 impersonate_groups: list[str] | None = None, timeout: float = 30.0,
                 ca_file: str | None = None, verify: bool = True, client_cert: tuple[str, str] | None = None):
        in_cluster = False
        if base_url is None:
            base_url = os.environ.get("KFAMD_API_URL")
            if not base_url and os.environ.get("KUBERNETES_SERVICE_HOST"):
                # rest.InClusterConfig: the kubernetes service is HTTPS
                base_url = f"https://{os.environ['KUBERNETES_SERVICE_HOST']}:{os.environ.get('KUBERNETES_SERVICE_PORT', '443')}"
                in_cluster = True
        if not base_url:
            raise ValueError("no API server URL (set KFAMD_API_URL)")
        self.base = base_url.rstrip("/")
        self.timeout = timeout
        self.session = requests.Session()
        self.session.trust_env = False
        if ca_file is None:
            ca_file = os.environ.get("KFAMD_CA_FILE") or None
            if ca_file is None and in_cluster and os.path.exists(f"{_SA_DIR}/ca.crt"):
                ca_file = f"{_SA_DIR}/ca.crt"
        self.session.verify = (ca_file or True) if verify else False
        if client_cert:
            self.session.cert = client_cert
        if token is None and in_cluster and os.path.exists(f"{_SA_DIR}/token"):
            with open(f"{_SA_DIR}/token") as f:
                token = f.read().strip()
        self.headers: dict[str, str] = {"Accept": "application/json"}
        if token:
            self.headers["Authorization"] = f"Bearer {token}"
        if impersonate:
            self.headers["Impersonate-User"] = impersonate
            if impersonate_groups:
                self.headers["Impersonate-Group"] = ",".join(impersonate_groups)
        self._res: dict[tuple[str, str], tuple[str, bool]] = {}
        self._lock = threading.Lock()
        # server warnings (unknown / pruned fields, deprecations): kept in ``warnings`` and passed to
        # ``warning_handler`` (the CLIs set print_warning, as kubectl prints them)
        self.warnings: list[str] = []
        self.warning_handler: Callable[[str], None] | None = None

    # ---- plumbing ----------------------------------------------------------------------------
    def _req(self, method: str, path: str, body: Any = None, params: dict | None = None,
             content_type: str = "application/json", raw: bool = False, timeout: float | None = None):
        headers = dict(self.headers)
        data = None
        if body is not None:
            data = json.dumps(body)
            headers["Content-Type"] = content_type
        r = self.session.request(method, self.base + path, data=data, params=params, headers=headers,
                                 timeout=timeout or self.timeout)
        if "Warning" in r.headers:
            for w in parse_warning_header(r.headers["Warning"]):
                self.warnings.append(w)
                if self.warning_handler:
                    self.warning_handler(w)
        if raw:
            if r.status_code >= 400:
                raise ApiException(r.status_code, r.reason, _safe_json(r.text))
            return r.text
        payload = _safe_json(r.text)
        if r.status_code >= 400:
            raise ApiException(r.status_code, (payload or {}).get("reason", r.reason) if isinstance(payload, dict) else r.reason,
                               payload)
        return payload

    def resource(self, api_version: str, kind: str) -> tuple[str, bool]:
        key = (api_version, kind)
        with self._lock:
            if key in self._res:
                return self._res[key]
        g, v = _split_api_version(api_version)
        disc = self._req("GET", f"/apis/{g}/{v}" if g else f"/api/{v}")
        with self._lock:
            for r in disc.get("resources", []):
                if "/" in r["name"]:
                    continue
                self._res[(api_version, r["kind"])] = (r["name"], r.get("namespaced", True))
            if key not in self._res:
                raise ApiException(404, "NotFound", {"message": f"kind {kind} not served by {api_version}"})
            return self._res[key]

    def path(self, api_version: str, kind: str, namespace: str | None = None, name: str | None = None,
             subresource: str | None = None) -> str:
        plural, namespaced = self.resource(api_version, kind)
        g, v = _split_api_version(api_version)
        p = f"/apis/{g}/{v}" if g else f"/api/{v}"
        if namespaced and namespace:
            p += f"/namespaces/{urllib.parse.quote(namespace)}"
        p += f"/{plural}"
        if name:
            p += f"/{urllib.parse.quote(name)}"
        if subresource:
            p += f"/{subresource}"
        return p

    # ---- CRUD -------------------------------------------------------------------------------------
    def get(self, api_version: str, kind: str, name: str, namespace: str | None = None) -> dict:
        return self._req("GET", self.path(api_version, kind, namespace, name))

    def list(self, api_version: str, kind: str, namespace: str | None = None, label_selector: str = "",
             field_selector: str = "", limit: int = 0) -> dict:
        params = {}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        if limit:
            params["limit"] = str(limit)
        return self._req("GET", self.path(api_version, kind, namespace), params=params)

    def create(self, obj: dict, namespace: str | None = None, dry_run: bool = False) -> dict:
        ns = namespace or obj.get("metadata", {}).get("namespace")
        params = {"dryRun": "All"} if dry_run else None
        return self._req("POST", self.path(obj["apiVersion"], obj["kind"], ns), obj, params=params)

    def update(self, obj: dict, dry_run: bool = False) -> dict:
        md = obj["metadata"]
        params = {"dryRun": "All"} if dry_run else None
        return self._req("PUT", self.path(obj["apiVersion"], obj["kind"], md.get("namespace"), md["name"]), obj, params=params)

    def update_status(self, obj: dict) -> dict:
        md = obj["metadata"]
        return self._req("PUT", self.path(obj["apiVersion"], obj["kind"], md.get("namespace"), md["name"], "status"), obj)

    def patch(self, api_version: str, kind: str, name: str, body: Any, namespace: str | None = None,
              patch_type: str = "merge", subresource: str | None = None, dry_run: bool = False) -> dict:
        params = {"dryRun": "All"} if dry_run else None
        return self._req("PATCH", self.path(api_version, kind, namespace, name, subresource), body,
                         content_type=PATCH_TYPES.get(patch_type, patch_type), params=params)

    def delete(self, api_version: str, kind: str, name: str, namespace: str | None = None,
               propagation_policy: str | None = None, grace_period_seconds: int | None = None,
               dry_run: bool = False) -> dict:
        params = {}
        if propagation_policy:
            params["propagationPolicy"] = propagation_policy
        if grace_period_seconds is not None:
            params["gracePeriodSeconds"] = str(grace_period_seconds)
        if dry_run:
            params["dryRun"] = "All"
        return self._req("DELETE", self.path(api_version, kind, namespace, name), params=params)

    def apply(self, obj: dict, dry_run: bool = False) -> dict:
        """``kubectl apply`` (client-side): create, or three-way strategic merge patch against the
        last-applied-configuration annotation (kubeflow_rm_amd.apply). Returns the object."""
        from .apply import apply_object
        return apply_object(self, obj, dry_run=dry_run)[1]

    def exists(self, api_version: str, kind: str, name: str, namespace: str | None = None) -> bool:
        try:
            self.get(api_version, kind, name, namespace)
            return True
        except ApiException as e:
            if e.status == 404:
                return False
            raise

    def pod_logs(self, name: str, namespace: str, container: str | None = None, tail_lines: int | None = None) -> str:
        params = {}
        if container:
            params["container"] = container
        if tail_lines is not None:
            params["tailLines"] = str(tail_lines)
        return self._req("GET", f"/api/v1/namespaces/{namespace}/pods/{name}/log", params=params, raw=True)

    def pod_exec(self, name: str, namespace: str, command: list[str], container: str | None = None,
                 timeout: float = 30.0) -> dict:
        """Non-interactive exec: {"exitCode": n, "output": stdout+stderr}."""
        params = [("command", c) for c in command]
        if container:
            params.append(("container", container))
        params.append(("timeoutSeconds", str(int(max(1, timeout)))))
        return self._req("POST", f"/api/v1/namespaces/{namespace}/pods/{name}/exec", params=params,
                         timeout=timeout + 10)

    def subject_access_review(self, user: str, verb: str, group: str, resource: str, namespace: str | None = None,
                              name: str | None = None, subresource: str | None = None, groups: list[str] | None = None) -> dict:
        body = {"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview",
                "spec": {"user": user, "groups": groups or [],
                         "resourceAttributes": {"verb": verb, "group": group, "resource": resource,
                                                "namespace": namespace or "", "name": name or "",
                                                "subresource": subresource or ""}}}
        return self._req("POST", "/apis/authorization.k8s.io/v1/subjectaccessreviews", body)

    # ---- watch ------------------------------------------------------------------------------------
    def watch(self, api_version: str, kind: str, namespace: str | None = None, resource_version: str = "",
              label_selector: str = "", timeout_seconds: int = 60) -> Iterator[dict]:
        params = {"watch": "true", "timeoutSeconds": str(timeout_seconds)}
        if resource_version:
            params["resourceVersion"] = resource_version
        if label_selector:
            params["labelSelector"] = label_selector
        with self.session.get(self.base + self.path(api_version, kind, namespace), params=params, headers=self.headers,
                              stream=True, timeout=timeout_seconds + 5) as r:
            for line in r.iter_lines():
                if line:
                    yield json.loads(line)

    # ---- waits ------------------------------------------------------------------------------------
    def wait_for(self, api_version: str, kind: str, name: str, namespace: str | None,
                 predicate: Callable[[dict], bool], timeout: float = 30.0, interval: float = 0.05) -> dict:
        deadline = time.time() + timeout * _TIMEOUT_SCALE
        last: Any = None
        while time.time() < deadline:
            try:
                last = self.get(api_version, kind, name, namespace)
                if predicate(last):
                    return last
            except ApiException as e:
                if e.status != 404:
                    raise
                last = e
            time.sleep(interval)
        raise TimeoutError(f"timed out waiting for {kind} {namespace}/{name}; last={str(last)[:500]}")

    def wait_gone(self, api_version: str, kind: str, name: str, namespace: str | None, timeout: float = 30.0) -> None:
        deadline = time.time() + timeout * _TIMEOUT_SCALE
        while time.time() < deadline:
            if not self.exists(api_version, kind, name, namespace):
                return
            time.sleep(0.05)
        raise TimeoutError(f"{kind} {namespace}/{name} still present")


def _safe_json(text: str):
    try:
        return json.loads(text) if text else {}
    except ValueError:
        return {"message": text}
