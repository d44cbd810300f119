"""Dashboard services: Kubernetes reads, the KFAM (access-management) client and metrics.

* ``KubernetesService`` — namespaces, the dashboard ConfigMap (links + settings JSON), namespace
  events, platform info (node providerID + the `kubeflow` Application CR version)
  (reference centraldashboard/app/k8s_service.ts).
* ``KfamClient`` — REST client of native/kfam (bindings, profiles, cluster-admin check)
  (reference app/clients/profile_controller.ts, generated from the KFAM swagger).
* Metrics: ``PrometheusMetricsService`` (PROMETHEUS_URL; range queries) and
  ``LocalMetricsService`` — an in-process sampler for clusters without Prometheus that records
  node CPU / memory (psutil) and MI355X GPU allocation (amd.com/gpu requested by running pods vs
  node allocatable) every SAMPLE_PERIOD_S into a 3 h ring buffer
  (reference app/{metrics_service,prometheus_metrics_service,metrics_service_factory}.ts; the
  Stackdriver backend is GCP-only and not carried over).
"""
from __future__ import annotations

import collections
import logging
import os
import threading
import time
import urllib.parse

import requests

from kubeflow_rm_amd.client import ApiException, KubeClient

log = logging.getLogger(__name__)
INTERVALS_MIN = {"Last5m": 5, "Last15m": 15, "Last30m": 30, "Last60m": 60, "Last180m": 180}
GPU_RESOURCE = "amd.com/gpu"


class KubernetesService:
    def __init__(self, client: KubeClient, namespace: str | None = None, configmap: str | None = None):
        self.c = client
        self.namespace = namespace or os.environ.get("POD_NAMESPACE", "kubeflow")
        self.configmap = configmap or os.environ.get("DASHBOARD_CONFIGMAP", "centraldashboard-config")
        self.logout_url = os.environ.get("LOGOUT_URL", "/logout")

    def get_namespaces(self) -> list:
        try:
            return self.c.list("v1", "Namespace")["items"]
        except ApiException as e:
            log.error("Unable to fetch Namespaces: %s", e)
            return []

    def get_configmap(self) -> dict | None:
        try:
            return self.c.get("v1", "ConfigMap", self.configmap, self.namespace)
        except ApiException as e:
            log.error("Unable to fetch ConfigMap: %s", e)
            return None

    def get_events(self, namespace: str) -> list:
        try:
            return self.c.list("v1", "Event", namespace)["items"]
        except ApiException as e:
            log.error("Unable to fetch Events for %s: %s", namespace, e)
            return []

    def get_nodes(self) -> list:
        try:
            return self.c.list("v1", "Node")["items"]
        except ApiException as e:
            log.error("Unable to fetch Nodes: %s", e)
            return []

    def get_pods(self) -> list:
        try:
            return self.c.list("v1", "Pod")["items"]
        except ApiException as e:
            log.error("Unable to fetch Pods: %s", e)
            return []

    def _provider(self) -> str:
        for n in self.get_nodes():
            pid = (n.get("spec") or {}).get("providerID")
            if pid:
                return pid
        return "other://"

    def _kubeflow_version(self) -> str:
        try:
            apps = self.c.list("app.k8s.io/v1beta1", "Application", self.namespace)["items"]
        except (ApiException, KeyError, ValueError) as e:
            log.error("Unable to fetch Application information: %s", e)
            return "unknown"
        for app in apps:
            desc = ((app.get("spec") or {}).get("descriptor") or {})
            if str(desc.get("type", "")).lower() == "kubeflow":
                return desc.get("version", "unknown")
        return "unknown"

    def get_platform_info(self) -> dict:
        provider = self._provider()
        return {"kubeflowVersion": self._kubeflow_version(), "provider": provider,
                "providerName": provider.split(":")[0], "logoutUrl": self.logout_url}


class KfamError(Exception):
    def __init__(self, status: int, body: str):
        super().__init__(f"KFAM HTTP {status}: {body}")
        self.status, self.body = status, body


def _to_wire(binding: dict) -> dict:
    """KFAM's JSON names the role field `RoleRef` (Go field without a json tag); the API objects
    here use `roleRef`, like the reference's generated client (attribute baseName mapping)."""
    b = dict(binding)
    if "roleRef" in b:
        b["RoleRef"] = b.pop("roleRef")
    return b


def _from_wire(binding: dict) -> dict:
    b = dict(binding)
    if "RoleRef" in b:
        b["roleRef"] = b.pop("RoleRef")
    return b


class KfamClient:
    def __init__(self, base_url: str, timeout: float = 10.0):
        self.base = base_url.rstrip("/")
        self.timeout = timeout

    def _req(self, method, path, params=None, body=None, headers=None):
        r = requests.request(method, self.base + path, params=params, json=body, headers=headers or {},
                             timeout=self.timeout)
        if r.status_code >= 300:
            raise KfamError(r.status_code, r.text)
        return r

    def read_bindings(self, user: str | None = None, namespace: str | None = None, role: str | None = None) -> list:
        params = {k: v for k, v in (("user", user), ("namespace", namespace), ("role", role)) if v}
        r = self._req("GET", "/v1/bindings", params=params)
        return [_from_wire(b) for b in (r.json() if r.text else {}).get("bindings") or []]

    def is_cluster_admin(self, user: str) -> bool:
        return self._req("GET", "/v1/role/clusteradmin", params={"user": user}).text.strip() == "true"

    def create_binding(self, binding: dict, headers: dict) -> None:
        self._req("POST", "/v1/bindings", body=_to_wire(binding), headers=headers)

    def delete_binding(self, binding: dict, headers: dict) -> None:
        self._req("DELETE", "/v1/bindings", body=_to_wire(binding), headers=headers)

    def create_profile(self, profile: dict, headers: dict | None = None) -> None:
        self._req("POST", "/v1/profiles", body=profile, headers=headers)

    def delete_profile(self, name: str, headers: dict) -> str:
        return self._req("DELETE", "/v1/profiles/" + urllib.parse.quote(name), headers=headers).text


# ---- metrics -----------------------------------------------------------------------------------
class PrometheusMetricsService:
    QUERIES = {
        "node": "sum(rate(node_cpu_seconds_total[5m])) by (instance)",
        "podcpu": "sum(rate(container_cpu_usage_seconds_total[5m]))",
        "podmem": "sum(container_memory_usage_bytes)",
        # AMD device-metrics-exporter: GFX engine activity (%) per GPU
        "gpu": "avg(gpu_gfx_activity) by (gpu_id)",
    }

    def __init__(self, url: str, dashboard_url: str | None = None):
        self.url = url.rstrip("/")
        self.dashboard_url = dashboard_url

    def series(self, kind: str, interval: str) -> list:
        end = time.time()
        start = end - INTERVALS_MIN.get(interval, 15) * 60
        r = requests.get(self.url + "/api/v1/query_range",
                         params={"query": self.QUERIES[kind], "start": start, "end": end, "step": 10}, timeout=15)
        data = r.json().get("data", {})
        if data.get("resultType") != "matrix":
            log.warning("prometheus returned result type %s", data.get("resultType"))
            return []
        out = []
        for s in data.get("result", []):
            label = ",".join(f"{k}={v}" for k, v in (s.get("metric") or {}).items())
            # the chart multiplies timestamp by 1000 and value by 100
            out += [{"timestamp": float(t), "label": label, "value": float(v) / 100} for t, v in s.get("values", [])]
        return out

    def charts_link(self) -> dict:
        return {"resourceChartsLink": self.dashboard_url, "resourceChartsLinkText": "View in dashboard"}


class LocalMetricsService:
    SAMPLE_PERIOD_S = 10.0

    def __init__(self, k8s: KubernetesService, period: float | None = None, horizon_s: float = 3 * 3600):
        self.k8s = k8s
        self.period = period or self.SAMPLE_PERIOD_S
        self.samples: dict[str, collections.deque] = {
            k: collections.deque(maxlen=int(horizon_s / self.period) + 1) for k in ("node", "podcpu", "podmem", "gpu")}
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._thread = threading.Thread(target=self._run, name="dashboard-metrics", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()

    def sample_once(self) -> None:
        import psutil
        now = time.time()
        vals = {"node": [("instance=local", psutil.cpu_percent(interval=None) / 100.0)],
                "podmem": [("", float(psutil.virtual_memory().used) / 100.0)]}
        nodes, pods = self.k8s.get_nodes(), self.k8s.get_pods()
        running = [p for p in pods if (p.get("status") or {}).get("phase") == "Running"]
        cpu_req = 0.0
        for p in running:
            for c in (p.get("spec") or {}).get("containers", []):
                cpu_req += _cpu_cores(((c.get("resources") or {}).get("requests") or {}).get("cpu", "0"))
        cores = float(psutil.cpu_count() or 1)
        vals["podcpu"] = [("", cpu_req / cores)]
        gpu = []
        for n in nodes:
            alloc = int(((n.get("status") or {}).get("allocatable") or {}).get(GPU_RESOURCE, "0") or 0)
            if not alloc:
                continue
            used = sum(int(((c.get("resources") or {}).get("limits") or {}).get(GPU_RESOURCE, "0") or 0)
                       for p in running if (p.get("spec") or {}).get("nodeName") == n["metadata"]["name"]
                       for c in (p.get("spec") or {}).get("containers", []))
            gpu.append((f"node={n['metadata']['name']}", used / alloc))
        vals["gpu"] = gpu
        with self._lock:
            for k, pts in vals.items():
                for label, v in pts:
                    self.samples[k].append({"timestamp": now, "label": label, "value": v})

    def _run(self):
        while not self._stop.is_set():
            try:
                self.sample_once()
            except Exception as e:  # noqa: BLE001 - keep sampling
                log.warning("metrics sample failed: %s", e)
            self._stop.wait(self.period)

    def series(self, kind: str, interval: str) -> list:
        since = time.time() - INTERVALS_MIN.get(interval, 15) * 60
        with self._lock:
            return [s for s in self.samples[kind] if s["timestamp"] >= since]

    def charts_link(self) -> dict:
        return {"resourceChartsLink": None, "resourceChartsLinkText": "View in dashboard"}


def _cpu_cores(q: str) -> float:
    q = str(q)
    if q.endswith("m"):
        return float(q[:-1]) / 1000.0
    try:
        return float(q)
    except ValueError:
        return 0.0


def make_metrics_service(k8s: KubernetesService):
    """PROMETHEUS_URL -> Prometheus; METRICS_PROVIDER=local -> in-process sampler; else none (405)."""
    if os.environ.get("PROMETHEUS_URL"):
        return PrometheusMetricsService(os.environ["PROMETHEUS_URL"], os.environ.get("METRICS_DASHBOARD"))
    if os.environ.get("METRICS_PROVIDER", "").lower() == "local":
        return LocalMetricsService(k8s)
    return None
