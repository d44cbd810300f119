"""Process-wide Kubernetes client of a web app (the pod's service-account identity)."""
import threading

from kubeflow_rm_amd.client import KubeClient

_client = None
_lock = threading.Lock()


def client() -> KubeClient:
    global _client
    with _lock:
        if _client is None:
            _client = KubeClient()
        return _client


def set_client(c: KubeClient) -> None:
    global _client
    with _lock:
        _client = c
