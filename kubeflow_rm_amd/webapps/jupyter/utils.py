"""JWA utilities: config loading (TTL cache), GPU summary, list-row shaping, PVC helpers."""
from __future__ import annotations

import logging
import os
import random
import string
import threading
import time

from werkzeug import exceptions

from kubeflow_rm_amd.webapps.crud_backend import helpers

from . import status

log = logging.getLogger(__name__)
HERE = os.path.abspath(os.path.dirname(__file__))
DEV_CONFIG = os.path.join(HERE, "yaml", "spawner_ui_config.yaml")
CONFIGS = ["/etc/config/spawner_ui_config.yaml", DEV_CONFIG]
LAST_ACTIVITY_ANNOTATION = "notebooks.kubeflow.org/last-activity"

_cfg_lock = threading.Lock()
_cfg_cache: tuple[float, dict] | None = None
CONFIG_TTL_S = 60.0


def new_notebook(name: str, namespace: str, service_account: str, creator: str) -> dict:
    """The Notebook the spawner form is applied to (reference: the JWA notebook_template.yaml):
    served version v1beta1, one container named after the notebook, minimal requests the form
    overrides, creator + empty server-type annotations, ``app`` label."""
    container = {"name": name, "image": "", "env": [], "volumeMounts": [],
                 "resources": {"requests": {"cpu": "0.1", "memory": "0.1Gi"}}}
    pod_spec = {"serviceAccountName": service_account, "containers": [container], "volumes": [], "tolerations": []}
    meta = {"name": name, "namespace": namespace, "labels": {"app": name},
            "annotations": {"notebooks.kubeflow.org/server-type": "", "notebooks.kubeflow.org/creator": creator}}
    return {"apiVersion": "kubeflow.org/v1beta1", "kind": "Notebook", "metadata": meta,
            "spec": {"template": {"spec": pod_spec}}}


def random_string(size=9, chars=string.ascii_lowercase + string.digits) -> str:
    return "".join(random.choice(chars) for _ in range(size))


def load_spawner_ui_config() -> dict:
    global _cfg_cache
    with _cfg_lock:
        if _cfg_cache and time.time() - _cfg_cache[0] < CONFIG_TTL_S:
            return _cfg_cache[1]
        paths = [os.environ["SPAWNER_UI_CONFIG"]] if os.environ.get("SPAWNER_UI_CONFIG") else CONFIGS
        for p in paths:
            data = helpers.load_yaml(p)
            if data is not None:
                log.info("Using config file: %s", p)
                _cfg_cache = (time.time(), data["spawnerFormDefaults"])
                return _cfg_cache[1]
    raise exceptions.NotFound("Couldn't find any config file.")


def clear_config_cache() -> None:
    global _cfg_cache
    with _cfg_lock:
        _cfg_cache = None


def process_gpus(container: dict) -> dict:
    cfg = load_spawner_ui_config()
    vendors = {v["limitsKey"]: v["uiName"] for v in cfg.get("gpus", {}).get("value", {}).get("vendors", [])}
    limits = container.get("resources", {}).get("limits", {})
    count, parts = 0, []
    for key, ui in vendors.items():
        if key in limits:
            count += int(limits[key])
            parts.append(f"{limits[key]} {ui}")
    return {"count": count, "message": ", ".join(parts)}


def get_storage_class(vol: dict):
    if "class" not in vol or vol["class"] == "{none}":
        return None
    if vol["class"] == "{empty}":
        return ""
    return vol["class"]


def pvc_from_dict(vol: dict | None, namespace: str) -> dict | None:
    if vol is None:
        return None
    spec = {"accessModes": [vol["mode"]], "resources": {"requests": {"storage": vol["size"]}}}
    sc = get_storage_class(vol)
    if sc is not None:
        spec["storageClassName"] = sc
    return {"metadata": {"name": vol["name"], "namespace": namespace}, "spec": spec}


def get_notebook_last_activity(nb: dict) -> str:
    return (nb["metadata"].get("annotations") or {}).get(LAST_ACTIVITY_ANNOTATION, "")


def notebook_dict_from_k8s_obj(nb: dict) -> dict:
    c = nb["spec"]["template"]["spec"]["containers"][0]
    ann = nb["metadata"].get("annotations") or {}
    res = c.get("resources", {})
    return {
        "name": nb["metadata"]["name"],
        "namespace": nb["metadata"]["namespace"],
        "serverType": ann.get("notebooks.kubeflow.org/server-type"),
        "age": nb["metadata"]["creationTimestamp"],
        "last_activity": get_notebook_last_activity(nb),
        "image": c["image"],
        "shortImage": c["image"].split("/")[-1],
        "cpu": res.get("requests", {}).get("cpu"),
        "gpus": process_gpus(c),
        "memory": res.get("requests", {}).get("memory"),
        "volumes": [v["name"] for v in c.get("volumeMounts", [])],
        "status": status.process_status(nb),
        "metadata": nb["metadata"],
        # MI355X extension: placement + in-pod readiness op report
        "gpuPlacement": (nb.get("status") or {}).get("gpus"),
        "gpuReadiness": (nb.get("status") or {}).get("gpuReadiness"),
    }
