"""Spawner form -> Notebook CR (reference jupyter/backend/apps/common/form.py semantics).

Every field goes through ``get_form_value``: a field the admin pinned ``readOnly`` in the config
must not be sent (400) and takes the configured value; an absent non-optional field is a 400.
"""
from __future__ import annotations

import json
import logging

from werkzeug.exceptions import BadRequest

from . import utils

log = logging.getLogger(__name__)
SERVER_TYPE_ANNOTATION = "notebooks.kubeflow.org/server-type"
HEADERS_ANNOTATION = "notebooks.kubeflow.org/http-headers-request-set"
URI_REWRITE_ANNOTATION = "notebooks.kubeflow.org/http-rewrite-uri"
SERVER_TYPES = ("jupyter", "group-one", "group-two")


def get_form_value(body, defaults, body_field, defaults_field=None, optional=False):
    defaults_field = defaults_field or body_field
    user_value = body.get(body_field)
    if defaults_field not in defaults:
        return user_value
    if defaults[defaults_field].get("readOnly", False):
        if body_field in body:
            raise BadRequest(f"'{body_field}' is readonly but a value was provided: {user_value}")
        return defaults[defaults_field]["value"]
    if user_value is None:
        if not optional:
            raise BadRequest(f"No value provided for: {body_field}")
        return None
    return user_value


def _container(nb):
    return nb["spec"]["template"]["spec"]["containers"][0]


def set_notebook_image(nb, body, defaults):
    field = "customImage" if body.get("customImage", False) else "image"
    _container(nb)["image"] = get_form_value(body, defaults, field, "image").strip()


def set_notebook_image_pull_policy(nb, body, defaults):
    _container(nb)["imagePullPolicy"] = get_form_value(body, defaults, "imagePullPolicy")


def set_server_type(nb, body, defaults):
    server_type = get_form_value(body, defaults, "serverType") or "jupyter"
    if server_type not in SERVER_TYPES:
        raise BadRequest(f"'{server_type}' is not a valid server type")
    name = get_form_value(body, defaults, "name")
    ns = get_form_value(body, defaults, "namespace")
    ann = nb["metadata"]["annotations"]
    ann[SERVER_TYPE_ANNOTATION] = server_type
    if server_type in ("group-one", "group-two"):
        ann[URI_REWRITE_ANNOTATION] = "/"
    if server_type == "group-two":
        ann[HEADERS_ANNOTATION] = json.dumps({"X-RStudio-Root-Path": f"/notebook/{ns}/{name}/"}, separators=(",", ":"))


def _limit(value, factor, unit=""):
    return str(round(float(value.replace(unit, "")) * float(factor), 1)) + unit


def set_notebook_cpu(nb, body, defaults):
    c = _container(nb)
    cpu = get_form_value(body, defaults, "cpu")
    if cpu and "nan" in str(cpu).lower():
        raise BadRequest(f"Invalid value for cpu: {cpu}")
    cpu_limit = get_form_value(body, defaults, "cpuLimit", optional=True)
    if cpu_limit and "nan" in str(cpu_limit).lower():
        raise BadRequest(f"Invalid value for cpu limit: {cpu_limit}")
    factor = utils.load_spawner_ui_config()["cpu"].get("limitFactor")
    if not cpu_limit and factor not in (None, "none"):
        cpu_limit = _limit(str(cpu), factor)
    c["resources"]["requests"]["cpu"] = str(cpu)
    if not cpu_limit:
        return
    if float(cpu_limit) < float(cpu):
        raise BadRequest("CPU limit must be greater than the request")
    c["resources"].setdefault("limits", {})["cpu"] = str(cpu_limit)


def set_notebook_memory(nb, body, defaults):
    c = _container(nb)
    mem = get_form_value(body, defaults, "memory")
    if mem and "nan" in str(mem).lower():
        raise BadRequest(f"Invalid value for memory: {mem}")
    mem_limit = get_form_value(body, defaults, "memoryLimit", optional=True)
    if mem_limit and "nan" in str(mem_limit).lower():
        raise BadRequest(f"Invalid value for memory limit: {mem_limit}")
    factor = utils.load_spawner_ui_config()["memory"].get("limitFactor")
    if not mem_limit and factor not in (None, "none"):
        mem_limit = _limit(str(mem), factor, "Gi")
    c["resources"]["requests"]["memory"] = str(mem)
    if not mem_limit:
        return
    if float(str(mem_limit).replace("Gi", "")) < float(str(mem).replace("Gi", "")):
        raise BadRequest("Memory limit must be greater than the request")
    c["resources"].setdefault("limits", {})["memory"] = str(mem_limit)


def set_notebook_gpus(nb, body, defaults):
    gpus = get_form_value(body, defaults, "gpus")
    if not isinstance(gpus, dict) or "num" not in gpus:
        raise BadRequest("'gpus' must have a 'num' field")
    if gpus["num"] == "none":
        return
    if "vendor" not in gpus or not gpus["vendor"]:
        raise BadRequest("'gpus' must have a 'vendor' field")
    try:
        num = int(gpus["num"])
    except (TypeError, ValueError):
        raise BadRequest(f"gpus.num is not a valid number: {gpus['num']}")
    if num <= 0:
        raise BadRequest(f"gpus.num must be positive: {num}")
    _container(nb)["resources"].setdefault("limits", {})[gpus["vendor"]] = str(num)


def set_notebook_tolerations(nb, body, defaults):
    key = get_form_value(body, defaults, "tolerationGroup")
    if key in ("none", "", None):
        return
    for group in utils.load_spawner_ui_config().get("tolerationGroup", {}).get("options", []):
        if group["groupKey"] == key:
            nb["spec"]["template"]["spec"]["tolerations"].extend(group["tolerations"])
            return
    log.warning("Didn't find any Toleration Group with key '%s' in the config", key)


def set_notebook_affinity(nb, body, defaults):
    key = get_form_value(body, defaults, "affinityConfig")
    if key in ("none", "", None):
        return
    for cfg in utils.load_spawner_ui_config().get("affinityConfig", {}).get("options", []):
        if cfg["configKey"] == key:
            nb["spec"]["template"]["spec"]["affinity"] = cfg["affinity"]
            return
    log.warning("Didn't find any Affinity Config with key '%s' in the config", key)


def set_notebook_configurations(nb, body, defaults):
    labels = get_form_value(body, defaults, "configurations")
    if not isinstance(labels, list):
        raise BadRequest(f"Labels for PodDefaults are not list: {labels}")
    for label in labels:
        nb["metadata"]["labels"][label] = "true"


def set_notebook_shm(nb, body, defaults):
    if not get_form_value(body, defaults, "shm"):
        return
    nb["spec"]["template"]["spec"]["volumes"].append({"name": "dshm", "emptyDir": {"medium": "Memory"}})
    _container(nb)["volumeMounts"].append({"mountPath": "/dev/shm", "name": "dshm"})


def set_notebook_environment(nb, body, defaults):
    env = get_form_value(body, defaults, "environment", optional=True)
    if isinstance(env, str):
        env = json.loads(env) if env else {}
    env = env or {}
    _container(nb)["env"] += [{"name": k, "value": str(v)} for k, v in env.items()]
