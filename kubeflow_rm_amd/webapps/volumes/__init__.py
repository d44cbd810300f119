"""Volumes web app (VWA) backend (reference crud-web-apps/volumes/backend/apps).

Routes:
  GET    /api/namespaces/<ns>/pvcs                    rows + notebooks using each PVC + viewer state
  GET    /api/namespaces/<ns>/pvcs/<pvc>[/pods|/events]
  POST   /api/namespaces/<ns>/pvcs                    {name, mode, class, size, type}
  DELETE /api/namespaces/<ns>/pvcs/<pvc>              409 while a non-viewer pod mounts it; the
                                                      viewers mounting it are deleted first
  POST   /api/namespaces/<ns>/viewers                 {name} -> PVCViewer from viewer-spec.yaml
  DELETE /api/namespaces/<ns>/viewers/<viewer>
"""
from __future__ import annotations

import copy
import logging
import os
from string import Template

import yaml
from flask import request
from werkzeug import exceptions

from kubeflow_rm_amd.webapps import crud_backend
from kubeflow_rm_amd.webapps.crud_backend import api, config, decorators
from kubeflow_rm_amd.webapps.crud_backend.status import STATUS_PHASE, create_status

log = logging.getLogger(__name__)
HERE = os.path.abspath(os.path.dirname(__file__))
STATIC_DIR = os.path.join(HERE, "static")
VIEWER = ("kubeflow.org", "v1alpha1", "pvcviewers", "PVCViewer")
VIEWER_SPEC_PATHS = ["/etc/config/viewer-spec.yaml", os.path.join(HERE, "yaml", "viewer-spec.yaml")]
POD_PARENT_VIEWER_LABEL_KEY = "app.kubernetes.io/name"
DEFAULT_VIEWER_IMAGE = "filebrowser/filebrowser:latest"


# ---- form --------------------------------------------------------------------------------------
def handle_storage_class(vol: dict):
    """`{none}` -> "" (no class), `{empty}` / absent -> None (cluster default)."""
    if "class" not in vol or vol["class"] == "{empty}":
        return None
    if vol["class"] == "{none}":
        return ""
    return vol["class"]


def pvc_from_dict(body: dict, namespace: str) -> dict:
    spec = {"accessModes": [body["mode"]], "resources": {"requests": {"storage": body["size"]}}}
    sc = handle_storage_class(body)
    if sc is not None:
        spec["storageClassName"] = sc
    return {"metadata": {"name": body["name"], "namespace": namespace}, "spec": spec}


# ---- status ------------------------------------------------------------------------------------
def pvc_status(pvc: dict) -> dict:
    md = pvc["metadata"]
    if md.get("deletionTimestamp"):
        return create_status(STATUS_PHASE.TERMINATING, "Deleting Volume...")
    if (pvc.get("status") or {}).get("phase") == "Bound":
        return create_status(STATUS_PHASE.READY, "Bound")
    evs = api.list_pvc_events(md["namespace"], md["name"])["items"]
    if not evs:
        return create_status(STATUS_PHASE.WAITING, "Provisioning Volume...")
    ev = evs[0]
    msg, state = f"Pending: {ev.get('message', '')}", ev.get("reason", "")
    if state == "WaitForFirstConsumer":
        phase = STATUS_PHASE.UNAVAILABLE
        msg = ("Pending: This volume will be bound when its first consumer is created. E.g., when you "
               "first browse its contents, or attach it to a notebook server")
    elif state == "Provisioning":
        phase = STATUS_PHASE.WAITING
    elif state == "FailedBinding" or ev.get("type") == "Warning":
        phase = STATUS_PHASE.WARNING
    else:
        phase = STATUS_PHASE.READY
    return create_status(phase, msg, state)


def viewer_status(viewer: dict | None) -> str:
    if not viewer:
        return STATUS_PHASE.UNINITIALIZED
    if "deletionTimestamp" in (viewer.get("metadata") or {}):
        return STATUS_PHASE.TERMINATING
    if (viewer.get("status") or {}).get("ready", False):
        return STATUS_PHASE.READY
    return STATUS_PHASE.WAITING


# ---- utils -------------------------------------------------------------------------------------
def notebook_pvcs(nb: dict) -> list:
    vols = nb["spec"]["template"]["spec"].get("volumes") or []
    return [v["persistentVolumeClaim"]["claimName"] for v in vols if v.get("persistentVolumeClaim")]


def pod_pvcs(pod: dict) -> list:
    vols = (pod.get("spec") or {}).get("volumes") or []
    return [v["persistentVolumeClaim"]["claimName"] for v in vols if v.get("persistentVolumeClaim")]


def notebooks_using_pvc(pvc: str, notebooks: list) -> list:
    return [nb["metadata"]["name"] for nb in notebooks if pvc in notebook_pvcs(nb)]


def pods_using_pvc(pvc: str, namespace: str) -> list:
    return [p for p in api.list_pods(namespace)["items"] if pvc in pod_pvcs(p)]


def parse_pvc(pvc: dict, notebooks: list) -> dict:
    try:
        capacity = pvc["status"]["capacity"]["storage"]
    except (KeyError, TypeError):
        capacity = pvc["spec"]["resources"]["requests"]["storage"]
    return {"name": pvc["metadata"]["name"], "namespace": pvc["metadata"]["namespace"], "status": pvc_status(pvc),
            "age": pvc["metadata"]["creationTimestamp"], "capacity": capacity, "modes": pvc["spec"].get("accessModes"),
            "class": pvc["spec"].get("storageClassName"), "notebooks": notebooks_using_pvc(pvc["metadata"]["name"], notebooks)}


# ---- viewers -----------------------------------------------------------------------------------
def substitute(data, variables: dict):
    """$VAR / ${VAR} expansion in every string of the template (unknown names fail the request,
    malformed templates stay literal), like string.Template.substitute."""
    if isinstance(data, dict):
        return {k: substitute(v, variables) for k, v in data.items()}
    if isinstance(data, list):
        return [substitute(v, variables) for v in data]
    if isinstance(data, str):
        try:
            return Template(data).substitute(**variables)
        except ValueError:
            return data
        except KeyError as e:
            raise exceptions.InternalServerError(f"viewer-spec.yaml references undefined variable {e}")
    return data


def load_viewer_spec() -> dict:
    paths = [os.environ["VIEWER_SPEC_PATH"]] if os.environ.get("VIEWER_SPEC_PATH") else VIEWER_SPEC_PATHS
    for p in paths:
        if os.path.exists(p):
            with open(p) as f:
                return yaml.safe_load(f) or {}
    raise exceptions.NotFound("viewer-spec.yaml not found")


def create_viewer_template(name: str, namespace: str) -> dict:
    variables = {"VOLUME_VIEWER_IMAGE": DEFAULT_VIEWER_IMAGE, **os.environ,
                 "PVC_NAME": name, "NAMESPACE": namespace, "NAME": name}
    spec = substitute(copy.deepcopy(load_viewer_spec()), variables)
    return {"apiVersion": f"{VIEWER[0]}/{VIEWER[1]}", "kind": VIEWER[3],
            "metadata": {"name": name, "namespace": namespace}, "spec": spec}


def owning_viewer(pod: dict):
    return ((pod.get("metadata") or {}).get("labels") or {}).get(POD_PARENT_VIEWER_LABEL_KEY)


def create_app(cfg: config.Config | None = None):
    app = crud_backend.create_app(__name__, STATIC_DIR, cfg)

    def _viewer_api(verb, namespace, **kw):
        return api.custom_api(verb, VIEWER[0], VIEWER[1], VIEWER[2], VIEWER[3], namespace, **kw)

    @app.route("/api/namespaces/<namespace>/pvcs")
    def get_pvcs(namespace):
        notebooks = api.list_notebooks(namespace)["items"]
        rows = [parse_pvc(p, notebooks) for p in api.list_pvcs(namespace)["items"]]
        viewers = {v["metadata"]["name"]: v for v in _viewer_api("list", namespace)["items"]}
        for row in rows:
            v = viewers.get(row["name"], {})
            row["viewer"] = {"status": viewer_status(v), "url": (v.get("status") or {}).get("url")}
        return api.success_response("pvcs", rows)

    @app.route("/api/namespaces/<namespace>/pvcs/<pvc>")
    def get_pvc(namespace, pvc):
        return api.success_response("pvc", api.get_pvc(pvc, namespace))

    @app.route("/api/namespaces/<namespace>/pvcs/<pvc>/pods")
    def get_pvc_pods(namespace, pvc):
        return api.success_response("pods", pods_using_pvc(pvc, namespace))

    @app.route("/api/namespaces/<namespace>/pvcs/<pvc>/events")
    def get_pvc_events(namespace, pvc):
        return api.success_response("events", api.list_pvc_events(namespace, pvc)["items"])

    @app.route("/api/namespaces/<namespace>/pvcs", methods=["POST"])
    @decorators.request_is_json_type
    @decorators.required_body_params("name", "mode", "class", "size", "type")
    def post_pvc(namespace):
        api.create_pvc(pvc_from_dict(request.get_json(), namespace), namespace)
        return api.success_response("message", "PVC created successfully.")

    @app.route("/api/namespaces/<namespace>/pvcs/<pvc>", methods=["DELETE"])
    def delete_pvc(namespace, pvc):
        pods = pods_using_pvc(pvc, namespace)
        users = [p["metadata"]["name"] for p in pods if owning_viewer(p) is None]
        if users:
            raise exceptions.Conflict(f"Cannot delete PVC '{pvc}' because it is being used by pods: {users}")
        for v in {owning_viewer(p) for p in pods}:
            _viewer_api("delete", namespace, name=v)
        api.delete_pvc(pvc, namespace)
        return api.success_response("message", f"PVC {pvc} successfully deleted.")

    @app.route("/api/namespaces/<namespace>/viewers", methods=["POST"])
    @decorators.request_is_json_type
    @decorators.required_body_params("name")
    def post_viewer(namespace):
        _viewer_api("create", namespace, body=create_viewer_template(request.get_json()["name"], namespace))
        return api.success_response("message", "PVCViewer created successfully.")

    @app.route("/api/namespaces/<namespace>/viewers/<viewer>", methods=["DELETE"])
    def delete_viewer(namespace, viewer):
        _viewer_api("delete", namespace, name=viewer)
        return api.success_response("message", f"Viewer {viewer} successfully deleted.")

    return crud_backend.finalize(app)
