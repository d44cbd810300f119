"""Jupyter web app (JWA) backend: notebook spawner / list / start-stop / delete, MI355X GPUs.

Routes (reference jupyter/backend/apps/{common,default}/routes):
  GET    /api/config, /api/gpus
  GET    /api/namespaces/<ns>/{pvcs,poddefaults,notebooks}
  GET    /api/namespaces/<ns>/notebooks/<nb>[/pod[/<pod>/logs]|/events]
  POST   /api/namespaces/<ns>/notebooks              (dry-runs the CR and new PVCs first)
  PATCH  /api/namespaces/<ns>/notebooks/<nb>          {"stopped": bool}
  DELETE /api/namespaces/<ns>/notebooks/<nb>          (Foreground)
"""
from __future__ import annotations

import datetime as dt
import logging
import os

from flask import request
from werkzeug import exceptions

from kubeflow_rm_amd.webapps import crud_backend
from kubeflow_rm_amd.webapps.crud_backend import api, authn, config, helpers

from . import form, status, utils, volumes

log = logging.getLogger(__name__)
STATIC_DIR = os.path.join(os.path.abspath(os.path.dirname(__file__)), "static")


def _json_body():
    if not request.is_json:
        raise exceptions.BadRequest("Request is not JSON type")
    body = request.get_json(silent=True)
    if body is None:
        raise exceptions.BadRequest("Request doesn't have a body.")
    return body


def create_app(cfg: config.Config | None = None):
    app = crud_backend.create_app(__name__, STATIC_DIR, cfg)

    @app.route("/api/config")
    def get_config():
        return api.success_response("config", utils.load_spawner_ui_config())

    @app.route("/api/namespaces/<namespace>/pvcs")
    def get_pvcs(namespace):
        data = [{"name": p["metadata"]["name"], "size": p["spec"]["resources"]["requests"]["storage"],
                 "mode": p["spec"]["accessModes"][0]} for p in api.list_pvcs(namespace)["items"]]
        return api.success_response("pvcs", data)

    @app.route("/api/namespaces/<namespace>/poddefaults")
    def get_poddefaults(namespace):
        out = []
        for pd in api.list_poddefaults(namespace)["items"]:
            pd["label"] = list(pd["spec"]["selector"]["matchLabels"].keys())[0]
            pd["desc"] = pd["spec"].get("desc", pd["metadata"]["name"])
            out.append(pd)
        return api.success_response("poddefaults", out)

    @app.route("/api/namespaces/<namespace>/notebooks")
    def get_notebooks(namespace):
        return api.success_response("notebooks", [utils.notebook_dict_from_k8s_obj(nb)
                                                  for nb in api.list_notebooks(namespace)["items"]])

    @app.route("/api/namespaces/<namespace>/notebooks/<name>")
    def get_notebook(namespace, name):
        nb = api.get_notebook(name, namespace)
        nb["processed_status"] = status.process_status(nb)
        return api.success_response("notebook", nb)

    @app.route("/api/namespaces/<namespace>/notebooks/<name>/pod")
    def get_notebook_pod(namespace, name):
        pods = api.list_pods(namespace, label_selector="notebook-name=" + name)["items"]
        if not pods:
            raise exceptions.NotFound("No pod detected.")
        return api.success_response("pod", pods[0])

    @app.route("/api/namespaces/<namespace>/notebooks/<name>/pod/<pod>/logs")
    def get_pod_logs(namespace, name, pod):
        return api.success_response("logs", api.get_pod_logs(namespace, pod, name).split("\n"))

    @app.route("/api/namespaces/<namespace>/notebooks/<name>/events")
    def get_notebook_events(namespace, name):
        return api.success_response("events", api.list_notebook_events(name, namespace)["items"])

    @app.route("/api/gpus")
    def get_gpu_vendors():
        keys = [v.get("limitsKey", "") for v in utils.load_spawner_ui_config().get("gpus", {}).get("value", {}).get("vendors", [])]
        installed = set()
        for node in api.list_nodes()["items"]:
            installed.update(((node.get("status") or {}).get("capacity") or {}).keys())
        return api.success_response("vendors", sorted(installed.intersection(keys)))

    @app.route("/api/namespaces/<namespace>/notebooks", methods=["POST"])
    def post_notebook(namespace):
        body = _json_body()
        if "name" not in body:
            raise exceptions.BadRequest("Request body is missing the 'name' field")
        body.setdefault("namespace", namespace)
        user = authn.get_username()
        nb = utils.new_notebook(body["name"], namespace, service_account="default-editor",
                                creator=user if user is not None else "anonymous@kubeflow.org")
        defaults = utils.load_spawner_ui_config()
        for setter in (form.set_notebook_image, form.set_notebook_image_pull_policy, form.set_server_type,
                       form.set_notebook_cpu, form.set_notebook_memory, form.set_notebook_gpus,
                       form.set_notebook_tolerations, form.set_notebook_affinity, form.set_notebook_configurations,
                       form.set_notebook_shm, form.set_notebook_environment):
            setter(nb, body, defaults)
        api_volumes = list(form.get_form_value(body, defaults, "datavols", "dataVolumes") or [])
        workspace = form.get_form_value(body, defaults, "workspace", "workspaceVolume", optional=True)
        if workspace:
            api_volumes.append(workspace)
        # dry-run everything first so nothing is left behind when one object is invalid
        api.create_notebook(nb, namespace, dry_run=True)
        new_pvcs = [volumes.get_new_pvc(v, body["name"]) for v in api_volumes]
        for pvc in new_pvcs:
            if pvc is not None:
                api.create_pvc(pvc, namespace, dry_run=True)
        for v, pvc in zip(api_volumes, new_pvcs):
            if pvc is not None:
                pvc = api.create_pvc(pvc, namespace)
            pod_vol = volumes.get_pod_volume(v, pvc)
            volumes.add_notebook_volume(nb, pod_vol)
            volumes.add_notebook_container_mount(nb, volumes.get_container_mount(v, pod_vol["name"]))
        api.create_notebook(nb, namespace)
        return api.success_response("message", "Notebook created successfully.")

    @app.route("/api/namespaces/<namespace>/notebooks/<name>", methods=["PATCH"])
    def patch_notebook(namespace, name):
        body = _json_body()
        if "stopped" not in body:
            raise exceptions.BadRequest("Request body must include at least one supported key: ['stopped']")
        if body["stopped"]:
            nb = api.get_notebook(name, namespace)
            if status.STOP_ANNOTATION in ((nb.get("metadata") or {}).get("annotations") or {}):
                raise exceptions.Conflict(f"Notebook {namespace}/{name} is already stopped.")
            ts = dt.datetime.now(dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
            patch = {"metadata": {"annotations": {status.STOP_ANNOTATION: ts}}}
        else:
            patch = {"metadata": {"annotations": {status.STOP_ANNOTATION: None}}}
        api.patch_notebook(name, namespace, patch)
        return api.success_response()

    @app.route("/api/namespaces/<namespace>/notebooks/<name>", methods=["DELETE"])
    def delete_notebook(namespace, name):
        api.delete_notebook(name, namespace)
        return api.success_response("message", f"Notebook {name} successfully deleted.")

    return crud_backend.finalize(app)
