"""TensorBoards web app (TWA) backend (reference crud-web-apps/tensorboards/backend/app).

Routes:
  GET    /api/namespaces/<ns>/tensorboards      rows {name, namespace, logspath, age, status}
  GET    /api/namespaces/<ns>/pvcs              PVC names (for pvc:// log paths)
  GET    /api/namespaces/<ns>/poddefaults       with label/desc for the configuration picker
  POST   /api/namespaces/<ns>/tensorboards      {name, logspath, configurations?: [label]}
  DELETE /api/namespaces/<ns>/tensorboards/<tb>
The Tensorboard CR (tensorboard.kubeflow.org/v1alpha1) is reconciled by the native tensorboard
controller (native/controllers/tensorboard.cc); its server is kubeflow_rm_amd.images.tensorboard_server.
"""
from __future__ import annotations

import os

from flask import request
from werkzeug.exceptions import BadRequest

from kubeflow_rm_amd.webapps import crud_backend
from kubeflow_rm_amd.webapps.crud_backend import api, config, decorators
from kubeflow_rm_amd.webapps.crud_backend.status import STATUS_PHASE, create_status

STATIC_DIR = os.path.join(os.path.abspath(os.path.dirname(__file__)), "static")
TB = ("tensorboard.kubeflow.org", "v1alpha1", "tensorboards", "Tensorboard")


def parse_tensorboard(tb: dict) -> dict:
    if (tb.get("status") or {}).get("readyReplicas", 0) == 1:
        st = create_status(STATUS_PHASE.READY, "The Tensorboard server is ready to connect")
    else:
        st = create_status(STATUS_PHASE.UNAVAILABLE, "The Tensorboard server is currently unavailable")
    return {"name": tb["metadata"]["name"], "namespace": tb["metadata"]["namespace"],
            "logspath": tb["spec"]["logspath"], "age": tb["metadata"]["creationTimestamp"], "status": st}


def configuration_labels(body: dict) -> dict:
    labels = body.get("configurations", [])
    if not isinstance(labels, list):
        raise BadRequest(f"Labels for PodDefaults are not list: {labels}")
    return {label: "true" for label in labels}


def tensorboard_from_body(namespace: str, body: dict) -> dict:
    md = {"name": body["name"], "namespace": namespace}
    labels = configuration_labels(body)
    if labels:
        md["labels"] = labels
    return {"apiVersion": f"{TB[0]}/{TB[1]}", "kind": TB[3], "metadata": md, "spec": {"logspath": body["logspath"]}}


def create_app(cfg: config.Config | None = None):
    app = crud_backend.create_app(__name__, STATIC_DIR, cfg)

    @app.route("/api/namespaces/<namespace>/tensorboards")
    def get_tensorboards(namespace):
        items = api.custom_api("list", TB[0], TB[1], TB[2], TB[3], namespace)["items"]
        return api.success_response("tensorboards", [parse_tensorboard(t) for t in items])

    @app.route("/api/namespaces/<namespace>/pvcs")
    def get_pvcs(namespace):
        return api.success_response("pvcs", [p["metadata"]["name"] for p in api.list_pvcs(namespace)["items"]])

    @app.route("/api/namespaces/<namespace>/poddefaults")
    def get_poddefaults(namespace):
        out = []
        for pd in api.list_poddefaults(namespace)["items"]:
            pd["label"] = list(pd["spec"]["selector"]["matchLabels"].keys())[0]
            pd["desc"] = pd["spec"].get("desc", pd["metadata"]["name"])
            out.append(pd)
        return api.success_response("poddefaults", out)

    @app.route("/api/namespaces/<namespace>/tensorboards", methods=["POST"])
    @decorators.request_is_json_type
    @decorators.required_body_params("name", "logspath")
    def post_tensorboard(namespace):
        tb = tensorboard_from_body(namespace, request.get_json())
        api.custom_api("create", TB[0], TB[1], TB[2], TB[3], namespace, body=tb)
        return api.success_response("message", "Tensorboard created successfully.")

    @app.route("/api/namespaces/<namespace>/tensorboards/<name>", methods=["DELETE"])
    def delete_tensorboard(namespace, name):
        api.custom_api("delete", TB[0], TB[1], TB[2], TB[3], namespace, name=name)
        return api.success_response("message", "Tensorboard deleted successfully.")

    return crud_backend.finalize(app)
