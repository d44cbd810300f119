"""Central dashboard backend + shell UI (reference components/centraldashboard/app/{server,api,
api_workgroup,attach_user_middleware}.ts).

Routes (JSON, errors as ``{"error": msg}`` with the HTTP code):
  GET  /healthz, /debug
  GET  /api/namespaces, /api/activities/<ns>, /api/dashboard-links, /api/dashboard-settings
  GET  /api/metrics, /api/metrics/<node|podcpu|podmem|gpu>?interval=Last15m   (405 without a metrics service)
  GET  /api/workgroup/exists, /api/workgroup/env-info
  POST /api/workgroup/create                       {namespace?, user?}
  -- identity required below (405 otherwise) --
  DELETE /api/workgroup/nuke-self
  GET  /api/workgroup/get-all-namespaces, /api/workgroup/get-contributors/<ns>
  POST /api/workgroup/add-contributor/<ns>         {contributor}
  DELETE /api/workgroup/remove-contributor/<ns>    {contributor}
  GET  /*  -> static shell (index.html), /library.js for iframed apps

Workgroups are KFAM bindings (native/kfam): role names map admin<->owner, edit<->contributor,
view<->viewer. Only the auth headers of the user's request (authorization, cookie, the user-id
header) are forwarded to KFAM on contributor changes.
"""
from __future__ import annotations

import json
import logging
import os
import re

from flask import Flask, jsonify, request, send_from_directory

from kubeflow_rm_amd.client import KubeClient

from .services import INTERVALS_MIN, KfamClient, KfamError, KubernetesService, make_metrics_service

log = logging.getLogger(__name__)
STATIC_DIR = os.path.join(os.path.abspath(os.path.dirname(__file__)), "static")
EMAIL_RGX = re.compile(r"^[a-zA-Z0-9.!#$%&'*+/=?^_`{|}~-]+@[a-zA-Z0-9](?:[a-zA-Z0-9-]{0,61}[a-zA-Z0-9])?"
                       r"(?:\.[a-zA-Z0-9](?:[a-zA-Z0-9-]{0,61}[a-zA-Z0-9])?)*$")
ROLE_MAP = {"admin": "owner", "owner": "admin", "edit": "contributor", "contributor": "edit",
            "view": "viewer", "viewer": "view"}
ERRORS = {"operation_not_supported": "Operation not supported",
          "invalid_links_config": "Cannot load dashboard menu link",
          "invalid_settings": "Cannot load dashboard settings"}


def api_error(error: str, code: int = 400):
    return jsonify({"error": error}), code


def attach_user(header: str, prefix: str) -> dict:
    email, auth = "anonymous@kubeflow.org", None
    v = request.headers.get(header) if header else None
    if v:
        email = v[len(prefix):]
        auth = {header: v}
    return {"email": email, "username": email.split("@")[0],
            "domain": email.split("@")[1] if "@" in email else None, "hasAuth": auth is not None, "auth": auth}


def to_simple_bindings(bindings: list) -> list:
    return [{"user": b["user"]["name"], "namespace": b["referredNamespace"], "role": ROLE_MAP.get(b["roleRef"]["name"])}
            for b in bindings]


def to_workgroup_binding(user: str, namespace: str, role: str) -> dict:
    return {"user": {"kind": "User", "name": user}, "referredNamespace": namespace,
            "roleRef": {"kind": "ClusterRole", "name": ROLE_MAP[role]}}


def create_app(k8s_client: KubeClient | None = None, kfam_url: str | None = None, metrics=None,
               registration_flow: bool | None = None) -> Flask:
    prod = os.environ.get("NODE_ENV", os.environ.get("DASHBOARD_ENV", "production")) == "production"
    user_header = os.environ.get("USERID_HEADER", "kubeflow-userid")
    user_prefix = os.environ.get("USERID_PREFIX", "")
    if registration_flow is None:
        registration_flow = os.environ.get("REGISTRATION_FLOW", "true").lower() == "true"
    if kfam_url is None:
        host = os.environ.get("PROFILES_KFAM_SERVICE_HOST", "profiles-kfam.kubeflow" if prod else "localhost")
        kfam_url = f"http://{host}:{os.environ.get('PROFILES_KFAM_SERVICE_PORT', '8081')}/kfam"
    k8s = KubernetesService(k8s_client or KubeClient())
    kfam = KfamClient(kfam_url)
    metrics = metrics if metrics is not None else make_metrics_service(k8s)
    platform_cache: dict = {}

    app = Flask(__name__, static_folder=None)
    app.config["JSON_SORT_KEYS"] = False
    app.extensions["kfamd-dashboard"] = {"k8s": k8s, "kfam": kfam, "metrics": metrics}

    def user():
        return attach_user(user_header, user_prefix)

    def platform():
        if not platform_cache:
            platform_cache.update(k8s.get_platform_info())
        return platform_cache

    def workgroup_info(u):
        return {"isClusterAdmin": kfam.is_cluster_admin(u["email"]),
                "namespaces": to_simple_bindings(kfam.read_bindings(user=u["email"]))}

    def all_workgroups(fake_user):
        names = sorted({b["namespace"] for b in to_simple_bindings(kfam.read_bindings())})
        return [{"namespace": n, "role": "contributor", "user": fake_user} for n in names]

    def contributors(ns):
        return [b["user"] for b in to_simple_bindings(kfam.read_bindings(namespace=ns)) if b["role"] == "contributor"]

    def kfam_failure(msg, e):
        if isinstance(e, KfamError):
            log.error("%s %s", msg, e.body)
            return api_error(e.body or msg, e.status)
        log.exception(msg)
        return api_error(msg, 400)

    @app.get("/healthz")
    def healthz():
        return jsonify({"codeEnvironment": "production" if prod else "development", "message": "I tick, therfore I am!"})

    @app.get("/debug")
    def debug():
        return jsonify({"user": user(), "profilesServiceUrl": kfam_url,
                        "codeEnvironment": "production" if prod else "development",
                        "registrationFlowAllowed": registration_flow,
                        "headersForIdentity": {"USERID_HEADER": user_header, "USERID_PREFIX": user_prefix}})

    # ---- /api ---------------------------------------------------------------------------------
    @app.get("/api/metrics")
    def metrics_link():
        if metrics is None:
            return api_error(ERRORS["operation_not_supported"], 405)
        return jsonify(metrics.charts_link())

    @app.get("/api/metrics/<kind>")
    def metrics_series(kind):
        if kind not in ("node", "podcpu", "podmem", "gpu"):
            return api_error("Could not find the route you're looking for", 404)
        if metrics is None:
            return api_error(ERRORS["operation_not_supported"], 405)
        interval = request.args.get("interval", "Last15m")
        if interval not in INTERVALS_MIN:
            interval = "Last15m"
        return jsonify(metrics.series(kind, interval))

    @app.get("/api/namespaces")
    def namespaces():
        return jsonify(k8s.get_namespaces())

    @app.get("/api/activities/<namespace>")
    def activities(namespace):
        return jsonify(k8s.get_events(namespace))

    def _cm_json(key, err):
        cm = k8s.get_configmap()
        try:
            return jsonify(json.loads(cm["data"][key]))
        except (TypeError, KeyError, ValueError):
            return api_error(ERRORS[err], 500)

    @app.get("/api/dashboard-links")
    def dashboard_links():
        return _cm_json("links", "invalid_links_config")

    @app.get("/api/dashboard-settings")
    def dashboard_settings():
        return _cm_json("settings", "invalid_settings")

    # ---- /api/workgroup -----------------------------------------------------------------------
    @app.get("/api/workgroup/exists")
    def wg_exists():
        u = user()
        resp = {"hasAuth": u["hasAuth"], "user": u["username"], "hasWorkgroup": False,
                "registrationFlowAllowed": registration_flow}
        try:
            if u["hasAuth"]:
                resp["hasWorkgroup"] = any(w["role"] == "owner" for w in workgroup_info(u)["namespaces"])
            else:
                resp["hasWorkgroup"] = bool(all_workgroups(u["username"]))
        except Exception as e:  # noqa: BLE001
            return kfam_failure("Unable to contact Profile Controller", e)
        return jsonify(resp)

    @app.post("/api/workgroup/create")
    def wg_create():
        u = user()
        body = request.get_json(silent=True) or {}
        ns = body.get("namespace") or u["username"]
        try:
            kfam.create_profile({"metadata": {"name": ns},
                                 "spec": {"owner": {"kind": "User", "name": body.get("user") or u["email"]}}})
        except Exception as e:  # noqa: BLE001
            return kfam_failure("Unexpected error creating profile", e)
        return jsonify({"message": f"Created namespace {ns}"})

    @app.get("/api/workgroup/env-info")
    def wg_env_info():
        u = user()
        try:
            if u["hasAuth"]:
                info = workgroup_info(u)
                return jsonify({"user": u["email"], "platform": platform(), "namespaces": info["namespaces"],
                                "isClusterAdmin": info["isClusterAdmin"]})
            return jsonify({"user": u["email"], "platform": platform(), "namespaces": all_workgroups(u["email"]),
                            "isClusterAdmin": True})
        except KfamError as e:
            return api_error(e.body or "Unexpected error getting environment info", e.status)
        except Exception:  # noqa: BLE001
            log.exception("env-info")
            return api_error("Unexpected error getting environment info", 400)

    def require_identity():
        if not user()["hasAuth"]:
            return api_error("Unable to ascertain user identity from request, cannot access route.", 405)
        return None

    @app.delete("/api/workgroup/nuke-self")
    def wg_nuke_self():
        if (r := require_identity()) is not None:
            return r
        u = user()
        try:
            body = kfam.delete_profile(u["username"], u["auth"])
        except Exception as e:  # noqa: BLE001
            return kfam_failure("Unexpected error deleting profile", e)
        return jsonify({"message": f"Removed namespace/profile {u['username']}", "serverBody": body})

    @app.get("/api/workgroup/get-all-namespaces")
    def wg_all_namespaces():
        if (r := require_identity()) is not None:
            return r
        try:
            bindings = to_simple_bindings(kfam.read_bindings())
        except Exception as e:  # noqa: BLE001
            return kfam_failure("Unable to fetch all workgroup data", e)
        table: dict = {}
        for b in bindings:
            ns = table.setdefault(b["namespace"], {"owner": None, "contributors": []})
            if b["role"] == "owner":
                ns["owner"] = b["user"]
            else:
                ns["contributors"].append(b["user"])
        return jsonify([[n, v["owner"], ", ".join(v["contributors"])] for n, v in table.items()])

    @app.get("/api/workgroup/get-contributors/<namespace>")
    def wg_contributors(namespace):
        if (r := require_identity()) is not None:
            return r
        try:
            return jsonify(contributors(namespace))
        except Exception as e:  # noqa: BLE001
            return kfam_failure(f"Unable to fetch contributors for {namespace}", e)

    def handle_contributor(action, namespace):
        if (r := require_identity()) is not None:
            return r
        contributor = (request.get_json(silent=True) or {}).get("contributor")
        missing = [f for f, v in (("contributor", contributor), ("namespace", namespace)) if not v]
        if missing:
            return api_error(f"Missing {' and '.join(missing)} field{'s' if len(missing) > 1 else ''}.")
        if not EMAIL_RGX.match(contributor):
            return api_error("Contributor doesn't look like a valid email address")
        keep = {"authorization", "cookie", user_header.lower()}
        headers = {k: v for k, v in request.headers.items() if k.lower() in keep}
        binding = to_workgroup_binding(contributor, namespace, "contributor")
        try:
            (kfam.create_binding if action == "create" else kfam.delete_binding)(binding, headers)
        except Exception as e:  # noqa: BLE001
            return kfam_failure(f"Unable to {'add new' if action == 'create' else 'remove'} contributor for {namespace}", e)
        try:
            return jsonify(contributors(namespace))
        except Exception as e:  # noqa: BLE001
            return kfam_failure(f"Unable to fetch contributors for {namespace}", e)

    @app.post("/api/workgroup/add-contributor/<namespace>")
    def wg_add(namespace):
        return handle_contributor("create", namespace)

    @app.delete("/api/workgroup/remove-contributor/<namespace>")
    def wg_remove(namespace):
        return handle_contributor("remove", namespace)

    @app.route("/api/<path:_rest>", methods=["GET", "POST", "PUT", "PATCH", "DELETE"])
    def api_not_found(_rest):
        return api_error("Could not find the route you're looking for", 404)

    # ---- static shell -------------------------------------------------------------------------
    @app.get("/")
    @app.get("/<path:path>")
    def shell(path=""):
        if path and os.path.isfile(os.path.join(STATIC_DIR, path)):
            return send_from_directory(STATIC_DIR, path)
        return send_from_directory(STATIC_DIR, "index.html")

    return app


def serve(app: Flask, default_port: int = 8082) -> None:
    from werkzeug.serving import run_simple
    port = int(os.environ.get("PORT_1") or os.environ.get("PORT")
               or (os.environ.get("KFAMD_CONTAINER_PORTS") or str(default_port)).split(",")[0])
    run_simple((os.environ.get("KFAMD_BIND_IP") or os.environ.get("POD_IP", "0.0.0.0")), port, app, threaded=True, use_reloader=False)
