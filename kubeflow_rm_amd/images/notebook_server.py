"""Jupyter-server-compatible notebook image (jupyter / jupyter-pytorch-rocm / codeserver / rstudio).

Contract (reference components/example-notebook-servers/README.md, "Image Requirements"):
HTTP on :8888, everything under the NB_PREFIX base URL, user home = $HOME (workspace PVC),
and the Jupyter REST endpoints the culler polls (notebook-controller/controllers/culling_controller.go:209-293):
  GET  {prefix}/api/kernels   -> [{id, name, last_activity, execution_state, connections}]
  GET  {prefix}/api/terminals -> [{name, last_activity}]
Kernels/terminals can be created (POST), deleted (DELETE) and driven busy/idle
(POST {prefix}/api/kernels/{id}/execute {"seconds": s}) so culling is testable end to end.
Requests that arrive without the prefix (rewritten routes of group-one / group-two servers) are
served too. GET {prefix}/api/gpu reports the GPUs this pod was given (HIP_VISIBLE_DEVICES) and
the readiness-op result when present.
"""
from __future__ import annotations

import datetime as _dt
import json
import os
import sys
import threading
import time
import uuid

from ._http import JsonHandler, run_forever, serve

_LOCK = threading.Lock()
KERNELS: dict[str, dict] = {}
TERMINALS: dict[str, dict] = {}
STARTED = time.time()


def _now() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def _kernel_view(k: dict) -> dict:
    busy_until = k.get("_busy_until", 0)
    state = "busy" if busy_until > time.time() else "idle"
    if state == "idle" and k.get("_was_busy"):
        k["last_activity"] = _dt.datetime.fromtimestamp(busy_until, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")
        k["_was_busy"] = False
    return {"id": k["id"], "name": k["name"], "last_activity": k["last_activity"],
            "execution_state": state, "connections": k.get("connections", 0)}


def make_handler(prefix: str):
    prefix = prefix.rstrip("/")

    class H(JsonHandler):
        def _route(self):
            path = self.path.split("?", 1)[0]
            if prefix and path.startswith(prefix):
                path = path[len(prefix):] or "/"
            return path

        def do_GET(self):
            p = self._route()
            if p in ("/api", "/api/"):
                return self.send_json(200, {"version": "2.14.0-kflite"})
            if p == "/api/status":
                with _LOCK:
                    return self.send_json(200, {"started": _dt.datetime.fromtimestamp(STARTED, _dt.timezone.utc).isoformat(),
                                                "kernels": len(KERNELS), "connections": 0,
                                                "last_activity": _now()})
            if p.rstrip("/") == "/api/kernels":
                with _LOCK:
                    return self.send_json(200, [_kernel_view(k) for k in KERNELS.values()])
            if p.startswith("/api/kernels/"):
                kid = p.split("/")[3]
                with _LOCK:
                    k = KERNELS.get(kid)
                    return self.send_json(200, _kernel_view(k)) if k else self.send_json(404, {"message": "kernel not found"})
            if p.rstrip("/") == "/api/terminals":
                with _LOCK:
                    return self.send_json(200, [{"name": t["name"], "last_activity": t["last_activity"]}
                                                for t in TERMINALS.values()])
            if p == "/api/gpu":
                info = {"HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES"),
                        "ring": os.environ.get("KFAMD_XGMI_RING"),
                        "topology": os.environ.get("KFAMD_GPU_TOPOLOGY")}
                return self.send_json(200, info)
            if p in ("/", "/lab", "/tree", "/lab/"):
                html = (f"<html><head><title>kflite notebook</title></head><body><h1>Notebook server</h1>"
                        f"<p>base url: {prefix}/</p><p>home: {os.environ.get('HOME')}</p></body></html>")
                return self.send_text(200, html, "text/html; charset=utf-8")
            return self.send_json(404, {"message": f"not found: {p}"})

        def do_POST(self):
            p = self._route()
            body = self.read_json()
            if p.rstrip("/") == "/api/kernels":
                kid = str(uuid.uuid4())
                k = {"id": kid, "name": body.get("name", "python3"), "last_activity": _now(), "connections": 0}
                with _LOCK:
                    KERNELS[kid] = k
                    return self.send_json(201, _kernel_view(k))
            if p.startswith("/api/kernels/") and p.endswith("/execute"):
                kid = p.split("/")[3]
                with _LOCK:
                    k = KERNELS.get(kid)
                    if not k:
                        return self.send_json(404, {"message": "kernel not found"})
                    k["_busy_until"] = time.time() + float(body.get("seconds", 1))
                    k["_was_busy"] = True
                    k["last_activity"] = _now()
                    return self.send_json(200, _kernel_view(k))
            if p.rstrip("/") == "/api/terminals":
                with _LOCK:
                    name = str(len(TERMINALS) + 1)
                    TERMINALS[name] = {"name": name, "last_activity": _now()}
                    return self.send_json(200, TERMINALS[name])
            return self.send_json(404, {"message": "not found"})

        def do_DELETE(self):
            p = self._route()
            parts = p.strip("/").split("/")
            with _LOCK:
                if len(parts) == 3 and parts[1] == "kernels" and KERNELS.pop(parts[2], None):
                    return self.send_json(204, {})
                if len(parts) == 3 and parts[1] == "terminals" and TERMINALS.pop(parts[2], None):
                    return self.send_json(204, {})
            return self.send_json(404, {"message": "not found"})

    return H


def main(argv=None) -> int:
    prefix = os.environ.get("NB_PREFIX", "")
    port = int(os.environ.get("NB_PORT", (os.environ.get("KFAMD_CONTAINER_PORTS") or "8888").split(",")[0] or 8888))
    srv = serve(make_handler(prefix), port)
    print(f"[kflite-notebook] serving {prefix or '/'} on {srv.server_address[0]}:{port} home={os.environ.get('HOME')}",
          flush=True)
    run_forever([srv])
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
