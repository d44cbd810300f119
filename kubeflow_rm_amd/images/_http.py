"""Tiny stdlib HTTP helpers shared by the process images (fast cold start: no Flask import)."""
from __future__ import annotations

import json
import os
import socket
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


class Server(ThreadingHTTPServer):
    daemon_threads = True
    allow_reuse_address = True


def bind_host() -> str:
    """Where a process pod's server listens: its private app address behind the node's inbound
    enforcement listener when the pod is mesh-injected (KFAMD_BIND_IP), else the pod IP."""
    return os.environ.get("KFAMD_BIND_IP") or os.environ.get("POD_IP", "127.0.0.1")


def serve(handler_cls, port: int, host: str | None = None) -> Server:
    srv = Server((host or bind_host(), port), handler_cls)
    return srv


class JsonHandler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "kflite-image/1.0"

    def log_message(self, fmt, *args):  # quiet access log -> container log
        if os.environ.get("KFAMD_ACCESS_LOG"):
            super().log_message(fmt, *args)

    def send_json(self, code: int, obj, headers: dict | None = None):
        body = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        for k, v in (headers or {}).items():
            self.send_header(k, v)
        self.end_headers()
        self.wfile.write(body)

    def send_text(self, code: int, text: str, ctype: str = "text/plain; charset=utf-8"):
        body = text.encode()
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def read_json(self):
        n = int(self.headers.get("Content-Length") or 0)
        if n <= 0:
            return {}
        try:
            return json.loads(self.rfile.read(n) or b"{}")
        except ValueError:
            return {}


def run_forever(servers):
    threads = []
    for s in servers[1:]:
        t = threading.Thread(target=s.serve_forever, daemon=True)
        t.start()
        threads.append(t)
    servers[0].serve_forever()


def port_free(host: str, port: int) -> bool:
    with socket.socket() as s:
        try:
            s.bind((host, port))
            return True
        except OSError:
            return False


def mounts() -> dict:
    """Container mountPath -> host directory for this process pod (set by the kflite kubelet)."""
    try:
        return json.loads(os.environ.get("KFAMD_VOLUME_MOUNTS") or "{}")
    except ValueError:
        return {}


def resolve_path(container_path: str) -> str:
    """Translate a path as the container sees it into the host path backing it (longest mount
    prefix wins; anything else lives under the pod's rootfs)."""
    best = ""
    for mp in mounts():
        norm = mp.rstrip("/") or "/"
        if (container_path == norm or container_path.startswith(norm.rstrip("/") + "/")) and len(norm) > len(best):
            best = norm
    if best:
        rest = container_path[len(best):].lstrip("/")
        return os.path.join(mounts().get(best) or mounts().get(best + "/"), rest)
    root = os.environ.get("KFAMD_ROOTFS")
    if root and os.path.isabs(container_path):
        return os.path.join(root, container_path.lstrip("/"))
    return container_path
