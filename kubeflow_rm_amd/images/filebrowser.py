"""File browser for PVCViewer pods (the filebrowser/filebrowser image's role).

Env (same as the reference default podSpec): FB_ADDRESS, FB_PORT, FB_BASEURL, FB_NOAUTH,
FB_DATABASE; the root is the container working dir (/data = the viewer-volume PVC).
REST (filebrowser-compatible subset, relative to FB_BASEURL):
  GET    /api/resources/<path>   directory listing {"items": [...]} or file info
  GET    /api/raw/<path>         download
  POST   /api/resources/<path>   upload (body = content); directories when path ends in "/"
  DELETE /api/resources/<path>   remove
  GET    /health
"""
from __future__ import annotations

import html
import os
import shutil
import sys
from urllib.parse import unquote, urlparse

from kubeflow_rm_amd.images._http import JsonHandler, resolve_path, serve


def _info(root: str, rel: str) -> dict:
    p = os.path.join(root, rel)
    st = os.stat(p)
    return {"name": os.path.basename(rel.rstrip("/")) or "/", "path": "/" + rel, "size": st.st_size,
            "isDir": os.path.isdir(p), "modified": st.st_mtime}


def make_handler(root: str, base: str):
    def safe(rel: str) -> str | None:
        full = os.path.realpath(os.path.join(root, rel))
        return full if full == os.path.realpath(root) or full.startswith(os.path.realpath(root) + os.sep) else None

    class H(JsonHandler):
        def _rel(self):
            path = unquote(urlparse(self.path).path)
            if base and path.startswith(base.rstrip("/")):
                path = path[len(base.rstrip("/")):]
            return path

        def do_GET(self):
            path = self._rel()
            if path in ("/health", "/healthz"):
                return self.send_json(200, {"status": "OK"})
            if path.startswith("/api/resources"):
                rel = path[len("/api/resources"):].lstrip("/")
                full = safe(rel)
                if not full or not os.path.exists(full):
                    return self.send_json(404, {"error": "not found"})
                if os.path.isdir(full):
                    items = [_info(root, os.path.join(rel, n)) for n in sorted(os.listdir(full))]
                    return self.send_json(200, {**_info(root, rel), "items": items})
                return self.send_json(200, _info(root, rel))
            if path.startswith("/api/raw/"):
                full = safe(path[len("/api/raw/"):])
                if not full or not os.path.isfile(full):
                    return self.send_json(404, {"error": "not found"})
                with open(full, "rb") as f:
                    data = f.read()
                self.send_response(200)
                self.send_header("Content-Type", "application/octet-stream")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)
                return
            # HTML listing for browsers
            rel = path.lstrip("/")
            full = safe(rel)
            if not full or not os.path.isdir(full):
                return self.send_json(404, {"error": "not found"})
            rows = "".join(f"<li>{html.escape(n)}{'/' if os.path.isdir(os.path.join(full, n)) else ''}</li>"
                           for n in sorted(os.listdir(full)))
            self.send_text(200, f"<!doctype html><title>Files</title><h1>/{html.escape(rel)}</h1><ul>{rows}</ul>",
                           "text/html; charset=utf-8")

        def do_POST(self):
            path = self._rel()
            if not path.startswith("/api/resources/"):
                return self.send_json(404, {"error": "not found"})
            rel = path[len("/api/resources/"):]
            full = safe(rel)
            if not full:
                return self.send_json(403, {"error": "outside root"})
            if rel.endswith("/"):
                os.makedirs(full, exist_ok=True)
            else:
                os.makedirs(os.path.dirname(full), exist_ok=True)
                n = int(self.headers.get("Content-Length") or 0)
                with open(full, "wb") as f:
                    f.write(self.rfile.read(n))
            self.send_json(200, _info(root, rel.rstrip("/")))

        def do_DELETE(self):
            path = self._rel()
            full = safe(path[len("/api/resources/"):]) if path.startswith("/api/resources/") else None
            if not full or full == os.path.realpath(root) or not os.path.exists(full):
                return self.send_json(404, {"error": "not found"})
            shutil.rmtree(full) if os.path.isdir(full) else os.remove(full)
            self.send_json(200, {"deleted": path})
    return H


def main(argv=None) -> int:
    port = int(os.environ.get("FB_PORT", "8080"))
    base = os.environ.get("FB_BASEURL", "/")
    root = os.getcwd()
    wd = os.environ.get("KFAMD_WORKDIR")
    if wd:
        root = resolve_path(wd)
    os.makedirs(root, exist_ok=True)
    srv = serve(make_handler(root, base), port)
    print(f"filebrowser serving {root} at {base} on {srv.server_address[0]}:{port}", flush=True)
    srv.serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())
