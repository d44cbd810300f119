"""TensorBoard-compatible scalar server for the Tensorboard CR (`tensorboard --logdir=... --bind_all`).

Serves the TensorBoard HTTP data API subset used by scalar dashboards:
  GET /                                   minimal HTML dashboard (runs, tags, latest values)
  GET /data/runs                          ["run", ...]
  GET /data/plugins_listing               {"scalars": {...}}
  GET /data/plugin/scalars/tags           {run: {tag: {"displayName", "description"}}}
  GET /data/plugin/scalars/scalars?run=&tag=   [[wall_time, step, value], ...]
Event files are parsed with kubeflow_rm_amd.utils.tfevents (no TensorFlow in the image).
Cloud logdirs (gs://, s3://) are reported as unavailable offline.
"""
from __future__ import annotations

import argparse
import html
import os
import sys
import threading
import time
from urllib.parse import parse_qs, urlparse

from kubeflow_rm_amd.images._http import JsonHandler, resolve_path, serve
from kubeflow_rm_amd.utils import tfevents


class Store:
    def __init__(self, logdir: str, reload_s: float = 5.0):
        self.logdir = logdir
        self.reload_s = reload_s
        self._lock = threading.Lock()
        self._cache: dict[str, tuple[float, dict]] = {}  # file -> (mtime, scalars)
        self._loaded = 0.0
        self._runs: dict[str, dict] = {}

    def runs(self) -> dict[str, dict]:
        with self._lock:
            if time.time() - self._loaded > self.reload_s:
                self._reload()
            return self._runs

    def _reload(self):
        runs = {}
        if os.path.isdir(self.logdir):
            for run, files in tfevents.find_runs(self.logdir).items():
                merged: dict[str, list] = {}
                for f in files:
                    try:
                        m = os.path.getmtime(f)
                        c = self._cache.get(f)
                        if not c or c[0] != m:
                            c = (m, tfevents.read_scalars(f))
                            self._cache[f] = c
                    except (OSError, ValueError):
                        continue
                    for tag, pts in c[1].items():
                        merged.setdefault(tag, []).extend(pts)
                for pts in merged.values():
                    pts.sort(key=lambda p: (p[1], p[0]))
                runs[run] = merged
        self._runs = runs
        self._loaded = time.time()


def make_handler(store: Store, cloud: str | None):
    class H(JsonHandler):
        def do_GET(self):
            u = urlparse(self.path)
            q = {k: v[0] for k, v in parse_qs(u.query).items()}
            p = u.path.rstrip("/") or "/"
            runs = store.runs()
            if p in ("/", "/index.html"):
                rows = []
                for run, tags in sorted(runs.items()):
                    for tag, pts in sorted(tags.items()):
                        last = pts[-1]
                        rows.append(f"<tr><td>{html.escape(run)}</td><td>{html.escape(tag)}</td><td>{last[1]}</td>"
                                    f"<td>{last[2]:.6g}</td><td>{len(pts)}</td></tr>")
                note = f"<p>logdir {html.escape(cloud)} is a cloud path (not reachable offline)</p>" if cloud else ""
                self.send_text(200, "<!doctype html><title>TensorBoard</title><h1>TensorBoard (kfamd)</h1>" + note +
                               "<table border=1><tr><th>run</th><th>tag</th><th>step</th><th>value</th><th>points</th></tr>"
                               + "".join(rows) + "</table>", "text/html; charset=utf-8")
            elif p == "/data/runs":
                self.send_json(200, sorted(runs))
            elif p == "/data/plugins_listing":
                self.send_json(200, {"scalars": {"disable_reload": False, "enabled": True, "loading_mechanism": {"type": "NONE"},
                                                 "tab_name": "scalars"}})
            elif p == "/data/environment":
                self.send_json(200, {"data_location": cloud or store.logdir, "window_title": "TensorBoard"})
            elif p == "/data/plugin/scalars/tags":
                self.send_json(200, {r: {t: {"displayName": t, "description": ""} for t in tags} for r, tags in runs.items()})
            elif p == "/data/plugin/scalars/scalars":
                pts = runs.get(q.get("run", ""), {}).get(q.get("tag", ""))
                if pts is None:
                    self.send_json(404, {"error": "no such run/tag"})
                else:
                    self.send_json(200, [list(x) for x in pts])
            elif p in ("/healthz", "/data/status"):
                self.send_json(200, {"status": "ok"})
            else:
                self.send_json(404, {"error": "not found", "path": u.path})
    return H


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--logdir", default="/tensorboard_logs/")
    ap.add_argument("--bind_all", action="store_true")
    ap.add_argument("--port", type=int, default=6006)
    ap.add_argument("--reload_interval", type=float, default=5.0)
    a, _unknown = ap.parse_known_args(argv)
    cloud = a.logdir if a.logdir.startswith(("gs://", "s3://", "/cns/")) else None
    logdir = "" if cloud else resolve_path(a.logdir)
    srv = serve(make_handler(Store(logdir, a.reload_interval), cloud), a.port)
    print(f"TensorBoard (kfamd) serving {cloud or logdir} on {srv.server_address[0]}:{a.port}", flush=True)
    srv.serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())
