"""Start / stop an embedded kflite control plane (the envtest equivalent).

    with LocalCluster(env={"USE_ISTIO": "true"}) as c:
        c.client.create(notebook)

The process is started in its own session; stop() terminates exactly that process group
(never by pattern), and the kubelet inside tears down every pod process it started.
"""
from __future__ import annotations

import json
import secrets
import os
import random
import signal
import subprocess
import tempfile
import time
from pathlib import Path

from .client import KubeClient

ROOT = Path(__file__).resolve().parent.parent
# KFAMD_BIN_DIR: another build of the native binaries (tools/sanitize.sh points it at the TSAN /
# ASan builds, so the split components run instrumented too)
BIN = Path(os.environ.get("KFAMD_BIN_DIR") or Path(__file__).resolve().parent / "bin")


def kflite_binary() -> Path:
    p = Path(os.environ.get("KFAMD_KFLITE", BIN / "kflite"))
    if not p.exists():
        raise FileNotFoundError(f"{p} missing: build with `python -m kubeflow_rm_amd._build native`")
    return p


class LocalCluster:
    def __init__(self, data_dir: str | None = None, env: dict | None = None, args: list[str] | None = None,
                 controllers: str = "all", gpus: int | None = 8, startup_timeout: float = 30.0,
                 ca_file: str | None = None, zygote: bool | None = False, users: list[str] | dict | None = None):
        self._tmp = None
        # end users with bearer tokens (kflite --token-auth-file): the gateway authenticates them and
        # sets the userid header from the token (never from the client); ``user_headers(name)``
        self.users: dict[str, str] = {}
        for u in (users or []):
            self.users[u] = (users[u] if isinstance(users, dict) else "") or "tok-" + secrets.token_hex(16)
        # kubelet --pod-zygote (kflite's default): Python containers fork from a pre-imported
        # interpreter. False here by default: a test / dev cluster skips the per-node torch import
        # unless it asks for it; None = kflite's default
        self.zygote = zygote
        if data_dir is None:
            self._tmp = tempfile.TemporaryDirectory(prefix="kflite-")
            data_dir = self._tmp.name
        self.data_dir = data_dir
        self.env = dict(os.environ)
        self.env.update(env or {})
        self.args = list(args or [])
        self.controllers = controllers
        self.gpus = gpus
        self.startup_timeout = startup_timeout
        self.ca_file = ca_file  # verifies an https API server (kflite --tls-cert-file ...)
        self.proc: subprocess.Popen | None = None
        self.url = ""
        self.gateway = ""
        self.kfam = ""
        self.mesh = ""
        self.client: KubeClient | None = None

    def start(self) -> "LocalCluster":
        info = Path(self.data_dir) / "kflite.json"
        if info.exists():
            info.unlink()
        cmd = [str(kflite_binary()), "--data-dir", self.data_dir, "--controllers", self.controllers,
               "--restart-backoff", self.env.get("KFAMD_RESTART_BACKOFF", "1")]
        if self.gpus is not None:
            cmd += ["--gpus", str(self.gpus)]
        if not any(a.startswith("--pod-cidr-prefix") for a in self.args):
            # every pod listens on <pod-ip>:8888; a private loopback /16 per cluster keeps clusters
            # that overlap in time (pytest-xdist workers, a previous cluster's pods still in their
            # termination grace period) from answering each other's requests
            cmd += ["--pod-cidr-prefix", f"127.{random.randint(20, 250)}"]
        if not any(a.startswith("--repo-root") for a in self.args):
            # explicit: a kflite built elsewhere (sanitizer builds under build/) cannot derive the
            # package root from its own path, and pod image recipes run `python -m kubeflow_rm_amd...`
            cmd += ["--repo-root", str(ROOT)]
        if self.users and not any(a.startswith("--token-auth-file") for a in self.args):
            tf = Path(self.data_dir) / "tokens.json"
            tf.write_text(json.dumps({t: {"username": u, "groups": ["system:authenticated"]} for u, t in self.users.items()}))
            os.chmod(tf, 0o600)
            cmd += ["--token-auth-file", str(tf)]
        if self.zygote is not None and not any(a.startswith("--pod-zygote") for a in self.args):
            cmd += ["--pod-zygote" if self.zygote else "--pod-zygote=false"]
        cmd += self.args
        self.log_path = Path(self.data_dir) / "kflite.log"
        self._log = open(self.log_path, "ab")
        self.proc = subprocess.Popen(cmd, stdout=self._log, stderr=subprocess.STDOUT, env=self.env,
                                     start_new_session=True)
        deadline = time.time() + self.startup_timeout
        while time.time() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError(f"kflite exited early ({self.proc.returncode}):\n{self.log_path.read_text()[-3000:]}")
            if info.exists():
                try:
                    d = json.loads(info.read_text())
                except ValueError:
                    d = {}
                if d.get("server") and "gateway" in d:
                    self.url = d["server"]
                    self.gateway = d.get("gateway", "")
                    self.kfam = d.get("kfam", "")
                    self.mesh = d.get("mesh", "")
                    break
            time.sleep(0.02)
        else:
            self.stop()
            raise TimeoutError("kflite did not come up")
        self.client = KubeClient(self.url, ca_file=self.ca_file)
        return self

    def wait_zygotes(self, timeout: float = 120.0) -> list[str]:
        """Block until the kubelet's zygotes serve (their sockets exist), like waiting for a node's
        image pre-pull; returns the socket paths. The first ``import torch`` on a fresh machine can
        take a minute or two."""
        root = Path(self.data_dir) / "kubelet"
        deadline = time.time() + timeout
        while time.time() < deadline:
            socks = sorted(str(p) for p in root.glob("zygote-*.sock"))
            logs = sorted(root.glob("zygote-*.log"))
            if socks and len(socks) >= len(logs):
                self.wait_warm(max(0.0, deadline - time.time()))
                return socks
            for lg in logs:
                t = lg.read_text(errors="replace")
                if "refusing to serve" in t or "Traceback" in t:
                    raise RuntimeError(f"zygote failed: {t[-2000:]}")
            time.sleep(0.05)
        raise TimeoutError("zygote did not come up")

    def wait_warm(self, timeout: float = 30.0) -> dict:
        """Block until every zygote started with warm GPU children has reported each of them ready or
        failed (zygote.py: "[zygote] warm child <pid> for device <d> ready|failed"); a zygote without
        warm devices returns at once. Returns {device: "ready" | "failed"} of the last report each."""
        import re
        root = Path(self.data_dir) / "kubelet"
        deadline = time.time() + timeout
        state: dict = {}
        while True:
            want = set()
            for lg in root.glob("zygote-*.log"):
                t = lg.read_text(errors="replace")
                for dev, what in re.findall(r"warm child \d+ for device (\d+) (ready|failed)", t):
                    state[int(dev)] = what
            try:
                cmdlines = [open(f"/proc/{p}/cmdline", "rb").read().split(b"\0") for p in os.listdir("/proc") if p.isdigit()]
            except OSError:
                cmdlines = []
            for cl in cmdlines:
                if b"kubeflow_rm_amd.images.zygote" in cl and b"--warm-devices" in cl and str(root).encode() in b" ".join(cl):
                    i = cl.index(b"--warm-devices")
                    want |= {int(x) for x in cl[i + 1].decode().split(",") if x}
            if want <= set(state) or time.time() > deadline:
                return state
            time.sleep(0.05)

    def stop(self) -> None:
        if self.proc and self.proc.poll() is None:
            try:
                os.killpg(self.proc.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
            try:
                self.proc.wait(timeout=20)
            except subprocess.TimeoutExpired:
                os.killpg(self.proc.pid, signal.SIGKILL)
                self.proc.wait(timeout=10)
        if getattr(self, "_log", None):
            self._log.close()
            self._log = None
        if self._tmp:
            self._tmp.cleanup()
            self._tmp = None

    def user_headers(self, user: str) -> dict:
        """Request headers that authenticate ``user`` at the gateway (bearer token)."""
        return {"Authorization": f"Bearer {self.users[user]}"}

    def logs(self) -> str:
        try:
            return self.log_path.read_text()
        except OSError:
            return ""

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
