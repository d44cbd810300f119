"""Jupyter-server-compatible notebook image (jupyter / jupyter-pytorch-rocm / codeserver / rstudio).

Contract (reference components/example-notebook-servers/README.md, "Image Requirements"):
HTTP on :8888, everything under the NB_PREFIX base URL, user home = $HOME (workspace PVC),
and the Jupyter REST endpoints the culler polls (notebook-controller/controllers/culling_controller.go:209-293):
  GET  {prefix}/api/kernels   -> [{id, name, last_activity, execution_state, connections}]
  GET  {prefix}/api/terminals -> [{name, last_activity}]
Kernels/terminals can be created (POST), deleted (DELETE) and driven busy/idle
(POST {prefix}/api/kernels/{id}/execute {"seconds": s}) so culling is testable end to end.
Kernel channels are a real WebSocket (RFC 6455) at {prefix}/api/kernels/{id}/channels speaking
the Jupyter messaging protocol's JSON form (kernel_info / execute requests get status, stream,
execute_reply messages; an open channel counts in the kernel's `connections`, which the culler
reads). {prefix}/api/events/stream is a text/event-stream (server-sent events) endpoint, for
checking that proxies relay responses as they are produced.
KFAMD_WARMUP=torch (the jupyter-pytorch-rocm recipe in the cold-start bench): before it listens,
the server imports torch and kubeflow_rm_amd.ops and runs one bf16 MFMA GEMM on the pod's GPU —
the kernel-runtime start that SURVEY §7.4(5) names as the dominant cold-start phase; with a
readinessProbe on {prefix}/api/status the pod is Ready only once torch can use the GPU. The
timings are served at {prefix}/api/gpu ("warmup").
Requests that arrive without the prefix (rewritten routes of group-one / group-two servers) are
served too. GET {prefix}/api/gpu reports the GPUs this pod was given (HIP_VISIBLE_DEVICES) and
the readiness-op result when present.
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import json
import os
import struct
import sys
import threading
import time
import uuid

from ._http import JsonHandler, run_forever, serve

_LOCK = threading.Lock()
KERNELS: dict[str, dict] = {}
TERMINALS: dict[str, dict] = {}
STARTED = time.time()
WARMUP: dict = {}
PREINIT: dict = {}  # cumulative ms of the HIP pre-init thread's steps


def _hip_lib() -> str | None:
    """torch's bundled libamdhip64 (same SONAME torch links, so torch reuses the initialised runtime)."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    locs = list(spec.submodule_search_locations or []) if spec else []
    return next((os.path.join(d, "lib", "libamdhip64.so") for d in locs
                 if os.path.exists(os.path.join(d, "lib", "libamdhip64.so"))), None)


def _hip_preinit_run(lib: str) -> None:
    """HIP runtime + this process's device context + the first GPU operation (the null stream's HW
    queue, the runtime's blit kernels: ~90 ms), through HIP's own entry points only (ctypes drops the
    GIL for each call). Every step stamps PREINIT (ms since the thread started) so a stall names its step."""
    import ctypes
    t = time.perf_counter()

    def stamp(k):
        PREINIT[k] = round((time.perf_counter() - t) * 1e3, 1)

    try:
        PREINIT["step"] = "dlopen"
        hip = ctypes.CDLL(lib, mode=ctypes.RTLD_GLOBAL)
        stamp("dlopen_ms")
        PREINIT["step"] = "hipInit"
        ok = hip.hipInit(0) == 0
        stamp("hip_init_ms")
        PREINIT["step"] = "context"
        if ok and hip.hipSetDevice(0) == 0:
            hip.hipFree(None)  # creates the device context now
            stamp("context_ms")
            PREINIT["step"] = "first_op"
            buf = ctypes.c_void_p()
            if hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(4096)) == 0:
                hip.hipMemset(buf, 0, ctypes.c_size_t(4096))
                hip.hipDeviceSynchronize()
                hip.hipFree(buf)
            stamp("first_op_ms")
        PREINIT["step"] = "done"
    except OSError as e:
        PREINIT["step"] = f"error: {e}"  # torch initialises on first use as usual


class _AfterTorchC:
    """sys.meta_path hook: runs ``callback`` right after the extension module ``torch._C`` has been
    created, i.e. after libtorch / libtorch_hip are loaded and every static constructor that registers
    torch's HIP fat binaries has run. The rest of ``import torch`` (~1 s of pure-Python module imports)
    then overlaps the HIP pre-init thread, and no HIP call on that thread can race a dlopen whose
    constructors call into HIP (the loader-lock / registration interleaving of the old
    whole-import overlap)."""

    def __init__(self, callback):
        self.callback = callback
        self.fired = False

    def find_spec(self, fullname, path=None, target=None):
        if fullname != "torch._C" or self.fired:
            return None
        import importlib.machinery
        spec = importlib.machinery.PathFinder.find_spec(fullname, path)
        if spec is None or spec.loader is None:
            return None
        inner, hook = spec.loader, self

        class _Loader:
            def create_module(self, s):
                m = inner.create_module(s)
                hook._fire()
                return m

            def exec_module(self, m):
                inner.exec_module(m)

        spec.loader = _Loader()
        return spec

    def _fire(self):
        if not self.fired:
            self.fired = True
            try:
                sys.meta_path.remove(self)
            except ValueError:
                pass
            self.callback()


def _preinit_hip() -> dict | None:
    """Bring up the HIP runtime and this process's device context on a side thread while the main
    thread finishes ``import torch``. KFAMD_HIP_PREINIT selects when the thread starts:

    * ``after-c`` (default): once ``torch._C`` exists (torch's HIP code objects registered); overlaps
      the Python half of the import.
    * ``thread``: before the import starts (overlaps the whole import, including the dlopen of
      libtorch_hip whose constructors register fat binaries while hipInit runs on the side thread —
      kept only for the A/B in profiles/r4_coldstart).
    * ``0``: off; torch initialises HIP on first use.

    Returns {"mode", "thread"} (thread may still be None while waiting for torch._C)."""
    mode = os.environ.get("KFAMD_HIP_PREINIT", "after-c")
    if mode in ("0", "off", ""):
        return None
    lib = _hip_lib()
    if lib is None:
        return None
    st: dict = {"mode": mode, "thread": None}

    def start():
        PREINIT["start_ms"] = round((time.perf_counter() - _T_WARMUP[0]) * 1e3, 1)
        th = threading.Thread(target=_hip_preinit_run, args=(lib,), name="hip-preinit", daemon=True)
        st["thread"] = th
        th.start()

    if mode == "thread" or "torch._C" in sys.modules:
        start()
    else:
        st["hook"] = _AfterTorchC(start)
        sys.meta_path.insert(0, st["hook"])
    return st


_T_WARMUP = [time.perf_counter()]


def warmup_torch() -> dict:
    """import torch + the framework's kernels and run one GEMM on cuda:0 (the pod's first GPU).

    While it runs, ``faulthandler`` dumps every thread's Python stack to the container log every
    KFAMD_WARMUP_TRACE_S seconds (default 5; 0 disables), so a slow or stuck warmup leaves the
    evidence of where it is in the pod log the cold-start bench collects on failure."""
    import faulthandler
    trace_s = float(os.environ.get("KFAMD_WARMUP_TRACE_S", "5") or 0)
    if trace_s > 0:
        faulthandler.dump_traceback_later(trace_s, repeat=True, file=sys.stderr)
    try:
        return _warmup_torch()
    finally:
        if trace_s > 0:
            faulthandler.cancel_dump_traceback_later()


def _warmup_torch() -> dict:
    t0 = _T_WARMUP[0] = time.perf_counter()
    pre = _preinit_hip()
    import torch
    t1 = time.perf_counter()
    if pre is not None and pre.get("hook") is not None and not pre["hook"].fired:
        try:  # torch._C came from somewhere the hook did not see (already imported): start now
            sys.meta_path.remove(pre["hook"])
        except ValueError:
            pass
        pre["hook"]._fire()
    if pre is not None and pre["thread"] is not None:
        pre["thread"].join(timeout=30)
        if pre["thread"].is_alive():
            PREINIT["joined"] = False  # reported; torch goes on and initialises HIP itself
    t_join = time.perf_counter()
    from kubeflow_rm_amd import ops
    t2 = time.perf_counter()
    dev = torch.device("cuda", 0)
    # operands made on the host and copied in (DMA), the GEMM on the framework's MFMA kernel on torch's
    # stream and caching allocator, the result copied back and spot-checked on the host: proves torch's
    # GPU runtime and the pod's GPU work without launching (and so code-object loading) any of torch's
    # own kernels before Ready — the first of those costs ~100 ms and lands in the user's first cell
    g = torch.Generator().manual_seed(0)
    ha = (torch.rand(1024, 1024, generator=g) * 2 - 1).to(torch.bfloat16)
    hb = (torch.rand(1024, 1024, generator=g) * 2 - 1).to(torch.bfloat16)
    c = ops.gemm_nt(ha.to(dev), hb.to(dev))
    hc = c.cpu()
    t3 = time.perf_counter()
    # spot check: 3 rows x 16 columns against fp32 on the host. Small tensors (below the CPU kernels'
    # parallel grain, so no OpenMP pool start) and index_select only:
    # the full 3 x 1024 reference (a parallel 1M-element convert) and list indexing (the advanced-
    # indexing path's first call) each cost 60-150 ms of CPU on the cold-start critical path
    rows = torch.tensor([0, 511, 1023])
    ref = ha.index_select(0, rows).float() @ hb[::64].float().t()
    got = hc.index_select(0, rows)[:, ::64].float()
    err = (got - ref).abs().max().item()
    ok = bool(torch.isfinite(got).all().item()) and err <= 1e-2 * ref.abs().max().item() + 1e-2
    t4 = time.perf_counter()
    return {"ok": ok, "check_ms": round((t4 - t3) * 1e3, 1), "import_torch_ms": round((t1 - t0) * 1e3, 1), "import_ops_ms": round((t2 - t1) * 1e3, 1),
            "first_gemm_ms": round((t3 - t2) * 1e3, 1), "total_ms": round((t3 - t0) * 1e3, 1), "hip_preinit": (pre or {}).get("mode"), "preinit_join_ms": round((t_join - t1) * 1e3, 1),
            "preinit_ms": dict(PREINIT),
            "max_abs_err": err}


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


_WS_GUID = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11"


def _ws_read_frame(rfile):
    """One client frame -> (opcode, payload); None on EOF. Client frames are masked (RFC 6455 5.3)."""
    h = rfile.read(2)
    if len(h) < 2:
        return None
    op, n = h[0] & 0x0F, h[1] & 0x7F
    if n == 126:
        n = struct.unpack(">H", rfile.read(2))[0]
    elif n == 127:
        n = struct.unpack(">Q", rfile.read(8))[0]
    mask = rfile.read(4) if h[1] & 0x80 else b"\0\0\0\0"
    data = bytearray(rfile.read(n))
    for i in range(len(data)):
        data[i] ^= mask[i & 3]
    return op, bytes(data)


def _ws_frame(payload: bytes, op: int = 1) -> bytes:
    n = len(payload)
    if n < 126:
        head = struct.pack(">BB", 0x80 | op, n)
    elif n < 1 << 16:
        head = struct.pack(">BBH", 0x80 | op, 126, n)
    else:
        head = struct.pack(">BBQ", 0x80 | op, 127, n)
    return head + payload


def _jmsg(parent: dict, msg_type: str, channel: str, content: dict) -> dict:
    return {"header": {"msg_id": str(uuid.uuid4()), "msg_type": msg_type, "session": parent.get("header", {}).get("session", ""),
                       "username": "kflite", "date": _now(), "version": "5.3"},
            "parent_header": parent.get("header", {}), "metadata": {}, "content": content, "channel": channel}


def _kernel_replies(k: dict, msg: dict) -> list[dict]:
    mt = msg.get("header", {}).get("msg_type", "")
    if mt == "kernel_info_request":
        return [_jmsg(msg, "kernel_info_reply", "shell",
                      {"status": "ok", "protocol_version": "5.3", "implementation": "kfamd-kflite",
                       "language_info": {"name": "python", "version": sys.version.split()[0]}})]
    if mt == "execute_request":
        k["execution_count"] = k.get("execution_count", 0) + 1
        k["last_activity"] = _now()
        code = msg.get("content", {}).get("code", "")
        return [_jmsg(msg, "status", "iopub", {"execution_state": "busy"}),
                _jmsg(msg, "execute_input", "iopub", {"code": code, "execution_count": k["execution_count"]}),
                _jmsg(msg, "stream", "iopub", {"name": "stdout", "text": code}),
                _jmsg(msg, "execute_reply", "shell", {"status": "ok", "execution_count": k["execution_count"]}),
                _jmsg(msg, "status", "iopub", {"execution_state": "idle"})]
    return [_jmsg(msg, mt.replace("_request", "_reply") if mt.endswith("_request") else "error", "shell",
                  {"status": "error", "ename": "NotImplemented", "evalue": mt})]


def make_handler(prefix: str):
    prefix = prefix.rstrip("/")

    class H(JsonHandler):
        def _route(self):
            path = self.path.split("?", 1)[0]
            if prefix and path.startswith(prefix):
                path = path[len(prefix):] or "/"
            return path

        def _kernel_channels(self, kid: str):
            with _LOCK:
                k = KERNELS.get(kid)
            if not k:
                return self.send_json(404, {"message": "kernel not found"})
            key = self.headers.get("Sec-WebSocket-Key", "")
            if self.headers.get("Upgrade", "").lower() != "websocket" or not key:
                return self.send_json(400, {"message": "expected a WebSocket upgrade"})
            accept = base64.b64encode(hashlib.sha1((key + _WS_GUID).encode()).digest()).decode()
            self.send_response(101, "Switching Protocols")
            self.send_header("Upgrade", "websocket")
            self.send_header("Connection", "Upgrade")
            self.send_header("Sec-WebSocket-Accept", accept)
            self.end_headers()
            self.wfile.flush()
            self.close_connection = True
            with _LOCK:
                k["connections"] = k.get("connections", 0) + 1
            try:
                while True:
                    fr = _ws_read_frame(self.rfile)
                    if fr is None or fr[0] == 8:  # EOF / close
                        if fr is not None:
                            self.wfile.write(_ws_frame(b"", 8))
                        return
                    op, data = fr
                    if op == 9:  # ping -> pong
                        self.wfile.write(_ws_frame(data, 10))
                        continue
                    if op != 1:
                        continue
                    try:
                        msg = json.loads(data)
                    except ValueError:
                        continue
                    with _LOCK:
                        replies = _kernel_replies(k, msg)
                    for r in replies:
                        self.wfile.write(_ws_frame(json.dumps(r).encode()))
                    self.wfile.flush()
            except OSError:
                return
            finally:
                with _LOCK:
                    k["connections"] = max(0, k.get("connections", 1) - 1)

        def _event_stream(self):
            q = dict(pair.split("=", 1) for pair in (self.path.split("?", 1)[1:] or [""])[0].split("&") if "=" in pair)
            n, interval = int(q.get("n", "5")), float(q.get("interval_ms", "100")) / 1000.0
            self.send_response(200)
            self.send_header("Content-Type", "text/event-stream")
            self.send_header("Cache-Control", "no-cache")
            self.send_header("Transfer-Encoding", "chunked")
            self.end_headers()
            for i in range(n):
                ev = f"id: {i}\ndata: {json.dumps({'seq': i, 't': time.time()})}\n\n".encode()
                self.wfile.write(b"%x\r\n%s\r\n" % (len(ev), ev))
                self.wfile.flush()
                time.sleep(interval)
            self.wfile.write(b"0\r\n\r\n")
            self.close_connection = True

        def do_GET(self):
            p = self._route()
            parts = p.strip("/").split("/")
            if len(parts) == 4 and parts[:2] == ["api", "kernels"] and parts[3] == "channels":
                return self._kernel_channels(parts[2])
            if p == "/api/events/stream":
                return self._event_stream()
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
                if WARMUP and "device" not in WARMUP:
                    # looked up on the first request, not before Ready: torch's device-properties
                    # query cost ~100 ms of the cold start
                    import torch
                    WARMUP["device"] = torch.cuda.get_device_name(0)
                info = {"HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES"),
                        "ring": os.environ.get("KFAMD_XGMI_RING"),
                        "topology": os.environ.get("KFAMD_GPU_TOPOLOGY"), "warmup": WARMUP or None,
                        "KFAMD_CPU_AFFINITY": os.environ.get("KFAMD_CPU_AFFINITY"),
                        "cpus_allowed": sorted(os.sched_getaffinity(0))}
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
    t_main = time.time()
    if os.environ.get("KFAMD_WARMUP") == "torch":
        WARMUP.update(warmup_torch())
        print(f"[kflite-notebook] warmup {json.dumps(WARMUP)}", flush=True)
    srv = serve(make_handler(prefix), port)
    if WARMUP:  # wall-clock stamps for the cold-start breakdown (bench_coldstart)
        WARMUP["main_ts"] = t_main
        WARMUP["listen_ts"] = time.time()
    print(f"[kflite-notebook] serving {prefix or '/'} on {srv.server_address[0]}:{port} home={os.environ.get('HOME')}",
          flush=True)
    run_forever([srv])
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
