#!/usr/bin/env python3
"""Where the HIP init of a torch-ready container goes (profiles/r3d_zygote).

Times hipInit / device context / first op through torch's own libamdhip64 (ctypes, no torch GPU
call) in fresh child processes, four ways:
  bare     the library alone (nothing else loaded)
  torch    after `import torch` (torch's fat binaries registered with the runtime)
  forked   in a child forked from a parent that imported torch (the zygote case)
  forked_env  the same with HIP_ENABLE_DEFERRED_LOADING=1 / AMD_LOG_LEVEL=0 set explicitly
Each variant runs in its own process (never after a GPU init in the same process). One JSON line
per run.
"""
from __future__ import annotations

import ctypes
import importlib.util
import json
import os
import subprocess
import sys
import time


def _lib() -> str:
    spec = importlib.util.find_spec("torch")
    for d in spec.submodule_search_locations or []:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            return p
    raise SystemExit("no torch libamdhip64")


def _time_init() -> dict:
    out = {}
    t = time.perf_counter()
    hip = ctypes.CDLL(_lib(), mode=ctypes.RTLD_GLOBAL)
    out["dlopen_ms"] = round((time.perf_counter() - t) * 1e3, 1)
    t = time.perf_counter()
    rc = hip.hipInit(0)
    out["hipInit_ms"] = round((time.perf_counter() - t) * 1e3, 1)
    t = time.perf_counter()
    hip.hipSetDevice(0)
    hip.hipFree(None)
    out["context_ms"] = round((time.perf_counter() - t) * 1e3, 1)
    t = time.perf_counter()
    buf = ctypes.c_void_p()
    hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(4096))
    hip.hipMemset(buf, 0, ctypes.c_size_t(4096))
    hip.hipDeviceSynchronize()
    out["first_op_ms"] = round((time.perf_counter() - t) * 1e3, 1)
    out["rc"] = rc
    return out


def _time_steps() -> dict:
    """First-use cost of each kind of first GPU operation, in order, after init + context."""
    out = {}
    hip = ctypes.CDLL(_lib(), mode=ctypes.RTLD_GLOBAL)
    t = time.perf_counter()

    def lap(name):
        nonlocal t
        hip.hipDeviceSynchronize()
        now = time.perf_counter()
        out[name] = round((now - t) * 1e3, 1)
        t = now
    hip.hipInit(0)
    hip.hipSetDevice(0)
    hip.hipFree(None)
    lap("init_context_ms")
    s = ctypes.c_void_p()
    hip.hipStreamCreate(ctypes.byref(s))
    lap("stream_create_ms")
    buf = ctypes.c_void_p()
    hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(1 << 20))
    lap("malloc_ms")
    host = ctypes.create_string_buffer(1 << 20)
    hip.hipMemcpy(buf, host, ctypes.c_size_t(1 << 20), 1)  # H2D
    lap("memcpy_h2d_ms")
    hip.hipMemcpy(host, buf, ctypes.c_size_t(1 << 20), 2)  # D2H
    lap("memcpy_d2h_ms")
    hip.hipMemsetAsync(buf, 0, ctypes.c_size_t(4096), s)
    lap("memset_ms")
    hip.hipMemsetAsync(buf, 1, ctypes.c_size_t(4096), s)
    lap("memset2_ms")
    return out


def child(mode: str) -> None:
    if mode == "steps":
        print(json.dumps({"mode": mode, "comgr_cache": os.environ.get("AMD_COMGR_CACHE_DIR"), **_time_steps()}), flush=True)
        return
    if mode in ("torch", "forked", "forked_env"):
        t = time.perf_counter()
        import torch  # noqa: F401
        imp = round((time.perf_counter() - t) * 1e3, 1)
    else:
        imp = 0.0
    if mode.startswith("forked"):
        if mode == "forked_env":
            os.environ["HIP_ENABLE_DEFERRED_LOADING"] = "1"
        r, w = os.pipe()
        pid = os.fork()
        if pid == 0:
            os.close(r)
            res = _time_init()
            os.write(w, json.dumps(res).encode())
            os._exit(0)
        os.close(w)
        data = b""
        while True:
            chunk = os.read(r, 65536)
            if not chunk:
                break
            data += chunk
        os.waitpid(pid, 0)
        res = json.loads(data)
    else:
        res = _time_init()
    res.update(mode=mode, import_torch_ms=imp)
    print(json.dumps(res), flush=True)


def main() -> int:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "--steps":
        import tempfile
        cache = tempfile.mkdtemp(prefix="comgr-")
        # env variants of the HIP runtime's first-queue path (after one warm-up run fills the cache)
        variants = [{}] + [dict([kv.split("=", 1)]) for kv in sys.argv[2:]]
        subprocess.run([sys.executable, __file__, "--child", "steps"], check=True, timeout=120,
                       env={**os.environ, "AMD_COMGR_CACHE_DIR": cache})
        for rep in range(3):
            for v in variants:
                time.sleep(0.3)
                print(json.dumps({"variant": v}), flush=True)
                subprocess.run([sys.executable, __file__, "--child", "steps"], check=True, timeout=120,
                               env={**os.environ, "AMD_COMGR_CACHE_DIR": cache, **v})
        return 0
    for rep in range(3):
        for mode in ("bare", "torch", "forked", "forked_env"):
            subprocess.run([sys.executable, __file__, "--child", mode], check=True, timeout=120)
            time.sleep(0.3)  # KFD teardown of the previous process
    return 0


if __name__ == "__main__":
    sys.exit(main())
