"""ctypes binding of ``libkfcore_capi.so`` — the control plane's pure C++ helpers.

``call("generate_statefulset", notebook=nb)`` runs the same code the native reconcilers run
(see native/capi/capi.cc for the function table). Used by the unit tests (the reference's
table-driven Go tests, ported) and by the web apps.
"""
from __future__ import annotations

import ctypes
import json
import threading
from pathlib import Path

_LIB_PATH = Path(__file__).resolve().parent / "lib" / "libkfcore_capi.so"
_lib = None
_lock = threading.Lock()


class NativeCallError(RuntimeError):
    pass


def _load():
    global _lib
    with _lock:
        if _lib is None:
            if not _LIB_PATH.exists():
                raise FileNotFoundError(f"{_LIB_PATH} missing: build with `python -m kubeflow_rm_amd._build native`")
            lib = ctypes.CDLL(str(_LIB_PATH))
            lib.kf_call.restype = ctypes.c_void_p
            lib.kf_call.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
            lib.kf_functions.restype = ctypes.c_void_p
            lib.kf_free.argtypes = [ctypes.c_void_p]
            _lib = lib
    return _lib


def _take(lib, ptr) -> str:
    try:
        return ctypes.string_at(ptr).decode()
    finally:
        lib.kf_free(ptr)


def call(fn: str, /, **args):
    lib = _load()
    out = json.loads(_take(lib, lib.kf_call(fn.encode(), json.dumps(args).encode())))
    if not out.get("ok"):
        raise NativeCallError(out.get("error", "unknown error"))
    return out.get("result")


def functions() -> list[str]:
    lib = _load()
    return json.loads(_take(lib, lib.kf_functions()))
