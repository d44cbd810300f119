"""Loader for the in-tree gfx950 kernel library (``kubeflow_rm_amd/lib/libkfamd_kernels.so``).

The library is loaded with ctypes *after* torch so that both share one HIP runtime (the
``libamdhip64.so.7`` SONAME torch already mapped). There is no silent fallback: on a machine
with a GPU, a missing or unloadable library raises :class:`NativeLibraryError`.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent.parent / "lib" / "libkfamd_kernels.so"

_lock = threading.Lock()
_lib: ctypes.CDLL | None = None

c_ll = ctypes.c_longlong
c_vp = ctypes.c_void_p
c_int = ctypes.c_int
c_float = ctypes.c_float

_SIGNATURES = {
    "kfamd_gemm_nt_bf16": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                   c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_float, c_int, c_vp]),
    "kfamd_gemm_nt_bf16_variant": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int,
                                           c_int, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll,
                                           c_float, c_int, c_vp]),
    "kfamd_gemm_bf16_ex": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                   c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_float, c_int, c_vp]),
    "kfamd_w4_splitk_nt": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_ll, c_ll,
                                   c_ll, c_ll, c_vp]),
    "kfamd_w4_splitk_t": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_ll,
                                  c_ll, c_ll, c_ll, c_vp]),
    "kfamd_w4_splitk_fix": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_ll, c_ll,
                                    c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_float, c_vp, c_vp, c_int, c_int, c_vp]),
    "kfamd_w4_streamk_nt": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_ll, c_ll, c_ll, c_ll,
                                    c_float, c_int, c_vp, c_vp, ctypes.c_uint, c_int, c_int, c_vp]),
    "kfamd_splitk_reduce": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_ll, c_ll, c_ll,
                                    c_ll, c_float, c_int, c_vp]),
    "kfamd_pad_k_bf16": (c_int, [c_vp, c_vp, c_ll, c_ll, c_vp, c_vp, c_ll, c_ll, c_int, c_int, c_vp]),
    "kfamd_act_grad_workspace": (c_ll, [c_int, c_int]),
    "kfamd_adamw_tensor_bytes": (c_int, []),
    "kfamd_adamw_chunk": (c_int, []),
    "kfamd_adamw_bf16": (c_int, [c_vp, c_vp, c_ll, c_float, c_float, c_float, c_float, c_float, c_float, c_float,
                                 c_vp]),
    "kfamd_qkv_pack_bf16": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_ll, c_ll, c_ll, c_ll, c_ll,
                                    c_ll, c_ll, c_ll, c_ll, c_vp]),
    "kfamd_act_fwd_bf16": (c_int, [c_vp, c_vp, c_ll, c_int, c_vp]),
    "kfamd_xent_fwd_bf16": (c_int, [c_vp, c_ll, c_vp, c_vp, c_vp, c_int, c_int, c_ll, c_vp]),
    "kfamd_xent_bwd_bf16": (c_int, [c_vp, c_ll, c_vp, c_vp, c_vp, c_ll, c_int, c_int, c_ll, c_vp, c_vp, c_vp]),
    "kfamd_act_grad_bf16": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    "kfamd_act_grad_bf16_v2": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_vp]),
    "kfamd_colsum_finalize": (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    "kfamd_w4_dgrad_act_workspace": (c_ll, [c_int, c_int]),
    "kfamd_w4_wgrad_pair": (c_int, [c_vp, c_vp, c_vp, c_int, c_ll, c_ll, c_ll, c_vp, c_vp, c_vp, c_int, c_ll, c_ll,
                                    c_ll, c_int, c_int, c_vp]),
    "kfamd_w4_wgrad_pair_v2": (c_int, [c_vp, c_vp, c_vp, c_int, c_ll, c_ll, c_ll, c_vp, c_vp, c_vp, c_int, c_ll,
                                       c_ll, c_ll, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "kfamd_w4_dgrad_act": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_ll, c_ll, c_ll, c_ll, c_int, c_vp,
                                   c_vp, c_int, c_vp]),
    "kfamd_layernorm_fwd_bf16": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_float, c_vp]),
    "kfamd_rmsnorm_fwd_bf16": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_float, c_vp]),
    "kfamd_layernorm_bwd_workspace": (c_ll, [c_int, c_int]),
    "kfamd_layernorm_bwd_bf16": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                         c_int, c_int, c_vp]),
    "kfamd_layernorm_bwd_bf16_v2": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int,
                                            c_int, c_vp]),
    "kfamd_layernorm_bwd_bf16_v3": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp,
                                            c_int, c_int, c_vp]),
    "kfamd_allreduce_oneshot_flag_bytes": (c_ll, [c_int, c_int]),
    "kfamd_allreduce_oneshot_blocks": (c_int, [c_ll, c_int]),
    "kfamd_allreduce_oneshot_set_timeout_ms": (None, [c_int]),
    "kfamd_allreduce_oneshot": (c_int, [ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_int, c_int,
                                        c_int, c_ll, c_int, ctypes.c_uint, c_int, c_vp, c_vp]),
    "kfamd_allreduce_twoshot_blocks": (c_int, [c_ll, c_int, c_int]),
    "kfamd_allreduce_twoshot": (c_int, [ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_int, c_int,
                                        c_int, c_ll, c_int, ctypes.c_uint, c_int, c_vp, c_vp]),
    "kfamd_ipc_alloc": (c_int, [c_ll, c_int, ctypes.POINTER(c_vp), ctypes.c_char_p]),
    "kfamd_ipc_open": (c_int, [ctypes.c_char_p, ctypes.POINTER(c_vp)]),
    "kfamd_ipc_close": (c_int, [c_vp]),
    "kfamd_ipc_free": (c_int, [c_vp]),
    "kfamd_copy_async": (c_int, [c_vp, c_vp, c_ll, c_vp]),
    "kfamd_attn_fwd_bf16": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_float, c_int,
                                    ctypes.POINTER(c_ll), c_vp]),
    "kfamd_attn_bwd_workspace": (c_ll, [c_int, c_int, c_int, c_int]),
    "kfamd_attn_bwd_bf16": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int,
                                    c_int, c_float, c_int, ctypes.POINTER(c_ll), c_vp]),
    "kfamd_build_info": (ctypes.c_char_p, []),
}

STATUS = {0: "ok", -1: "invalid argument / shape contract", -2: "alignment contract"}


class NativeLibraryError(RuntimeError):
    """The HIP kernel library is missing, failed to load, or a launch returned an error."""


def lib() -> ctypes.CDLL:
    """Return the loaded kernel library, loading it on first use (raises if unavailable)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  -- map torch's HIP runtime first (shared SONAME)

        path = Path(os.environ.get("KFAMD_KERNEL_LIB", str(LIB_PATH)))
        if not path.exists():
            raise NativeLibraryError(
                f"{path} not found: build it with `python -m kubeflow_rm_amd._build kernels` "
                "(or __graft_entry__.build())")
        try:
            handle = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the machine
            raise NativeLibraryError(f"failed to load {path}: {e}") from e
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def available() -> bool:
    try:
        lib()
        return True
    except NativeLibraryError:
        return False


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = STATUS.get(rc, f"hipError_t {rc}")
        raise NativeLibraryError(f"{what} failed: {msg}")


def build_info() -> str:
    return lib().kfamd_build_info().decode()
