"""Torch-facing wrappers of the hand-written gfx950 kernels (no silent eager fallback)."""
from ._lib import NativeLibraryError, available, build_info, lib  # noqa: F401
from .gemm import act_grad, dgrad_act, flops, gemm_nt, gemm_nt_preact, linear, matmul, mlp, mm, wgrad_pair  # noqa: F401
from .layernorm import layer_norm, layer_norm_fwd, layer_norm_residual, rms_norm, rms_norm_fwd  # noqa: F401
from .xent import cross_entropy  # noqa: F401
from .attention import attention_qkv, attn_block, flash_attention, split_heads  # noqa: F401
from .attention import supported as attention_supported  # noqa: F401
from .allreduce import OneShotAllReduce  # noqa: F401
from .graph import GraphedCallable  # noqa: F401


# A/B switch for the model layers (kubeflow_rm_amd.models / parallel.tp): inside torch_reference()
# GPU tensors run torch's F.linear / F.layer_norm instead of these kernels. Benchmarks use it to
# compare the two on the same model; nothing in the framework switches it on by itself.
import contextlib as _contextlib

_native = True


def native_enabled() -> bool:
    return _native


@_contextlib.contextmanager
def torch_reference():
    global _native
    prev, _native = _native, False
    try:
        yield
    finally:
        _native = prev
