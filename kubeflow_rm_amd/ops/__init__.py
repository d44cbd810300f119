"""Torch-facing wrappers of the hand-written gfx950 kernels (no silent eager fallback)."""
from ._lib import NativeLibraryError, available, build_info, lib  # noqa: F401
from .gemm import act_grad, flops, gemm_nt, gemm_nt_preact, linear, matmul, mm  # noqa: F401
from .layernorm import layer_norm, layer_norm_fwd, rms_norm, rms_norm_fwd  # noqa: F401
from .allreduce import OneShotAllReduce  # noqa: F401
from .graph import GraphedCallable  # noqa: F401
