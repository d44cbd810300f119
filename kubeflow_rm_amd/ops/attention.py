"""Attention-side glue around torch's scaled_dot_product_attention.

``split_heads(qkv, h, hd)`` turns the fused QKV projection output ``[B, T, 3 * h * hd]`` into the
``[B, h, T, hd]`` q / k / v views SDPA takes, exactly as ``qkv.view(B, T, 3, h, hd).permute(2, 0, 3, 1,
4)`` does. Its backward writes SDPA's dq / dk / dv straight into the QKV gradient layout with one
HIP pass (``kernels/qkv_pack_bf16.hip``). Autograd's route for the view/permute stacks the three and
then copies the stack into place: 204 us per gpt-1b layer, against one read and one write here
(``profiles/r4_train_trace``).
"""
from __future__ import annotations

import torch

from . import _lib


def _stream_ptr(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


class _SplitHeads(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, h, hd):
        B, T, _ = qkv.shape
        ctx.dims = (B, T, h, hd)
        q, k, v = qkv.view(B, T, 3, h, hd).permute(2, 0, 3, 1, 4)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        B, T, h, hd = ctx.dims
        ref = next(g for g in (dq, dk, dv) if g is not None)
        out = torch.empty(B, T, 3 * h * hd, dtype=ref.dtype, device=ref.device)
        grads = [g if g is None or g.stride(-1) == 1 else g.contiguous() for g in (dq, dk, dv)]
        strides = []
        for g in grads:
            strides += list(g.stride()[:3]) if g is not None else [0, 0, 0]
        rc = _lib.lib().kfamd_qkv_pack_bf16(*(g.data_ptr() if g is not None else None for g in grads), out.data_ptr(),
                                           B, T, h, hd, *strides, _stream_ptr(ref))
        if rc != 0:  # off the kernel's alignment contract: autograd's own layout change
            z = [g if g is not None else torch.zeros(B, h, T, hd, dtype=ref.dtype, device=ref.device) for g in grads]
            out.view(B, T, 3, h, hd).copy_(torch.stack(z, 0).permute(1, 3, 0, 2, 4))
        return out, None, None


def split_heads(qkv: torch.Tensor, h: int, hd: int):
    """q, k, v ``[B, h, T, hd]`` views of the fused QKV output ``[B, T, 3 * h * hd]``."""
    from . import native_enabled
    if (native_enabled() and qkv.is_cuda and qkv.dtype == torch.bfloat16 and hd % 8 == 0
            and qkv.is_contiguous() and torch.is_grad_enabled() and qkv.requires_grad):
        return _SplitHeads.apply(qkv, h, hd)
    B, T, _ = qkv.shape
    q, k, v = qkv.view(B, T, 3, h, hd).permute(2, 0, 3, 1, 4)
    return q, k, v
