"""Softmax cross-entropy on bf16 logits (kernels/xent_bf16.hip): no fp32 copy of the logits.

The forward stores one fp32 log-sum-exp per row; the backward re-reads the logits once and writes
``(softmax - onehot) * g / count`` with the upstream gradient and the counted-row total read on the
device (no host sync). Matches ``F.cross_entropy(logits.float(), target, ignore_index=...)`` with
the mean reduction.
"""
from __future__ import annotations

import torch

from . import _lib
from .gemm import _check_operand, _stream_ptr


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        V = logits.shape[-1]
        x2 = logits.reshape(-1, V)
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        rows = x2.shape[0]
        t = target.reshape(-1).to(torch.int64).contiguous()
        if t.numel() != rows:
            raise ValueError(f"target has {t.numel()} entries for {rows} rows")
        loss_rows = torch.empty(rows, dtype=torch.float32, device=logits.device)
        lse = torch.empty_like(loss_rows)
        rc = _lib.lib().kfamd_xent_fwd_bf16(x2.data_ptr(), x2.stride(0), t.data_ptr(), loss_rows.data_ptr(),
                                           lse.data_ptr(), rows, V, int(ignore_index), _stream_ptr(logits))
        _lib.check(rc, f"xent_fwd[{rows}x{V}]")
        count = ((t != ignore_index) & (t >= 0) & (t < V)).sum().to(torch.float32).reshape(1)
        ctx.save_for_backward(x2, t, lse, count)
        ctx.ignore_index = int(ignore_index)
        ctx.shape = logits.shape
        return loss_rows.sum() / count[0]

    @staticmethod
    def backward(ctx, g):
        x2, t, lse, count = ctx.saved_tensors
        rows, V = x2.shape
        grad = torch.empty_like(x2)
        g32 = g.detach().to(torch.float32).reshape(1).contiguous()
        rc = _lib.lib().kfamd_xent_bwd_bf16(x2.data_ptr(), x2.stride(0), t.data_ptr(), lse.data_ptr(),
                                           grad.data_ptr(), grad.stride(0), rows, V, ctx.ignore_index,
                                           g32.data_ptr(), count.data_ptr(), _stream_ptr(x2))
        _lib.check(rc, f"xent_bwd[{rows}x{V}]")
        return grad.view(ctx.shape), None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean softmax cross-entropy over the last dim of bf16 ``logits`` (autograd-aware)."""
    _check_operand(logits, "logits")
    return _CrossEntropy.apply(logits, target, ignore_index)
