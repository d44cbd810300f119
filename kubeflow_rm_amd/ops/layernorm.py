"""LayerNorm / RMSNorm on the hand-written gfx950 kernels (kernels/layernorm_bf16.hip)."""
from __future__ import annotations

import torch

from . import _lib
from .gemm import _check_operand, _stream_ptr


def layer_norm_fwd(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None, eps: float = 1e-5,
                   save_stats: bool = False):
    _check_operand(x, "x")
    _check_operand(weight, "weight")
    H = x.shape[-1]
    x2 = x.reshape(-1, H).contiguous()
    rows = x2.shape[0]
    y = torch.empty_like(x2)
    mean = rstd = None
    if save_stats:
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    rc = _lib.lib().kfamd_layernorm_fwd_bf16(
        x2.data_ptr(), weight.contiguous().data_ptr(),
        bias.contiguous().data_ptr() if bias is not None else None, y.data_ptr(),
        mean.data_ptr() if mean is not None else None, rstd.data_ptr() if rstd is not None else None,
        rows, H, float(eps), _stream_ptr(x))
    _lib.check(rc, f"layernorm_fwd[{rows}x{H}]")
    return y.view(x.shape), mean, rstd


def rms_norm_fwd(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-6, save_stats: bool = False):
    _check_operand(x, "x")
    H = x.shape[-1]
    x2 = x.reshape(-1, H).contiguous()
    y = torch.empty_like(x2)
    rstd = torch.empty(x2.shape[0], dtype=torch.float32, device=x.device) if save_stats else None
    rc = _lib.lib().kfamd_rmsnorm_fwd_bf16(x2.data_ptr(), weight.contiguous().data_ptr(), y.data_ptr(),
                                           rstd.data_ptr() if rstd is not None else None, x2.shape[0], H,
                                           float(eps), _stream_ptr(x))
    _lib.check(rc, f"rmsnorm_fwd[{x2.shape[0]}x{H}]")
    return y.view(x.shape), rstd


class _RMSNorm(torch.autograd.Function):
    """Forward on the HIP kernel (fp32 rstd saved); backward from the saved rstd:
    dx = rstd * (w*dy - xhat * mean(w*dy*xhat)), dw = sum(dy * xhat), xhat = x * rstd."""

    @staticmethod
    def forward(ctx, x, weight, eps):
        y, rstd = rms_norm_fwd(x, weight, eps, save_stats=True)
        ctx.save_for_backward(x, weight, rstd)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, rstd = ctx.saved_tensors
        H = x.shape[-1]
        xf = x.reshape(-1, H).float()
        r = rstd.unsqueeze(-1)
        xhat = xf * r
        gyf = gy.reshape(-1, H).float()
        gdy = gyf * weight.float()
        dx = r * (gdy - xhat * (gdy * xhat).mean(-1, keepdim=True))
        dw = (gyf * xhat).sum(0)
        return dx.to(x.dtype).view(x.shape), dw.to(weight.dtype), None


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    """Autograd-aware RMSNorm over the last dim (bf16 I/O, fp32 statistics)."""
    return _RMSNorm.apply(x, weight, eps)


def _ln_backward(ctx, gy, gres=None):
    x, weight, mean, rstd = ctx.saved_tensors
    H = x.shape[-1]
    x2 = x.reshape(-1, H).contiguous()
    rows = x2.shape[0]
    if gy is None:  # only the residual output was used
        return gres, None, None, None
    gy2 = gy.reshape(-1, H).contiguous().to(torch.bfloat16)
    res = gres.reshape(-1, H).contiguous().to(torch.bfloat16) if gres is not None else None
    dx = torch.empty_like(x2)
    pbf16 = weight.dtype == torch.bfloat16
    gdt = torch.bfloat16 if pbf16 else torch.float32
    dgamma = torch.empty(H, dtype=gdt, device=x.device)
    dbeta = torch.empty(H, dtype=gdt, device=x.device)
    ws_bytes = _lib.lib().kfamd_layernorm_bwd_workspace(rows, H)
    ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=x.device)
    rc = _lib.lib().kfamd_layernorm_bwd_bf16_v3(
        gy2.data_ptr(), res.data_ptr() if res is not None else None, x2.data_ptr(), weight.contiguous().data_ptr(),
        mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), int(pbf16),
        ws.data_ptr(), rows, H, _stream_ptr(x))
    _lib.check(rc, f"layernorm_bwd[{rows}x{H}]")
    return (dx.view(x.shape), dgamma.to(weight.dtype), dbeta.to(weight.dtype) if ctx.has_bias else None, None)


class _LayerNormResidual(torch.autograd.Function):
    """(LayerNorm(x), x): the second output is the pre-norm block's residual stream. Both outputs'
    gradients come back to this one node, and the backward kernel sums them in its dx store
    (kfamd_layernorm_bwd_bf16_v3 dres) — autograd would otherwise add the two with a separate
    elementwise kernel per norm (2 x 17 us per gpt-1b layer, profiles/r4_train_trace)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        y, mean, rstd = layer_norm_fwd(x, weight, bias, eps, save_stats=True)
        ctx.save_for_backward(x, weight, mean, rstd)
        ctx.has_bias = bias is not None
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gres):
        return _ln_backward(ctx, gy, gres)


def layer_norm_residual(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
                        eps: float = 1e-5):
    """``(layer_norm(x), r)`` where ``r`` is ``x`` for the residual add: use ``r`` (not ``x``) as the
    residual and the two gradient contributions to ``x`` are summed inside the LayerNorm backward."""
    return _LayerNormResidual.apply(x, weight, bias, eps)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        y, mean, rstd = layer_norm_fwd(x, weight, bias, eps, save_stats=True)
        ctx.save_for_backward(x, weight, mean, rstd)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, mean, rstd = ctx.saved_tensors
        H = x.shape[-1]
        x2 = x.reshape(-1, H).contiguous()
        gy2 = gy.reshape(-1, H).contiguous().to(torch.bfloat16)
        rows = x2.shape[0]
        dx = torch.empty_like(x2)
        # the parameter grads in the parameter dtype straight from the kernel (fp32 sums either way)
        pbf16 = weight.dtype == torch.bfloat16
        gdt = torch.bfloat16 if pbf16 else torch.float32
        dgamma = torch.empty(H, dtype=gdt, device=x.device)
        dbeta = torch.empty(H, dtype=gdt, device=x.device)
        ws_bytes = _lib.lib().kfamd_layernorm_bwd_workspace(rows, H)
        ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=x.device)
        rc = _lib.lib().kfamd_layernorm_bwd_bf16_v2(
            gy2.data_ptr(), x2.data_ptr(), weight.contiguous().data_ptr(), mean.data_ptr(),
            rstd.data_ptr(), dx.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), int(pbf16), ws.data_ptr(),
            rows, H, _stream_ptr(x))
        _lib.check(rc, f"layernorm_bwd[{rows}x{H}]")
        return (dx.view(x.shape), dgamma.to(weight.dtype),
                dbeta.to(weight.dtype) if ctx.has_bias else None, None)


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
               eps: float = 1e-5) -> torch.Tensor:
    """Autograd-aware LayerNorm over the last dim (bf16 I/O, fp32 statistics)."""
    return _LayerNorm.apply(x, weight, bias, eps)
