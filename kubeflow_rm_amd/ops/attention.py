"""Attention on the hand-written gfx950 flash kernels (``kernels/attention_bf16.hip``).

``attention_qkv(qkv, h, hd)`` is the model's path: the fused QKV projection output
``[B, T, 3 * h * hd]`` is read in place by the forward kernel, which writes the attention output
straight into ``[B, T, h * hd]`` (the output projection's input: no head transpose) plus the
per-row log-sum-exp; the backward kernels recompute P from the LSE and write dq / dk / dv straight
into the QKV gradient layout ``[B, T, 3 * h * hd]`` (no stack / permute / copy).

``flash_attention(q, k, v)`` takes ``[B, H, T, D]`` views with any strides (contiguous head dim) —
the form the numerics tests compare against fp32 ``F.scaled_dot_product_attention``.

``split_heads(qkv, h, hd)`` remains for torch's SDPA path (CPU, other head dims): its backward
packs SDPA's dq / dk / dv into the QKV gradient layout in one HIP pass (``qkv_pack_bf16.hip``).

There is no silent fallback on a GPU: a kernel that rejects its arguments raises.
"""
from __future__ import annotations

import math

import torch

from . import _lib

HEAD_DIMS = (64, 128)


def _stream_ptr(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def supported(qkv_or_q: torch.Tensor, head_dim: int) -> bool:
    """True when the flash kernels take this tensor (CUDA bf16, head dim 64 / 128)."""
    return qkv_or_q.is_cuda and qkv_or_q.dtype == torch.bfloat16 and head_dim in HEAD_DIMS


def _strides(*ts) -> "ctypes.Array":
    import ctypes
    vals = []
    for t in ts:
        vals += [int(t.stride(0)), int(t.stride(1)), int(t.stride(2))]
    return (ctypes.c_longlong * len(vals))(*vals)


def _check_views(*ts) -> None:
    for t in ts:
        if t.dtype != torch.bfloat16 or not t.is_cuda or t.dim() != 4 or t.stride(-1) != 1:
            raise ValueError("flash attention: bf16 CUDA [B, H, T, D] views with a contiguous head dim expected")


def _fwd(q, k, v, o, causal: bool, scale: float) -> torch.Tensor:
    """q, k, v, o: [B, H, T, D] views. Returns lse [B, H, T] (f32)."""
    B, H, T, D = q.shape
    lse = torch.empty(B, H, T, device=q.device, dtype=torch.float32)
    rc = _lib.lib().kfamd_attn_fwd_bf16(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                                        B, H, T, D, float(scale), int(causal), _strides(q, k, v, o), _stream_ptr(q))
    _lib.check(rc, f"attn_fwd[B={B} H={H} T={T} D={D}]")
    return lse


def _bwd(q, k, v, o, do, lse, dq, dk, dv, causal: bool, scale: float) -> None:
    B, H, T, D = q.shape
    L = _lib.lib()
    ws = torch.empty(L.kfamd_attn_bwd_workspace(B, H, T, D), device=q.device, dtype=torch.uint8)
    rc = L.kfamd_attn_bwd_bf16(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(),
                               dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), ws.data_ptr(), B, H, T, D, float(scale),
                               int(causal), _strides(q, k, v, o, do, dq, dk, dv), _stream_ptr(q))
    _lib.check(rc, f"attn_bwd[B={B} H={H} T={T} D={D}]")


def _bhtd(x: torch.Tensor) -> torch.Tensor:
    """[B, T, H, D] storage as a [B, H, T, D] view."""
    return x.permute(0, 2, 1, 3)


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        _check_views(q, k, v)
        B, H, T, D = q.shape
        o = _bhtd(torch.empty(B, T, H, D, device=q.device, dtype=q.dtype))
        lse = _fwd(q, k, v, o, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        B, H, T, D = q.shape
        if do.stride(-1) != 1 or any(s % 8 for s in do.stride()[:3]):
            do = do.contiguous()
        grads = [_bhtd(torch.empty(B, T, H, D, device=q.device, dtype=q.dtype)) for _ in range(3)]
        _bwd(q, k, v, o, do, lse, *grads, ctx.causal, ctx.scale)
        return grads[0], grads[1], grads[2], None, None


class _FlashAttnQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, h, hd, causal, scale):
        B, T, _ = qkv.shape
        x = qkv.view(B, T, 3, h, hd)
        q, k, v = (_bhtd(x[:, :, i]) for i in range(3))
        o = torch.empty(B, T, h, hd, device=qkv.device, dtype=qkv.dtype)
        lse = _fwd(q, k, v, _bhtd(o), causal, scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.dims, ctx.causal, ctx.scale = (h, hd), causal, scale
        return o.view(B, T, h * hd)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        h, hd = ctx.dims
        B, T, _ = qkv.shape
        do = do.contiguous().view(B, T, h, hd)
        x = qkv.view(B, T, 3, h, hd)
        dqkv = torch.empty(B, T, 3, h, hd, device=qkv.device, dtype=qkv.dtype)
        _bwd(*(_bhtd(x[:, :, i]) for i in range(3)), _bhtd(o), _bhtd(do), lse,
             *(_bhtd(dqkv[:, :, i]) for i in range(3)), ctx.causal, ctx.scale)
        return dqkv.view(B, T, 3 * h * hd), None, None, None, None


class _AttnBlock(torch.autograd.Function):
    """x -> qkv = x Wqkv^T + bqkv -> flash attention -> o Wproj^T + bproj (+ residual), one autograd
    node. Its backward orders the work across the three: the projection's dgrad, the attention
    backward, the QKV dgrad, and then both weight gradients in ONE launch (gemm.wgrad_pair: 192 + 64
    tiles at gpt-1b, where apart the QKV wgrad filled 75 % of the CUs and the projection's ran
    split-K). The forward is the separate layers' (gemm_nt with bias, _fwd, gemm_nt with bias and
    residual)."""

    @staticmethod
    def forward(ctx, x, wqkv, bqkv, wproj, bproj, h, hd, causal, scale, residual):
        from .gemm import gemm_nt
        B, T, D = x.shape
        x2 = x.reshape(B * T, D)
        if x2.stride(-1) != 1 or x2.stride(0) != D:
            x2 = x2.contiguous()
        qkv = gemm_nt(x2, wqkv, bias=bqkv).view(B, T, 3, h, hd)
        o = torch.empty(B, T, h, hd, device=x.device, dtype=x.dtype)
        lse = _fwd(*(_bhtd(qkv[:, :, i]) for i in range(3)), _bhtd(o), causal, scale)
        o2 = o.view(B * T, h * hd)
        res = residual.reshape(B * T, wproj.shape[0]).contiguous() if residual is not None else None
        out = gemm_nt(o2, wproj, bias=bproj, residual=res)
        ctx.save_for_backward(x2, wqkv, bqkv, wproj, bproj, qkv, o, lse)
        ctx.dims, ctx.causal, ctx.scale = (B, T, D, h, hd), causal, scale
        return out.view(B, T, wproj.shape[0])

    @staticmethod
    def backward(ctx, gy):
        from .gemm import act_grad, mm, wgrad_pair
        x2, wqkv, bqkv, wproj, bproj, qkv, o, lse = ctx.saved_tensors
        B, T, D, h, hd = ctx.dims
        ni = ctx.needs_input_grad
        gy2 = gy.reshape(B * T, wproj.shape[0])
        if not gy2.is_contiguous():
            gy2 = gy2.contiguous()

        def bias_grad(g, bias, need):
            if not need:
                return None
            _, db = act_grad(g, None, "none", True,
                             db_dtype=torch.bfloat16 if bias.dtype == torch.bfloat16 else torch.float32)
            return db.to(bias.dtype)
        gbp = bias_grad(gy2, bproj, bproj is not None and ni[4])
        o2 = o.view(B * T, h * hd)
        do = mm(gy2, wproj).view(B, T, h, hd)  # the projection's dgrad
        dqkv = torch.empty(B, T, 3, h, hd, device=qkv.device, dtype=qkv.dtype)
        _bwd(*(_bhtd(qkv[:, :, i]) for i in range(3)), _bhtd(o), _bhtd(do), lse,
             *(_bhtd(dqkv[:, :, i]) for i in range(3)), ctx.causal, ctx.scale)
        dqkv2 = dqkv.view(B * T, 3 * h * hd)
        gbq = bias_grad(dqkv2, bqkv, bqkv is not None and ni[2])
        dx = mm(dqkv2, wqkv).view(B, T, D) if ni[0] else None
        gwq = gwp = None
        pair = wgrad_pair(dqkv2, x2, gy2, o2) if ni[1] and ni[3] else None
        if pair is not None:
            gwq, gwp = pair
        else:
            gwq = mm(dqkv2, x2, trans_a=True) if ni[1] else None
            gwp = mm(gy2, o2, trans_a=True) if ni[3] else None
        return dx, gwq, gbq, gwp, gbp, None, None, None, None, (gy if ni[9] else None)


def attn_block(x: torch.Tensor, wqkv: torch.Tensor, bqkv: torch.Tensor | None, wproj: torch.Tensor,
               bproj: torch.Tensor | None, h: int, hd: int, residual: torch.Tensor | None = None,
               causal: bool = True, scale: float | None = None) -> torch.Tensor:
    """A transformer block's attention half on the HIP kernels: ``proj(attn(qkv(x))) (+ residual)``,
    x ``[B, T, D]``, wqkv ``[3 h hd, D]`` (q | k | v rows, heads inside each), wproj ``[D_out, h hd]``."""
    if x.dim() != 3 or wqkv.shape[0] != 3 * h * hd or wproj.shape[1] != h * hd:
        raise ValueError("attn_block: x [B, T, D], wqkv [3 h hd, D], wproj [D_out, h hd] expected")
    if not supported(x, hd):
        raise ValueError(f"attn_block: bf16 CUDA input with head dim in {HEAD_DIMS} expected")
    return _AttnBlock.apply(x, wqkv, bqkv, wproj, bproj, h, hd, causal,
                            scale if scale is not None else 1.0 / math.sqrt(hd), residual)


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                    scale: float | None = None) -> torch.Tensor:
    """softmax(scale * q k^T (+ causal mask)) v for [B, H, T, D] bf16 views (D = 64 / 128)."""
    D = q.shape[-1]
    return _FlashAttn.apply(q, k, v, causal, scale if scale is not None else 1.0 / math.sqrt(D))


def attention_qkv(qkv: torch.Tensor, h: int, hd: int, causal: bool = True, scale: float | None = None) -> torch.Tensor:
    """Attention of the fused QKV output ``[B, T, 3 * h * hd]`` (q | k | v, heads inside each) ->
    ``[B, T, h * hd]``, the output projection's input layout."""
    if not qkv.is_contiguous() or qkv.shape[-1] != 3 * h * hd:
        raise ValueError("attention_qkv: contiguous [B, T, 3 * h * hd] expected")
    if not supported(qkv, hd):
        raise ValueError(f"attention_qkv: bf16 CUDA input with head dim in {HEAD_DIMS} expected")
    return _FlashAttnQKV.apply(qkv, h, hd, causal, scale if scale is not None else 1.0 / math.sqrt(hd))


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
