"""bf16 GEMM on the hand-written gfx950 MFMA kernel (kernels/gemm_bf16.hip).

``gemm_nt(a, b)`` computes ``a @ b.T`` (``b`` stored [N, K], K contiguous — the ``F.linear``
weight layout), optionally batched, with a fused epilogue: ``alpha``, bias, activation
(relu / gelu_tanh / silu) or residual add. ``linear`` is the autograd-aware ``F.linear``
replacement used by :mod:`kubeflow_rm_amd.models` and the TP layers.
"""
from __future__ import annotations

import torch

from . import _lib

ACTS = {"none": 0, "relu": 1, "gelu_tanh": 2, "gelu": 2, "silu": 3}
VARIANTS = {"auto": 0, "fast": 1, "generic": 2, "pipe": 3, "pipe_sched": 4, "w4": 6, "w4s": 9}


def _stream_ptr(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _check_operand(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name} must be bfloat16, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if t.stride(-1) != 1:
        raise ValueError(f"{name} must have a contiguous last dimension")


# Shapes off the MFMA tiles (M, N % 128, K % 64) would run on the generic kernel at a third to a
# half of the tiled kernels' rate (profiles/r2_gemm_unaligned). Above this size the operands are
# zero-padded up to the tiles instead: the copies cost a few percent of the GEMM.
_PAD_MIN_FLOPS = 2.0 * 1024 ** 3


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _gemm_nt_padded(a3, b, bias, residual, alpha, act, out, batched, batch, M, N, K):
    """Zero-pad to the tile grid, run the tiled kernel, copy the [M, N] corner into ``out``."""
    big = -(-M // 256) * -(-N // 256) * batch > 128  # the auto dispatch's 256-tile threshold
    tm = 256 if big else 128
    Mp, Np, Kp = _round_up(M, tm), _round_up(N, tm), _round_up(K, 64)
    F = torch.nn.functional

    def pad(t, cols, rows):  # copy only an operand that is off the grid (e.g. just B for an odd N)
        return t if cols == 0 and rows == 0 else F.pad(t, (0, cols, 0, rows))

    ap = pad(a3, Kp - K, Mp - M)
    bp = pad(b, Kp - K, Np - N)
    bias_p = F.pad(bias, (0, Np - N)) if bias is not None and Np != N else bias
    res_p = None
    if residual is not None:
        r3 = residual.view(batch, M, N) if batched else residual.reshape(M, N)
        res_p = pad(r3, Np - N, Mp - M)
    c3 = out.view(batch, M, N) if batched else out.view(M, N)
    if Mp == M and Np == N:  # only K was off the grid: write straight into out
        gemm_nt(ap, bp, bias=bias_p, residual=res_p, alpha=alpha, act=act, out=c3)
        return out
    cp = gemm_nt(ap, bp, bias=bias_p, residual=res_p, alpha=alpha, act=act)
    c3.copy_(cp[..., :M, :N])
    return out


def gemm_nt(a: torch.Tensor, b: torch.Tensor, *, bias: torch.Tensor | None = None,
            residual: torch.Tensor | None = None, alpha: float = 1.0, act: str = "none",
            out: torch.Tensor | None = None, variant: str = "auto") -> torch.Tensor:
    """C = act(alpha * a @ b^T + bias) (+ residual). a: [..., M, K] or [B, M, K]; b: [N, K] or [B, N, K]."""
    _check_operand(a, "a")
    _check_operand(b, "b")
    batched = b.dim() == 3
    if batched:
        if a.dim() != 3 or a.shape[0] != b.shape[0]:
            raise ValueError("batched gemm_nt needs a: [B, M, K] and b: [B, N, K]")
        batch, M, K = a.shape
        N = b.shape[1]
        a3 = a
    else:
        if b.dim() != 2:
            raise ValueError("b must be [N, K] or [B, N, K]")
        K = a.shape[-1]
        a3 = a.reshape(-1, K) if a.dim() != 2 else a
        if a3.stride(-1) != 1:
            a3 = a3.contiguous()
        batch, M = 1, a3.shape[0]
        N = b.shape[0]
    if b.shape[-1] != K:
        raise ValueError(f"inner dims differ: a has K={K}, b has K={b.shape[-1]}")
    out_shape = (batch, M, N) if batched else (*a.shape[:-1], N)
    if out is None:
        out = torch.empty(out_shape, dtype=torch.bfloat16, device=a.device)
    else:
        # the kernel writes bf16 bit patterns with a 16-byte-aligned, unit-stride row layout
        _check_operand(out, "out")
        if out.device != a.device or tuple(out.shape) != tuple(out_shape):
            raise ValueError(f"out must be a bf16 {tuple(out_shape)} tensor on {a.device}, got {tuple(out.shape)} on {out.device}")
    c3 = out.view(batch, M, N) if batched else out.view(M, N)
    lda = a3.stride(-2) if a3.dim() >= 2 else K
    ldb = b.stride(-2)
    ldc = c3.stride(-2)
    sa = a3.stride(0) if batched else M * lda
    sb = b.stride(0) if batched else N * ldb
    sc = c3.stride(0) if batched else M * ldc
    if bias is not None:
        _check_operand(bias, "bias")
        if bias.numel() != N or not bias.is_contiguous():
            raise ValueError("bias must be a contiguous [N] tensor")
    if (variant == "auto" and (M % 128 or N % 128 or K % 64)
            and flops(M, N, K, batch) >= _PAD_MIN_FLOPS):
        return _gemm_nt_padded(a3, b, bias, residual, alpha, act, out, batched, batch, M, N, K)
    r_ptr, ldr, sr = None, 0, 0
    if residual is not None:
        _check_operand(residual, "residual")
        r3 = residual.view(batch, M, N) if batched else residual.reshape(M, N)
        r_ptr, ldr = r3.data_ptr(), r3.stride(-2)
        sr = r3.stride(0) if batched else M * ldr
    rc = _lib.lib().kfamd_gemm_nt_bf16_variant(
        VARIANTS[variant], a3.data_ptr(), b.data_ptr(), c3.data_ptr(),
        bias.data_ptr() if bias is not None else None, r_ptr,
        M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, float(alpha), ACTS[act],
        _stream_ptr(a))
    _lib.check(rc, f"gemm_nt[{M}x{N}x{K}x{batch}]")
    return out


def matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b with b stored [K, N] (row-major). Transposes b once into the NT layout."""
    return gemm_nt(a, b.t().contiguous())


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act):
        y = gemm_nt(x, weight, bias=bias, act=act if bias is not None or act != "none" else "none")
        ctx.save_for_backward(x, weight, bias, y if act == "relu" else None)
        ctx.act = act
        if act not in ("none", "relu"):
            # need pre-activation for gelu/silu backward: recompute cheaply in backward
            ctx.needs_preact = True
        else:
            ctx.needs_preact = False
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, bias, y = ctx.saved_tensors
        K = x.shape[-1]
        N = weight.shape[0]
        x2 = x.reshape(-1, K)
        gy2 = gy.reshape(-1, N).contiguous()
        if ctx.act == "relu":
            gy2 = gy2 * (y.reshape(-1, N) > 0)
        elif ctx.needs_preact:
            pre = gemm_nt(x2, weight, bias=bias).float()
            with torch.enable_grad():
                p = pre.detach().requires_grad_(True)
                f = torch.nn.functional.gelu(p, approximate="tanh") if ctx.act in ("gelu", "gelu_tanh") \
                    else torch.nn.functional.silu(p)
                (g,) = torch.autograd.grad(f, p, gy2.float())
            gy2 = g.to(torch.bfloat16)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = gemm_nt(gy2, weight.t().contiguous()).reshape(x.shape)
        if ctx.needs_input_grad[1]:
            gw = gemm_nt(gy2.t().contiguous(), x2.t().contiguous())
        if bias is not None and ctx.needs_input_grad[2]:
            gb = gy2.float().sum(0).to(bias.dtype)
        return gx, gw, gb, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
           act: str = "none") -> torch.Tensor:
    """Autograd-aware ``act(F.linear(x, weight, bias))`` on the MFMA kernel."""
    return _Linear.apply(x, weight, bias, act)


def flops(M: int, N: int, K: int, batch: int = 1) -> float:
    return 2.0 * M * N * K * batch
