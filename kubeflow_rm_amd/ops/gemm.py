"""bf16 GEMM on the hand-written gfx950 MFMA kernel (kernels/gemm_bf16.hip).

``gemm_nt(a, b)`` computes ``a @ b.T`` (``b`` stored [N, K], K contiguous — the ``F.linear``
weight layout), optionally batched, with a fused epilogue: ``alpha``, bias, activation
(relu / gelu_tanh / silu) or residual add. ``linear`` is the autograd-aware ``F.linear``
replacement used by :mod:`kubeflow_rm_amd.models` and the TP layers.
"""
from __future__ import annotations

import os

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


# The w4 kernels handle edge tiles in-kernel (gemm_w4.h) for M, N >= 128 with K % 8 == 0, any N
# and output alignment (NT layout). K off the 8-grid costs one fused pack of both operands
# (kfamd_pad_k_bf16); M or N below the tile would run on the generic kernel at a third to a half
# of the tiled kernels' rate (profiles/r2_gemm_unaligned): above this size they are zero-padded.
_PAD_MIN_FLOPS = 2.0 * 1024 ** 3


def _w4_shape(M: int, N: int, K: int) -> bool:
    """Every w4 layout and split-K (16-B rows along N too)."""
    return M >= 128 and N >= 128 and N % 8 == 0 and K % 8 == 0


def _w4_nt_shape(M: int, N: int, K: int) -> bool:
    """The NT w4 kernel (any N: the epilogue stores odd widths element-wise)."""
    return M >= 128 and N >= 128 and K % 8 == 0


def pad_k(x: torch.Tensor, y: torch.Tensor | None, Kp: int):
    """Zero-pad the last dim of one or two bf16 operands to Kp (% 8) in one kernel launch."""
    outs = []
    jobs = []
    for t in (x, y):
        if t is None:
            continue
        t2 = t.reshape(-1, t.shape[-1]) if t.dim() != 2 else t
        if t2.stride(-1) != 1 or (t.dim() == 3 and t.stride(0) != t.shape[1] * t.stride(1)):
            t2 = t.contiguous().reshape(-1, t.shape[-1])
        d = torch.empty(*t.shape[:-1], Kp, dtype=torch.bfloat16, device=t.device)
        outs.append(d)
        jobs.append((t2.data_ptr(), d.data_ptr(), t2.shape[0], t2.stride(0)))
    j1 = jobs[1] if len(jobs) > 1 else (None, None, 0, 0)
    rc = _lib.lib().kfamd_pad_k_bf16(*jobs[0], *j1, x.shape[-1], Kp, _stream_ptr(x))
    _lib.check(rc, f"pad_k[{x.shape[-1]}->{Kp}]")
    return outs[0], (outs[1] if y is not None else None)


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _gemm_nt_padded(a3, b, bias, residual, alpha, act, out, batched, batch, M, N, K):
    """Zero-pad to the tile grid, run the tiled kernel, copy the [M, N] corner into ``out``."""
    Kp = _round_up(K, 8)
    if M >= 128 and N >= 128:  # only K is off the grid: pack both operands, write out directly
        ap, bp = pad_k(a3, b, Kp)
        c3 = out.view(batch, M, N) if batched else out.view(M, N)
        gemm_nt(ap, bp, bias=bias, residual=residual, alpha=alpha, act=act, out=c3)
        return out
    # pad only up to the w4 contract (M, N >= 128, K % 8): the kernel handles the rest
    Mp, Np = max(M, 128), max(N, 128)
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
    if (variant == "auto" and not _w4_nt_shape(M, N, K)
            and ((M >= 128 and N >= 128) or flops(M, N, K, batch) >= _PAD_MIN_FLOPS)):
        return _gemm_nt_padded(a3, b, bias, residual, alpha, act, out, batched, batch, M, N, K)
    r_ptr, ldr, sr = None, 0, 0
    if residual is not None:
        _check_operand(residual, "residual")
        r3 = residual.view(batch, M, N) if batched else residual.reshape(M, N)
        r_ptr, ldr = r3.data_ptr(), r3.stride(-2)
        sr = r3.stride(0) if batched else M * ldr
    fx = (fixk_plan(M, N, K, batch) if variant == "auto" and bias is None and act == "none" else None)
    if fx is not None and _fixk(0, 0, a3, b, c3, M, N, K, batch, lda, ldb, ldc, sa, sb, sc, fx, r_ptr=r_ptr, ldr=ldr,
                                sr=sr, alpha=alpha) == 0:
        return out
    plan = splitk_plan(M, N, K, batch) if variant == "auto" else None
    if plan is not None and _splitk(0, 0, a3, b, c3, M, N, K, batch, lda, ldb, ldc, sa, sb, sc, plan, bias=bias,
                                    r_ptr=r_ptr, ldr=ldr, sr=sr, aux=None, alpha=alpha, act=act) == 0:
        return out
    skp = streamk_plan(M, N, K, batch) if variant == "auto" and plan is None else None
    if skp is not None and _streamk(a3, b, c3, M, N, K, lda, ldb, ldc, skp, bias=bias, r_ptr=r_ptr, ldr=ldr,
                                     aux=None, alpha=alpha, act=act) == 0:
        return out
    rc = _lib.lib().kfamd_gemm_nt_bf16_variant(
        VARIANTS[variant], a3.data_ptr(), b.data_ptr(), c3.data_ptr(),
        bias.data_ptr() if bias is not None else None, r_ptr,
        M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr, float(alpha), ACTS[act],
        _stream_ptr(a))
    _lib.check(rc, f"gemm_nt[{M}x{N}x{K}x{batch}]")
    return out


# Split-K (kfamd_w4_splitk_*): a problem with too few 128x128 output tiles leaves CUs idle, so it is
# split along K (fp32 partials + one reduce launch carrying the epilogue). The split count minimises a
# small cost model: the busiest CU's share of MFMA work (a w4s block takes 80 KB of LDS, so two run
# per CU, and a second resident block adds ~15 % throughput by hiding the other's latency), plus the
# partials' HBM round trip and the reduce launch. Each split is at least _SPLITK_MIN_K deep. Below
# _SPLITK_MIN_TOTAL_K the unsplit kernel finishes in ~10 us and the extra launch costs more than it
# saves (profiles/r3_splitk: 1000^3 10.7 us unsplit vs 15.9 split). Measured against the one-block-
# per-CU plan on the gpt-small weight-gradient shapes (profiles/r3_splitk_slots): 3072x768x32768
# 256 -> 184 us, 768x3072x32768 259 -> 170, 2304x768x32768 146 -> 124.
_NUM_CUS = 256
_SPLITK_MIN_K = 512
_SPLITK_MIN_TOTAL_K = 2048
_SPLITK_MAX = 8
SPLITK = True  # kill switch (benchmarks/tests compare against the unsplit kernel)
_CU_TFLOPS = 5.1e12        # one w4s block alone on a CU (~1.3 PF/s over 256 CUs)
_HBM_BPS = 5.0e12          # partial write + read in the split path
_REDUCE_LAUNCH_S = 5e-6


def _splitk_cost(M: int, N: int, K: int, batch: int, s: int) -> float:
    tiles = -(-M // 128) * -(-N // 128) * batch
    per_cu = -(-tiles * s // _NUM_CUS)
    gemm = per_cu * (2.0 * 128 * 128 * -(-K // s)) / _CU_TFLOPS * (0.85 if per_cu >= 2 else 1.0)
    if s == 1:
        return gemm
    return gemm + s * M * N * batch * 8.0 / _HBM_BPS + _REDUCE_LAUNCH_S


def splitk_plan(M: int, N: int, K: int, batch: int = 1) -> tuple[int, int] | None:
    """(splits, kper) for a w4-shaped problem that under-fills the chip, else None."""
    if not SPLITK or K < _SPLITK_MIN_TOTAL_K or not _w4_shape(M, N, K):
        return None
    tiles = -(-M // 128) * -(-N // 128) * batch
    if tiles >= 2 * _NUM_CUS:
        return None
    best, best_cost = 1, _splitk_cost(M, N, K, batch, 1)
    for s in range(2, min(_SPLITK_MAX, K // _SPLITK_MIN_K) + 1):
        c = _splitk_cost(M, N, K, batch, s)
        if c < 0.95 * best_cost:  # a finer split has to pay for its extra partials clearly
            best, best_cost = s, c
    if best < 2:
        return None
    kper = _round_up(-(-K // best), 64)
    splits = -(-K // kper)
    return (splits, kper) if splits >= 2 else None


def _splitk(la, lb, a, b, c, M, N, K, batch, lda, ldb, ldc, sa, sb, sc, plan, *, bias, r_ptr, ldr, sr, aux,
            alpha, act) -> int:
    splits, kper = plan
    L = _lib.lib()
    w = torch.empty(splits * batch * M * N, dtype=torch.float32, device=a.device)
    st = _stream_ptr(a)
    if la == 0 and lb == 0:
        rc = L.kfamd_w4_splitk_nt(a.data_ptr(), b.data_ptr(), w.data_ptr(), M, N, K, batch, splits, kper,
                                  lda, ldb, sa, sb, st)
    else:
        rc = L.kfamd_w4_splitk_t(la, lb, a.data_ptr(), b.data_ptr(), w.data_ptr(), M, N, K, batch, splits, kper,
                                 lda, ldb, sa, sb, st)
    if rc != 0:
        return rc
    return L.kfamd_splitk_reduce(w.data_ptr(), c.data_ptr(), bias.data_ptr() if bias is not None else None, r_ptr,
                                 aux.data_ptr() if aux is not None else None, M, N, batch, splits, ldc, ldr, sc, sr,
                                 float(alpha), ACTS[act], st)


# Split-K with the in-kernel fixup (kfamd_w4_splitk_fix, gemm_w4.h SPLIT == 2): a problem with far
# fewer 256x256 tiles than CUs (a weight gradient of a square projection: 2048^2 x 8192 is 64 tiles)
# runs S K-splits per tile on the 256 tile; every split stores its fp32 partial in fragment order
# (whole 128-B lines per store), the last split of a tile to arrive adds the others and runs the
# epilogue. No reduce launch, no waiting, no co-residency assumption. FIXK_SPLITS pins S for A/B runs.
FIXK = True
FIXK_SPLITS: int | None = None
_FIXK_MIN_KT = 32            # K-tiles (x64) per split: shallower splits pay more for the partial than they save
_FIXK_MAX = 7
_fixk_ws: dict = {}          # (device, stream) -> [W fp32 partials, arrival counters]


def fixk_plan(M: int, N: int, K: int, batch: int = 1) -> tuple[int, int] | None:
    """(splits, kper) for a 256-tile split-K fixup run of a problem with too few tiles, else None.

    Measured against the previous plans (profiles/r4_fixk/fixk.jsonl; hot = operands cache-resident,
    cold = after a 512 MiB eviction): each split publishes a 256 KiB fp32 partial through the CU's
    store path and the owner reads the others back, which pays when every split keeps >= 32 K-tiles
    and the splits fill >= 70 % of the CUs: 2048^2 x 8192 at 4 splits 69.0 / 86.4 us vs 69.5 / 106.0
    on the 128 tile; 4096x2048x8192 at 2 104.8 / 115.5 vs 116.9 / 140.3; 3072x768x32768 at 7
    152.6 / 164.2 vs 179.6 / 222.9 (128-tile split-K); 2304x768x32768 at 7 113.9 / 151.6 vs
    127.6 / 170.4. More than 7 splits lose (the owner reads every partial)."""
    if not FIXK or M < 256 or N < 256 or not _w4_shape(M, N, K):
        return None
    tiles = -(-M // 256) * -(-N // 256) * batch
    kt = -(-K // 64)
    if FIXK_SPLITS is not None:
        best = FIXK_SPLITS
    else:
        if tiles < 24 or tiles > _NUM_CUS // 2:
            return None
        best = min(_NUM_CUS // tiles, kt // _FIXK_MIN_KT, _FIXK_MAX)
        if best < 2 or tiles * best < _NUM_CUS * 7 // 10:
            return None
    if best < 2:
        return None
    kper = _round_up(-(-K // best), 64)
    splits = -(-K // kper)
    return (splits, kper) if splits >= 2 else None


def _fixk(la, lb, a, b, c, M, N, K, batch, lda, ldb, ldc, sa, sb, sc, plan, *, r_ptr, ldr, sr, alpha) -> int:
    splits, kper = plan
    tiles = -(-M // 256) * -(-N // 256) * batch
    key = (a.device, _stream_ptr(a))
    ws = _fixk_ws.get(key)
    need_w = splits * tiles * 256 * 256
    if ws is None or ws[0].numel() < need_w or ws[1].numel() < tiles:
        old = (ws[0].numel(), ws[1].numel()) if ws is not None else (0, 0)
        ws = [torch.empty(max(need_w, old[0]), dtype=torch.float32, device=a.device),
              torch.zeros(max(tiles, old[1], 1024), dtype=torch.int32, device=a.device)]
        _fixk_ws[key] = ws
    return _lib.lib().kfamd_w4_splitk_fix(la, lb, a.data_ptr(), b.data_ptr(), c.data_ptr(), r_ptr, M, N, K, batch,
                                          lda, ldb, ldc, ldr, sa, sb, sc, sr, float(alpha), ws[0].data_ptr(),
                                          ws[1].data_ptr(), splits, kper, _stream_ptr(a))


# Stream-K (kfamd_w4_streamk_nt, gemm_w4.h SK): a 256x256-tile problem whose tile count leaves the
# last wave of 256 CUs partly idle (e.g. 144 tiles of 3072^2: 56 % of one wave) runs as a persistent
# grid of one block per CU: the whole waves as plain tiles, then the leftover tiles in S K-splits
# each, round-robin over all blocks; the block with a tile's last split adds the others' fp32
# partials in its epilogue (no reduce launch).
# Off by default: correct (tests/test_gpu_kernels.py) but slower than the plain kernel on every
# measured shape. Each split moves a 256 KB fp32 partial tile through HBM twice, which costs more
# than the idle CUs it fills (profiles/r3_streamk: 3072^2 x 8192 at 3 splits 189 us vs 144 plain,
# 120 us with the partial traffic ablated).
STREAMK = False
_STREAMK_MIN_KT = 16        # K-tiles (x64) per tile: shallower problems are prologue / epilogue bound
_STREAMK_MAX_WAVES = 4      # beyond this the partial last wave costs < 1/8 of the run
_STREAMK_UNIT_COST = 3      # per-split overhead in K-tiles (prologue, partial store / add, epilogue)
_streamk_ws: dict = {}      # (device, stream) -> [W fp32 partials, flags u32, epoch]


def streamk_plan(M: int, N: int, K: int, batch: int = 1) -> tuple[int, int] | None:
    """(grid, splits) for a stream-K run of an NT problem that leaves the last wave under-filled, else None."""
    if not STREAMK or batch != 1 or not _w4_nt_shape(M, N, K) or M < 256 or N < 256:
        return None
    tiles = -(-M // 256) * -(-N // 256)
    kt = -(-K // 64)
    G = _NUM_CUS
    rem = tiles % G
    if kt < _STREAMK_MIN_KT or rem == 0 or tiles > _STREAMK_MAX_WAVES * G or rem > G * 7 // 8:
        return None

    P = 8 if rem >= 8 else 1  # XCD partitions of the leftover tiles (gemm_w4.h SK)

    def cost(S):  # leftover part: rounds of units, each ceil(KT / S) K-tiles + the per-unit overhead
        return -(-S * -(-rem // P) // (G // P)) * (-(-kt // S) + (_STREAMK_UNIT_COST if S > 1 else 0))

    best = min(range(1, min(64, kt // 4) + 1), key=lambda S: (cost(S), S))
    if best == 1 or cost(best) >= 0.9 * cost(1):
        return None
    return G, best


def _streamk(a, b, c, M, N, K, lda, ldb, ldc, plan, *, bias, r_ptr, ldr, aux, alpha, act,
             _force_deadline: bool = False) -> int:
    grid, splits = plan
    rem = (-(-M // 256) * -(-N // 256)) % grid
    key = (a.device, _stream_ptr(a))
    ws = _streamk_ws.get(key)
    need_w, need_f = max(1, (splits - 1) * rem) * 256 * 256, splits * rem
    if ws is None or ws[0].numel() < need_w or ws[1].numel() < need_f:
        old = (ws[0].numel(), ws[1].numel()) if ws is not None else (0, 0)
        ws = [torch.empty(max(need_w, old[0]), dtype=torch.float32, device=a.device),
              torch.zeros(max(need_f, old[1], 1024), dtype=torch.int32, device=a.device), 0]
        _streamk_ws[key] = ws
    ws[2] += 1
    if ws[2] >= 2 ** 32 - 1:  # epochs never repeat a value a flag may still hold
        ws[1].zero_()
        ws[2] = 1
    return _lib.lib().kfamd_w4_streamk_nt(
        a.data_ptr(), b.data_ptr(), c.data_ptr(), bias.data_ptr() if bias is not None else None, r_ptr,
        aux.data_ptr() if aux is not None else None, M, N, K, lda, ldb, ldc, ldr, float(alpha), ACTS[act],
        ws[0].data_ptr(), ws[1].data_ptr(), ws[2], grid, -splits if _force_deadline else splits, _stream_ptr(a))


def _ex(la, lb, a, b, c, M, N, K, batch, lda, ldb, ldc, sa, sb, sc, *, bias=None, residual=None, aux=None,
        alpha=1.0, act="none") -> int:
    """Raw kfamd_gemm_bf16_ex call (split-K when the problem under-fills the chip); returns the status
    (0 = launched)."""
    r_ptr, ldr, sr = None, 0, 0
    if residual is not None:
        r_ptr, ldr, sr = residual.data_ptr(), residual.stride(-2), (residual.stride(0) if residual.dim() == 3 else 0)
    fx = fixk_plan(M, N, K, batch) if bias is None and aux is None and act == "none" and (la, lb) != (1, 0) else None
    if fx is not None and _fixk(la, lb, a, b, c, M, N, K, batch, lda, ldb, ldc, sa, sb, sc, fx, r_ptr=r_ptr, ldr=ldr,
                                sr=sr, alpha=alpha) == 0:
        return 0
    plan = splitk_plan(M, N, K, batch)
    if plan is not None:
        rc = _splitk(la, lb, a, b, c, M, N, K, batch, lda, ldb, ldc, sa, sb, sc, plan, bias=bias, r_ptr=r_ptr,
                     ldr=ldr, sr=sr, aux=aux, alpha=alpha, act=act)
        if rc == 0:
            return 0
    # (the pre-activation output runs on the plain kernel: see kfamd_w4_streamk_nt)
    skp = streamk_plan(M, N, K, batch) if la == 0 and lb == 0 and plan is None and aux is None else None
    if skp is not None and _streamk(a, b, c, M, N, K, lda, ldb, ldc, skp, bias=bias, r_ptr=r_ptr, ldr=ldr,
                                     aux=aux, alpha=alpha, act=act) == 0:
        return 0
    return _lib.lib().kfamd_gemm_bf16_ex(
        la, lb, a.data_ptr(), b.data_ptr(), c.data_ptr(), bias.data_ptr() if bias is not None else None, r_ptr,
        aux.data_ptr() if aux is not None else None, M, N, K, batch, lda, ldb, ldc, ldr, sa, sb, sc, sr,
        float(alpha), ACTS[act], _stream_ptr(a))


def mm(a: torch.Tensor, b: torch.Tensor, *, trans_a: bool = False, trans_b: bool = False,
       out: torch.Tensor | None = None, residual: torch.Tensor | None = None, alpha: float = 1.0) -> torch.Tensor:
    """``alpha * op(a) @ op(b) (+ residual)`` for 2-D or batched 3-D bf16 operands, op = transpose when
    the flag is set, on the w4 MFMA kernel in whichever operand layout the tensors already have: a
    transposed operand is read k-major through ``ds_read_b64_tr_b16`` instead of being copied
    (``kernels/gemm_bf16_w4_t.hip``). Shapes the tiled kernel does not take (a dimension < 128, an odd
    inner extent) run ``gemm_nt`` on transposed copies. ``residual`` may be ``out`` itself
    (accumulate)."""
    _check_operand(a, "a")
    _check_operand(b, "b")
    if a.dim() != b.dim() or a.dim() not in (2, 3) or (a.dim() == 3 and a.shape[0] != b.shape[0]):
        raise ValueError("mm needs two 2-D or two equally batched 3-D operands")
    batched = a.dim() == 3
    batch = a.shape[0] if batched else 1
    M, K = (a.shape[-1], a.shape[-2]) if trans_a else (a.shape[-2], a.shape[-1])
    Kb, N = (b.shape[-1], b.shape[-2]) if trans_b else (b.shape[-2], b.shape[-1])
    if K != Kb:
        raise ValueError(f"inner dims differ: {K} vs {Kb}")
    out_shape = (batch, M, N) if batched else (M, N)
    if out is None:
        out = torch.empty(out_shape, dtype=torch.bfloat16, device=a.device)
    else:
        _check_operand(out, "out")
        if tuple(out.shape) != out_shape or out.device != a.device:
            raise ValueError(f"out must be a bf16 {out_shape} tensor on {a.device}")
    if residual is not None:
        _check_operand(residual, "residual")
        if tuple(residual.shape) != out_shape:
            raise ValueError(f"residual must be {out_shape}")
    la = 1 if trans_a else 0          # kernel A operand [M][K]: K contiguous unless a is read transposed
    lb = 0 if trans_b else 1          # kernel B operand [N][K]: b [K][N] is k-major
    sa = a.stride(0) if batched else 0
    sb = b.stride(0) if batched else 0
    sc = out.stride(0) if batched else 0
    rc = _ex(la, lb, a, b, out, M, N, K, batch, a.stride(-2), b.stride(-2), out.stride(-2), sa, sb, sc,
             residual=residual, alpha=alpha)
    if rc > 0:
        _lib.check(rc, f"mm[{M}x{N}x{K}x{batch}]")
    if rc == 0:
        return out
    # fallback: materialise the NT operands (shape outside the tiled kernel's contract)
    a_nt = (a.transpose(-1, -2) if trans_a else a).contiguous()
    b_nt = (b if trans_b else b.transpose(-1, -2)).contiguous()
    res = residual.clone() if residual is not None and residual.data_ptr() == out.data_ptr() else residual
    return gemm_nt(a_nt, b_nt, residual=res, alpha=alpha, out=out)


def matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b with b stored [K, N] (row-major), read k-major in place (no transposed copy):
    [M, K] @ [K, N], [..., M, K] @ [K, N] (leading dims folded into M) and batched
    [B, M, K] @ [B, K, N]."""
    if b.dim() == 2:
        if a.dim() == 2:
            return mm(a, b)
        a2 = a.reshape(-1, a.shape[-1])
        return mm(a2, b).view(*a.shape[:-1], b.shape[-1])
    if a.dim() == 3 and b.dim() == 3:
        return mm(a, b)
    return gemm_nt(a, b.transpose(-1, -2).contiguous())


# gelu / silu forward: in the GEMM epilogue (second output z, the default) or as GEMM -> z, then one
# elementwise y = act(z) pass ("split"). With the 8 k-cycle epilogue the fused form wins or ties at
# every measured shape (profiles/r3_train_step: 8192x2048x8192 fwd 0.257 ms fused, 0.275 split,
# torch 0.261); the split form stays selectable for A/B runs.
PREACT_MODE = "auto"      # "fused" | "split" | "auto" (= fused)


def _preact_split(M: int, N: int) -> bool:
    return PREACT_MODE == "split" and N % 8 == 0


def gemm_nt_preact(x2: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None, act: str):
    """(y, z): y = act(x2 @ weight^T + bias) and the pre-activation z (for gelu/silu backward),
    either both from ONE GEMM (the epilogue's second output) or z from the GEMM and y from one
    elementwise pass (large grids, see PREACT_MODE)."""
    M, K = x2.shape
    N = weight.shape[0]
    y = torch.empty(M, N, dtype=torch.bfloat16, device=x2.device)
    z = torch.empty_like(y)
    if bias is not None:
        _check_operand(bias, "bias")
    if _preact_split(M, N):
        gemm_nt(x2, weight, bias=bias, out=z)
        _lib.check(_lib.lib().kfamd_act_fwd_bf16(z.data_ptr(), y.data_ptr(), M * N, ACTS[act], _stream_ptr(z)),
                   f"act_fwd[{M}x{N}]")
        return y, z
    rc = _ex(0, 0, x2, weight, y, M, N, K, 1, x2.stride(0), weight.stride(0), N, 0, 0, 0, bias=bias, aux=z,
             act=act)
    if rc > 0:
        _lib.check(rc, f"gemm_nt_preact[{M}x{N}x{K}]")
    if rc == 0:
        return y, z
    z = gemm_nt(x2, weight, bias=bias)
    F = torch.nn.functional
    yf = F.gelu(z.float(), approximate="tanh") if act in ("gelu", "gelu_tanh") else F.silu(z.float())
    return yf.to(torch.bfloat16), z


def act_grad(gy: torch.Tensor, z: torch.Tensor | None, act: str, need_bias_grad: bool,
             db_dtype: torch.dtype = torch.float32):
    """(g, db): g = gy * act'(z) (z = pre-activation; the output y for relu), db = column sums of g
    (accumulated in fp32, returned as ``db_dtype``: fp32 or bf16) — one fused HIP pass
    (kernels/act_grad_bf16.hip). act == 'none': g = gy."""
    rows, cols = gy.shape
    L = _lib.lib()
    if act == "none" and not need_bias_grad:
        return gy, None
    if cols % 8 or gy.stride(-1) != 1 or (z is not None and not z.is_contiguous()) or not gy.is_contiguous():
        F = torch.nn.functional
        if act == "none":
            g = gy
        elif act == "relu":
            g = gy * (z > 0)
        else:
            with torch.enable_grad():
                p = z.float().requires_grad_(True)
                f = F.gelu(p, approximate="tanh") if act in ("gelu", "gelu_tanh") else F.silu(p)
                (gf,) = torch.autograd.grad(f, p, gy.float())
            g = gf.to(torch.bfloat16)
        return g, (g.float().sum(0).to(db_dtype) if need_bias_grad else None)
    g = gy if act == "none" else torch.empty_like(gy)
    db = ws = None
    db_bf16 = db_dtype == torch.bfloat16
    if need_bias_grad:
        db = torch.empty(cols, dtype=torch.bfloat16 if db_bf16 else torch.float32, device=gy.device)
        ws = torch.empty(L.kfamd_act_grad_workspace(rows, cols) // 4, dtype=torch.float32, device=gy.device)
    rc = L.kfamd_act_grad_bf16_v2(gy.data_ptr(), z.data_ptr() if z is not None else None,
                                  g.data_ptr() if act != "none" else None, db.data_ptr() if db is not None else None,
                                  int(db_bf16), ws.data_ptr() if ws is not None else None, rows, cols, ACTS[act],
                                  _stream_ptr(gy))
    _lib.check(rc, f"act_grad[{rows}x{cols}]")
    return g, db


class _Linear(torch.autograd.Function):
    """y = act(x W^T + b). Forward: one GEMM whose epilogue also stores the pre-activation for gelu /
    silu. Backward: one fused act-grad + bias-grad pass, then dgrad (g·W, W read k-major) and wgrad
    (g^T·X, both read k-major) on the w4 kernel: no transposed copies, no recomputed GEMM."""

    @staticmethod
    def forward(ctx, x, weight, bias, act, residual):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        z = None
        if act in ("gelu", "gelu_tanh", "silu"):
            y, z = gemm_nt_preact(x2, weight, bias, act)
            y = y.view(*x.shape[:-1], weight.shape[0])
            if residual is not None:
                y = y + residual
        elif residual is not None and act == "none":
            # the residual add of a transformer block's output projection, in the GEMM epilogue
            y = gemm_nt(x, weight, bias=bias, residual=residual.contiguous())
        else:
            y = gemm_nt(x, weight, bias=bias, act=act)
            if act == "relu":
                z = y  # relu' is read from the activation output BEFORE the residual add
            if residual is not None:
                y = y + residual
        ctx.save_for_backward(x2, weight, bias, z)
        ctx.act = act
        ctx.xshape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        x2, weight, bias, zy = ctx.saved_tensors
        N = weight.shape[0]
        gy2 = gy.reshape(-1, N)
        if not gy2.is_contiguous():
            gy2 = gy2.contiguous()
        need_db = bias is not None and ctx.needs_input_grad[2]
        zz = zy.reshape(-1, N) if zy is not None else None
        g, db = act_grad(gy2, zz, ctx.act, need_db,
                         db_dtype=torch.bfloat16 if need_db and bias.dtype == torch.bfloat16 else torch.float32)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = mm(g, weight).reshape(ctx.xshape)
        if ctx.needs_input_grad[1]:
            gw = mm(g, x2, trans_a=True)
        if need_db:
            gb = db.to(bias.dtype)
        # y = ... + residual: the residual's gradient is gy itself
        gr = gy if ctx.needs_input_grad[4] else None
        return gx, gw, gb, None, gr


# An MLP's fc2 dgrad and fc1's activation backward (+ fc1's bias-gradient partials) in one GEMM
# (gemm_w4.h DACT, kernels/tu/w4_dgrad_act.hip) instead of the GEMM, then act_grad's pass over its
# output and the pre-activation. False: the two-step form (A/B runs, profiles/r5ze_mlp).
FUSED_DGRAD_ACT = os.environ.get("KFAMD_FUSED_DGRAD_ACT", "1") != "0"


def dgrad_act(gy2: torch.Tensor, weight: torch.Tensor, z: torch.Tensor, act: str, need_bias_grad: bool,
              db_dtype: torch.dtype = torch.float32):
    """(g, db): g = (gy2 @ weight) * act'(z) — the gradient at the pre-activation z of the layer
    feeding ``weight``'s layer — and db = column sums of g, from one GEMM whose epilogue reads z; or
    None when the shape is outside that kernel's contract (M, N multiples of 256, K of 64, 16-B
    rows), and the caller takes ``mm`` + ``act_grad``."""
    if not FUSED_DGRAD_ACT or act not in ACTS or act == "none":
        return None
    M, K = gy2.shape
    N = weight.shape[1]
    if (weight.dim() != 2 or weight.shape[0] != K or tuple(z.shape) != (M, N) or gy2.dtype != torch.bfloat16
            or weight.dtype != torch.bfloat16 or z.dtype != torch.bfloat16
            or not (gy2.is_contiguous() and weight.is_contiguous() and z.is_contiguous())):
        return None
    L = _lib.lib()
    g = torch.empty(M, N, dtype=torch.bfloat16, device=gy2.device)
    db = ws = None
    db_bf16 = db_dtype == torch.bfloat16
    if need_bias_grad:
        db = torch.empty(N, dtype=torch.bfloat16 if db_bf16 else torch.float32, device=gy2.device)
        ws = torch.empty(L.kfamd_w4_dgrad_act_workspace(M, N) // 4, dtype=torch.float32, device=gy2.device)
    rc = L.kfamd_w4_dgrad_act(gy2.data_ptr(), weight.data_ptr(), g.data_ptr(), z.data_ptr(), M, N, K, K, N, N, N,
                              ACTS[act], ws.data_ptr() if ws is not None else None,
                              db.data_ptr() if db is not None else None, int(db_bf16), _stream_ptr(gy2))
    if rc < 0:
        return None
    _lib.check(rc, f"dgrad_act[{M}x{N}x{K}]")
    return g, db


_pair_ws: dict = {}  # (device, stream) -> [W fp32 partial tiles, arrival counters]
WGRAD_PAIR = os.environ.get("KFAMD_WGRAD_PAIR", "1") != "0"  # False: always two mm's (A/B runs)


def pair_plan(M1: int, N1: int, M2: int, N2: int, K: int) -> tuple[int, int] | None:
    """(splits, kper) for one launch of two weight gradients ([M_i][N_i] over K), or None when apart
    is better: together they stay within one wave of the 256 CUs and each alone under-fills it;
    below three quarters of a wave the K range splits (in-kernel fixup) until the blocks fill it."""
    t1, t2 = -(-M1 // 256) * -(-N1 // 256), -(-M2 // 256) * -(-N2 // 256)
    if not WGRAD_PAIR or t1 >= _NUM_CUS or t2 >= _NUM_CUS or t1 + t2 > _NUM_CUS:
        return None
    if t1 + t2 >= _NUM_CUS * 3 // 4:
        return 1, 0
    splits = min(_NUM_CUS // (t1 + t2), -(-K // 64) // _FIXK_MIN_KT, 64)
    if splits < 2:
        return None
    kper = _round_up(-(-K // splits), 64)
    splits = -(-K // kper)
    return (splits, kper) if splits >= 2 else None


def wgrad_pair(g1: torch.Tensor, x1: torch.Tensor, g2: torch.Tensor, x2: torch.Tensor, force: bool = False,
               plan: tuple[int, int] | None = None):
    """(g1^T x1, g2^T x2) — two weight gradients (g_i [K][M_i], x_i [K][N_i]) as one launch of the w4
    kernel (kernels/tu/w4_wgrad_pair.hip) when together they fill the chip's 256 CUs far better than
    apart (pair_plan): a transformer block's QKV + output projection at gpt-1b (192 + 64 tiles), or
    an MLP's / attention block's pair at small widths with K split by the in-kernel fixup (gpt-small:
    36 + 36 and 27 + 9 tiles). Else None and the caller runs two ``mm``s. ``force`` launches whenever
    the shapes fit the kernel, with ``plan`` (default: whole K) — tests."""
    if any(t.dim() != 2 or t.dtype != torch.bfloat16 or t.stride(-1) != 1 for t in (g1, x1, g2, x2)):
        return None
    K, M1 = g1.shape
    M2, N1, N2 = g2.shape[1], x1.shape[1], x2.shape[1]
    if g2.shape[0] != K or x1.shape[0] != K or x2.shape[0] != K or min(M1, M2, N1, N2) < 256:
        return None
    plan = (plan or (1, 0)) if force else pair_plan(M1, N1, M2, N2, K)
    if plan is None:
        return None
    splits, kper = plan
    o1 = torch.empty(M1, N1, dtype=torch.bfloat16, device=g1.device)
    o2 = torch.empty(M2, N2, dtype=torch.bfloat16, device=g1.device)
    W = cnt = None
    if splits > 1:
        tiles = -(-M1 // 256) * -(-N1 // 256) + -(-M2 // 256) * -(-N2 // 256)
        key = (g1.device, _stream_ptr(g1))
        ws = _pair_ws.get(key)
        need = splits * tiles * 256 * 256
        if ws is None or ws[0].numel() < need or ws[1].numel() < tiles:
            old = (ws[0].numel(), ws[1].numel()) if ws is not None else (0, 0)
            ws = [torch.empty(max(need, old[0]), dtype=torch.float32, device=g1.device),
                  torch.zeros(max(tiles, old[1], 256), dtype=torch.int32, device=g1.device)]
            _pair_ws[key] = ws
        W, cnt = ws[0].data_ptr(), ws[1].data_ptr()
    rc = _lib.lib().kfamd_w4_wgrad_pair_v2(g1.data_ptr(), x1.data_ptr(), o1.data_ptr(), M1, g1.stride(0), x1.stride(0),
                                           N1, g2.data_ptr(), x2.data_ptr(), o2.data_ptr(), M2, g2.stride(0),
                                           x2.stride(0), N2, N1, N2, K, splits, kper, W, cnt, _stream_ptr(g1))
    if rc < 0:
        return None
    _lib.check(rc, f"wgrad_pair[{M1}x{N1}+{M2}x{N2}x{K}/{splits}]")
    return o1, o2


class _MLP(torch.autograd.Function):
    """out = act(x W1^T + b1) W2^T + b2 (+ residual) as one autograd node, so that fc2's dgrad can
    apply fc1's activation backward in its epilogue (dgrad_act): the backward runs fc2's bias
    gradient, ONE GEMM for dH * act'(z1) (+ fc1's bias-gradient partials), fc1's dgrad, then both
    weight gradients (one launch where they under-fill the chip, wgrad_pair). The forward is the two
    linears' (gemm_nt_preact, gemm_nt with bias / residual)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, act, residual):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        y1, z1 = gemm_nt_preact(x2, w1, b1, act)
        res = residual.reshape(-1, w2.shape[0]).contiguous() if residual is not None else None
        out = gemm_nt(y1, w2, bias=b2, residual=res)
        ctx.save_for_backward(x2, w1, b1, w2, b2, y1, z1)
        ctx.act = act
        ctx.xshape = x.shape
        return out.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, w1, b1, w2, b2, y1, z1 = ctx.saved_tensors
        gy2 = gy.reshape(-1, w2.shape[0])
        if not gy2.is_contiguous():
            gy2 = gy2.contiguous()
        ni = ctx.needs_input_grad
        need_db2 = b2 is not None and ni[4]
        need_db1 = b1 is not None and ni[2]
        _, db2 = act_grad(gy2, None, "none", need_db2,
                          db_dtype=torch.bfloat16 if need_db2 and b2.dtype == torch.bfloat16 else torch.float32)
        db1_dtype = torch.bfloat16 if need_db1 and b1.dtype == torch.bfloat16 else torch.float32
        fused = dgrad_act(gy2, w2, z1, ctx.act, need_db1, db1_dtype)
        if fused is None:
            g1, db1 = act_grad(mm(gy2, w2), z1, ctx.act, need_db1, db_dtype=db1_dtype)
        else:
            g1, db1 = fused
        gx = mm(g1, w1).reshape(ctx.xshape) if ni[0] else None
        # both weight gradients in one launch where apart they would under-fill the chip (small
        # widths: K split in-kernel, wgrad_pair); else one mm each
        pair = wgrad_pair(g1, x2, gy2, y1) if ni[1] and ni[3] else None
        if pair is not None:
            gw1, gw2 = pair
        else:
            gw1 = mm(g1, x2, trans_a=True) if ni[1] else None
            gw2 = mm(gy2, y1, trans_a=True) if ni[3] else None
        gb1 = db1.to(b1.dtype) if need_db1 else None
        gb2 = db2.to(b2.dtype) if need_db2 else None
        return gx, gw1, gb1, gw2, gb2, None, (gy if ni[6] else None)


def mlp(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor | None, w2: torch.Tensor, b2: torch.Tensor | None,
        act: str = "gelu_tanh", residual: torch.Tensor | None = None) -> torch.Tensor:
    """Autograd-aware ``F.linear(act(F.linear(x, w1, b1)), w2, b2) (+ residual)`` (act: gelu_tanh,
    silu or relu) on the MFMA kernels, fc2's dgrad fused with fc1's activation backward."""
    if act not in ("gelu", "gelu_tanh", "silu", "relu"):
        raise ValueError(f"mlp: unsupported activation {act!r}")
    if act == "relu":
        # relu's backward reads the activation output; the pre-activation form covers gelu / silu
        return linear(linear(x, w1, b1, act="relu"), w2, b2, residual=residual)
    return _MLP.apply(x, w1, b1, w2, b2, act, residual)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
           act: str = "none", residual: torch.Tensor | None = None) -> torch.Tensor:
    """Autograd-aware ``act(F.linear(x, weight, bias)) (+ residual)`` on the MFMA kernel (the
    residual rides in the GEMM epilogue when there is no activation)."""
    return _Linear.apply(x, weight, bias, act, residual)


def flops(M: int, N: int, K: int, batch: int = 1) -> float:
    return 2.0 * M * N * K * batch
