"""Tensor parallelism (Megatron-style column/row parallel linears) on the MFMA GEMM + RCCL.

On one MI355X node every GPU pair has a direct xGMI link, so TP up to 8 is practical; with
288 GB HBM per GPU the usual reason for TP is latency (smaller per-GPU GEMMs, one all-reduce per
block) rather than capacity. Layers:

* ``ColumnParallelLinear``: weight [out/tp, in]; input replicated (identity fwd, all-reduce of
  the input gradient in bwd); output stays sharded unless ``gather_output``.
* ``RowParallelLinear``: weight [out, in/tp]; input sharded along the feature dim; the partial
  products are all-reduced in fwd (identity in bwd); bias and an optional residual are added once
  after the reduce — or, without TP, both ride in the GEMM epilogue. (Adding them on rank 0's
  partial would be cheaper, but then only rank 0's copy of the replicated residual stream would
  get its gradient.)

GPU tensors run on the hand-written gfx950 GEMM (kubeflow_rm_amd.ops.linear, fused bias +
activation epilogue). CPU tensors (gloo tests) use torch's linear — they are not a fallback for
a GPU path.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist
import torch.nn.functional as F


def _linear(x, w, b=None, act="none", residual=None):
    if x.is_cuda:
        from kubeflow_rm_amd import ops
        if ops.native_enabled():
            return ops.linear(x, w, b, act=act, residual=residual)
    y = F.linear(x, w, b)
    if act == "relu":
        y = F.relu(y)
    elif act in ("gelu", "gelu_tanh"):
        y = F.gelu(y, approximate="tanh")
    elif act == "silu":
        y = F.silu(y)
    return y + residual if residual is not None else y


# Optional K3 fast path per TP group (kubeflow_rm_amd.parallel.oneshot): the row-parallel forward
# all-reduce of a decode step is a few KB, where one one-shot kernel beats RCCL's ring steps.
_FAST: dict = {}


def enable_oneshot(group=None, max_bytes: int = 1 << 20):
    """Route this group's TP all-reduces of <= max_bytes through the one-shot IPC kernel."""
    from kubeflow_rm_amd.parallel.oneshot import IpcOneShotAllReduce
    _FAST[group] = IpcOneShotAllReduce(group, max_bytes)
    return _FAST[group]


def _all_reduce(x, group):
    fast = _FAST.get(group)
    if fast is not None and x.is_cuda:
        return fast.all_reduce(x)
    dist.all_reduce(x, group=group)
    return x


def _world(group):
    return dist.get_world_size(group) if dist.is_initialized() else 1


# KFAMD_FORCE_DIST=1 (parallel.dist.force_pg_requested): a TP group of size 1 still issues its
# all-reduces / all-gathers, so a one-GPU box runs the same RCCL calls as a TP job
def _collective(group) -> bool:
    if not dist.is_initialized():
        return False
    if dist.get_world_size(group) > 1:
        return True
    from kubeflow_rm_amd.parallel.dist import force_pg_requested
    return force_pg_requested()


def _rank(group):
    return dist.get_rank(group) if dist.is_initialized() else 0


class _CopyToTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        if _collective(ctx.group):
            g = _all_reduce(g.contiguous(), ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        if _collective(group):
            x = _all_reduce(x.contiguous(), group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        n = _world(group)
        if not _collective(group):
            return x
        parts = [torch.empty_like(x) for _ in range(n)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, dim=-1)

    @staticmethod
    def backward(ctx, g):
        n = _world(ctx.group)
        if n == 1:
            return g, None
        return g.chunk(n, dim=-1)[_rank(ctx.group)].contiguous(), None


class _ScatterToTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        n = _world(group)
        return x if n == 1 else x.chunk(n, dim=-1)[_rank(group)].contiguous()

    @staticmethod
    def backward(ctx, g):
        n = _world(ctx.group)
        if not _collective(ctx.group):
            return g, None
        parts = [torch.empty_like(g) for _ in range(n)]
        dist.all_gather(parts, g.contiguous(), group=ctx.group)
        return torch.cat(parts, dim=-1), None


def copy_to_tp(x, group=None):
    return _CopyToTP.apply(x, group)


def reduce_from_tp(x, group=None):
    return _ReduceFromTP.apply(x, group)


def gather_from_tp(x, group=None):
    return _GatherFromTP.apply(x, group)


def scatter_to_tp(x, group=None):
    return _ScatterToTP.apply(x, group)


def full_weight(full_shape, seed) -> torch.Tensor:
    """The seeded unsharded initialisation (fp32, CPU) every rank derives its shard from."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    w = torch.empty(full_shape, dtype=torch.float32)
    bound = 1.0 / math.sqrt(full_shape[1])
    return w.uniform_(-bound, bound, generator=g)


def _init_shard(full_shape, shard_dim, group, dtype, device, seed):
    """Initialise the *full* weight identically on every rank (seeded) and keep this rank's
    shard: the TP model is then numerically the same model as the unsharded one."""
    w = full_weight(full_shape, seed)
    n = _world(group)
    shard = w.chunk(n, dim=shard_dim)[_rank(group)].contiguous()
    return shard.to(dtype=dtype, device=device)


class ColumnParallelLinear(torch.nn.Module):
    def __init__(self, in_features, out_features, bias=True, gather_output=False, act="none", group=None,
                 dtype=torch.bfloat16, device=None, seed=0):
        super().__init__()
        n = _world(group)
        if out_features % n:
            raise ValueError(f"out_features={out_features} not divisible by tp={n}")
        self.group, self.gather_output, self.act = group, gather_output, act
        self.weight = torch.nn.Parameter(_init_shard((out_features, in_features), 0, group, dtype, device, seed))
        self.bias = torch.nn.Parameter(torch.zeros(out_features // n, dtype=dtype, device=device)) if bias else None

    def forward(self, x):
        y = _linear(copy_to_tp(x, self.group), self.weight, self.bias, self.act)
        return gather_from_tp(y, self.group) if self.gather_output else y


class RowParallelLinear(torch.nn.Module):
    def __init__(self, in_features, out_features, bias=True, input_is_parallel=True, group=None,
                 dtype=torch.bfloat16, device=None, seed=0):
        super().__init__()
        n = _world(group)
        if in_features % n:
            raise ValueError(f"in_features={in_features} not divisible by tp={n}")
        self.group, self.input_is_parallel = group, input_is_parallel
        self.weight = torch.nn.Parameter(_init_shard((out_features, in_features), 1, group, dtype, device, seed))
        self.bias = torch.nn.Parameter(torch.zeros(out_features, dtype=dtype, device=device)) if bias else None

    def forward(self, x, residual=None):
        if not self.input_is_parallel:
            x = scatter_to_tp(x, self.group)
        if not _collective(self.group):
            return _linear(x, self.weight, self.bias, residual=residual)
        y = reduce_from_tp(_linear(x, self.weight), self.group)
        if self.bias is not None:
            y = y + self.bias
        return y + residual if residual is not None else y
