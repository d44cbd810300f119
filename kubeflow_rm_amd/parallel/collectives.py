"""RCCL collective micro-benchmarks over xGMI (K3 of the readiness ops, multi-process form).

``allreduce_sweep`` times ``dist.all_reduce`` for message sizes 8 B .. max_bytes (x8 steps) and
reports algorithm and bus bandwidth (busbw = algbw * 2(n-1)/n, the nccl-tests convention), so the
number is comparable across world sizes and with the per-link xGMI ceiling.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def allreduce_sweep(max_bytes: int = 256 << 20, min_bytes: int = 8, step: int = 8, iters_small: int = 50,
                    iters_large: int = 10, dtype=torch.float32, device=None, group=None) -> list[dict]:
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    esz = torch.tensor([], dtype=dtype).element_size()
    buf = torch.ones(max(max_bytes // esz, 1), dtype=dtype, device=dev)
    out = []
    nbytes = min_bytes
    while nbytes <= max_bytes:
        n = max(nbytes // esz, 1)
        x = buf[:n]
        iters = iters_small if nbytes < (1 << 20) else iters_large
        for _ in range(3):
            if world > 1:
                dist.all_reduce(x, group=group)
        _sync(dev)
        if world > 1:
            dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(iters):
            if world > 1:
                dist.all_reduce(x, group=group)
        _sync(dev)
        dt = (time.perf_counter() - t0) / iters
        algbw = n * esz / dt / 1e9 if dt > 0 else 0.0
        out.append({"bytes": n * esz, "us": dt * 1e6, "algbw_GBps": algbw,
                     "busbw_GBps": algbw * 2 * (world - 1) / world if world > 1 else 0.0})
        nbytes *= step
    return out
