"""Spawn N local ranks (one per GPU) from a notebook or a test — the torchrun equivalent.

``spawn(fn, nprocs, *args)`` starts ``nprocs`` fresh interpreter processes (spawn context: no
inherited HIP state), exports RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT and HSA_ENABLE_IPC_MODE_LEGACY=0, runs ``fn(rank, *args)`` in each and returns the
per-rank results in rank order; any rank failure raises in the parent.
"""
from __future__ import annotations

import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _to_host(v):
    import torch
    if isinstance(v, torch.Tensor):
        return v.detach().float().cpu().numpy() if v.dtype == torch.bfloat16 else v.detach().cpu().numpy()
    if isinstance(v, dict):
        return {k: _to_host(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return type(v)(_to_host(x) for x in v)
    return v


def _entry(rank, world, port, fn, args, q, extra_env):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    os.environ.update(extra_env or {})
    try:
        # tensors go back as numpy (a torch tensor would travel as a shared-memory handle that
        # dies with this process)
        q.put((rank, True, _to_host(fn(rank, *args))))
    except BaseException:  # noqa: BLE001 - reported to the parent
        q.put((rank, False, traceback.format_exc()))


def spawn(fn, nprocs: int, *args, env: dict | None = None, timeout: float = 600.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, nprocs, port, fn, args, q, env)) for r in range(nprocs)]
    for p in procs:
        p.start()
    results: dict[int, object] = {}
    errors = []
    try:
        for _ in range(nprocs):
            rank, ok, val = q.get(timeout=timeout)
            if ok:
                results[rank] = val
            else:
                errors.append(f"rank {rank}:\n{val}")
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    if errors:
        raise RuntimeError("\n".join(errors))
    return [results[r] for r in range(nprocs)]
