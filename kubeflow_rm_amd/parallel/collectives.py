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
    if not dist.is_initialized():
        raise RuntimeError("allreduce_sweep needs an initialised process group (world size 1 included)")
    world = dist.get_world_size(group)
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    esz = torch.tensor([], dtype=dtype).element_size()
    buf = torch.ones(max(max_bytes // esz, 1), dtype=dtype, device=dev)
    out = []
    nbytes = min_bytes
    while nbytes <= max_bytes:
        n = max(nbytes // esz, 1)
        x = buf[:n]
        iters = iters_small if nbytes < (1 << 20) else iters_large
        # every size runs the collective, world size 1 included: there RCCL still builds its
        # communicator and launches its kernel (a copy), so a one-GPU box exercises this exact path
        for _ in range(3):
            dist.all_reduce(x, group=group)
        _sync(dev)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x, group=group)
        _sync(dev)
        dt = (time.perf_counter() - t0) / iters
        algbw = n * esz / dt / 1e9 if dt > 0 else 0.0
        out.append({"bytes": n * esz, "us": dt * 1e6, "algbw_GBps": algbw,
                     "busbw_GBps": algbw * 2 * (world - 1) / world if world > 1 else 0.0})
        nbytes *= step
    return out


def fast_allreduce_sweep(sizes: list[int], algo: str, dtype=torch.bfloat16, iters: int = 20, group=None) -> list[dict]:
    """The hand-written IPC all-reduce (``algo`` = "oneshot" / "twoshot", kernels/allreduce_oneshot.hip)
    over the group's GPUs, one process per GPU; same algbw / busbw convention as ``allreduce_sweep``.
    Every result is checked against the exact rank-order sum of a known pattern."""
    from .oneshot import IpcOneShotAllReduce, OneShotTimeout, agree
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    esz = torch.tensor([], dtype=dtype).element_size()
    ar = IpcOneShotAllReduce(group=group, max_bytes=max(sizes))
    out = []
    try:
        for nbytes in sizes:
            n = max(nbytes // esz, 1)
            x = torch.full((n,), float(rank + 1), dtype=dtype, device=dev)
            err = None
            try:
                ar(x, algo=algo)
                _sync(dev)
                want = world * (world + 1) / 2
                correct = bool(torch.all(x == want).item())
                for _ in range(3):
                    ar(x, algo=algo)
                _sync(dev)
                ar.check()
            except OneShotTimeout as e:
                err = e
            # every rank leaves the sweep at the same size when any rank timed out (a rank raising
            # alone would leave the others in the next barrier)
            if not agree(err is None, group):
                out.append({"bytes": n * esz, "error": f"{type(err).__name__}: {err}" if err else "timeout on a peer rank"})
                break
            dist.barrier(group=group)
            t0 = time.perf_counter()
            for _ in range(iters):
                ar(x, algo=algo)
            _sync(dev)
            dt = (time.perf_counter() - t0) / iters
            ok_t = not ar.timed_out()
            algbw = n * esz / dt / 1e9
            out.append({"bytes": n * esz, "us": round(dt * 1e6, 1), "algbw_GBps": round(algbw, 1),
                        "busbw_GBps": round(algbw * 2 * (world - 1) / world, 1), "correct": correct and ok_t})
            if not agree(ok_t, group):
                break
    finally:
        ar.close()
    return out


def xgmi_probe(nbytes: int = 256 << 20, iters: int = 5, group=None) -> dict:
    """Peer-copy bandwidth between the group's GPUs (the per-link xGMI ceiling the
    collectives' busbw is judged against; spec 153 GB/s per link, 7 links per MI355X).

    Each rank registers ``nbytes`` of device memory for HIP IPC and maps every peer's buffer. Phase 1
    times one ordered pair at a time (rank s writes its buffer into rank d's with a stream-ordered
    D2D copy while every other rank waits): the single-link rate. Phase 2 has every rank write to all
    peers at once (one stream per peer): per-GPU egress with all links busy. Returns GB/s figures
    (10^9 B/s) plus the pair matrix."""
    import ctypes
    from kubeflow_rm_amd.ops import _lib
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    L = _lib.lib()
    own = ctypes.c_void_p()
    h = ctypes.create_string_buffer(64)
    _lib.check(L.kfamd_ipc_alloc(nbytes, 0, ctypes.byref(own), h), "kfamd_ipc_alloc")
    handles: list = [None] * world
    dist.all_gather_object(handles, h.raw, group=group)
    peers: dict[int, int] = {}
    try:
        from .oneshot import agree
        err = None
        try:
            for r in range(world):
                if r != rank:
                    p = ctypes.c_void_p()
                    _lib.check(L.kfamd_ipc_open(handles[r], ctypes.byref(p)), f"kfamd_ipc_open(rank {r})")
                    peers[r] = p.value
        except RuntimeError as e:
            err = e
        if not agree(err is None, group):  # every rank gives up together (the finally's barrier matches)
            raise err if err is not None else RuntimeError("xgmi_probe: a peer rank could not map the IPC buffers")
        src = torch.empty(nbytes, dtype=torch.uint8, device=dev).fill_(rank + 1)
        streams = {r: torch.cuda.Stream(dev) for r in peers}
        dist.barrier(group=group)

        def copy(dst_rank, stream):
            _lib.check(L.kfamd_copy_async(peers[dst_rank], src.data_ptr(), nbytes, stream.cuda_stream),
                       "kfamd_copy_async")

        pair = [[0.0] * world for _ in range(world)]
        for s in range(world):
            for d in range(world):
                if s == d:
                    continue
                dist.barrier(group=group)
                if rank == s:
                    st = streams[d]
                    copy(d, st)  # warm the path (first-touch mappings)
                    st.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(iters):
                        copy(d, st)
                    st.synchronize()
                    pair[s][d] = nbytes * iters / (time.perf_counter() - t0) / 1e9
        rows: list = [None] * world
        dist.all_gather_object(rows, pair[rank], group=group)
        for s in range(world):
            pair[s] = rows[s]
        # phase 2: every rank to every peer at once
        dist.barrier(group=group)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            for d, st in streams.items():
                copy(d, st)
        for st in streams.values():
            st.synchronize()
        egress = nbytes * iters * len(peers) / (time.perf_counter() - t0) / 1e9
        eg: list = [None] * world
        dist.all_gather_object(eg, egress, group=group)
        dist.barrier(group=group)
        vals = sorted(v for s in range(world) for d, v in enumerate(pair[s]) if s != d)
        return {"bytes": nbytes, "iters": iters, "pair_GBps": [[round(v, 1) for v in row] for row in pair],
                "pair_GBps_min": round(vals[0], 1) if vals else None,
                "pair_GBps_median": round(vals[len(vals) // 2], 1) if vals else None,
                "pair_GBps_max": round(vals[-1], 1) if vals else None,
                "all_pairs_egress_GBps_per_gpu": [round(v, 1) for v in eg],
                "spec_link_GBps": 153.0,
                "note": "hipMemcpyAsync D2D into an IPC-mapped peer buffer; pair = one link at a time"}
    finally:
        torch.cuda.synchronize(dev)
        dist.barrier(group=group)
        for p in peers.values():
            L.kfamd_ipc_close(p)
        L.kfamd_ipc_free(own.value)
