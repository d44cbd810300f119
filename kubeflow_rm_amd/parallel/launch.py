"""Spawn N local ranks (one per GPU) from a notebook or a test — the torchrun equivalent.

``spawn(fn, nprocs, *args)`` starts ``nprocs`` fresh interpreter processes (spawn context: no
inherited HIP state), exports RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT and HSA_ENABLE_IPC_MODE_LEGACY=0, runs ``fn(rank, *args)`` in each and returns the
per-rank results in rank order; any rank failure raises in the parent.

``run_ranks(argv, nproc)`` / ``python -m kubeflow_rm_amd.parallel.launch [--nproc N] -- prog ...``
is the command-line form used inside a multi-GPU notebook pod and by ``bench.py --gpus N``: it
starts ``nproc`` child processes (never exec — the parent may not have touched the GPU, but a
child is always safe) with RANK / LOCAL_RANK set and the pod's injected rendezvous
(MASTER_ADDR / MASTER_PORT from the kubelet, a private free port otherwise), forwards their
output, and returns the first non-zero exit code; one failing rank terminates the others.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
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


def rank_env(rank: int, nproc: int, master_addr: str, master_port: int, base: dict | None = None) -> dict:
    """Environment of local rank ``rank`` of ``nproc`` (single node: RANK == LOCAL_RANK)."""
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(nproc),
                "LOCAL_WORLD_SIZE": str(nproc), "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port),
                "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    return env


def run_ranks(argv: list[str], nproc: int, master_addr: str | None = None, master_port: int | None = None,
              extra_env: dict | None = None, timeout: float | None = None, poll_s: float = 0.05) -> int:
    """Run ``argv`` as ``nproc`` local ranks; returns 0 or the first failing rank's exit code
    (124 on ``timeout``). Rendezvous: explicit args, else the pod's MASTER_ADDR / MASTER_PORT
    (per-pod values injected by the kubelet), else 127.0.0.1 and a free port."""
    addr = master_addr or os.environ.get("MASTER_ADDR") or "127.0.0.1"
    port = master_port or int(os.environ.get("MASTER_PORT") or 0) or free_port()
    procs = []
    for r in range(nproc):
        env = rank_env(r, nproc, addr, port)
        env.update(extra_env or {})
        # own process group per rank: a failure can take down the rank's whole tree
        procs.append(subprocess.Popen(argv, env=env, start_new_session=True))
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0
    try:
        live = set(range(nproc))
        while live:
            for r in sorted(live):
                code = procs[r].poll()
                if code is None:
                    continue
                live.discard(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"launch: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr)
            if rc != 0:
                break
            if deadline is not None and time.monotonic() > deadline:
                print(f"launch: timeout after {timeout}s", file=sys.stderr)
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
    return rc


def main(args: list[str] | None = None) -> int:
    import argparse
    ap = argparse.ArgumentParser(prog="python -m kubeflow_rm_amd.parallel.launch",
                                 description="run a program as N local ranks (one per GPU of this pod)")
    ap.add_argument("--nproc", type=int, default=int(os.environ.get("LOCAL_WORLD_SIZE") or 0) or None,
                    help="ranks to start (default: the pod's LOCAL_WORLD_SIZE)")
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("prog", nargs=argparse.REMAINDER)
    ns = ap.parse_args(args)
    prog = ns.prog[1:] if ns.prog and ns.prog[0] == "--" else ns.prog
    if not prog:
        ap.error("no program given")
    if prog[0].endswith(".py"):
        prog = [sys.executable, "-u"] + prog
    return run_ranks(prog, ns.nproc or 1, timeout=ns.timeout)


if __name__ == "__main__":
    sys.exit(main())
