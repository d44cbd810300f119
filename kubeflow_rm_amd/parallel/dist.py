"""Process-group bring-up for multi-GPU notebooks (one process per GPU, RCCL over xGMI).

The notebook pod spec carries the wiring (injected by the kubelet's device plugin allocation,
native/gpu/topology.cc gpu_env_for): HIP_VISIBLE_DEVICES (pod-local ordinals 0..n-1),
KFAMD_XGMI_RING (ring order over direct xGMI links), WORLD_SIZE / LOCAL_WORLD_SIZE,
MASTER_ADDR / MASTER_PORT (the pod's own rendezvous endpoint: its 127.x address and a port
unique on the node, so concurrent multi-GPU notebooks never share a TCPStore), NCCL_IB_DISABLE=1, NCCL_P2P_LEVEL=SYS,
HSA_ENABLE_IPC_MODE_LEGACY=0. ``torchrun`` (or this module's ``spawn``) supplies RANK/LOCAL_RANK.

``init()`` maps LOCAL_RANK to the device at position LOCAL_RANK of the xGMI ring, so that ring
neighbours in RCCL's rank order are physically adjacent on the fabric (each hop is one direct
xGMI link; on a fully-connected 8x MI355X node every order is a ring, but on partial fabrics or
GPU subsets this keeps the collective on direct links).
"""
from __future__ import annotations

import datetime as _dt
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "gloo"

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_ENV: DistEnv | None = None


def xgmi_ring() -> list[int]:
    ring = os.environ.get("KFAMD_XGMI_RING", "")
    try:
        return [int(x) for x in ring.split(",") if x != ""]
    except ValueError:
        return []


def device_for_local_rank(local_rank: int) -> int:
    ring = xgmi_ring()
    if ring and local_rank < len(ring):
        return ring[local_rank]
    return local_rank


def force_pg_requested() -> bool:
    """``KFAMD_FORCE_DIST=1``: bring up the process group even at WORLD_SIZE=1, so a one-GPU run
    executes the same RCCL code (communicator init, barriers, bucketed all-reduces) as an N-GPU job."""
    return os.environ.get("KFAMD_FORCE_DIST", "") not in ("", "0")


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def init(backend: str | None = None, timeout_s: float = 600.0, force_pg: bool | None = None) -> DistEnv:
    """Initialise torch.distributed from the env (idempotent). backend: nccl (=RCCL on ROCm) when
    GPUs are visible, else gloo. ``force_pg`` (default: ``KFAMD_FORCE_DIST``) creates the process
    group at world size 1 too (a private 127.0.0.1 port is picked when MASTER_PORT is unset: no other
    rank can meet it there)."""
    global _ENV
    if _ENV is not None:
        return _ENV
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    device = torch.device("cpu")
    if use_gpu:
        dev = device_for_local_rank(local_rank) % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev)
        device = torch.device("cuda", dev)
    if force_pg is None:
        force_pg = force_pg_requested()
    if (world > 1 or force_pg) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and not os.environ.get("MASTER_PORT"):
            os.environ["MASTER_PORT"] = str(_free_port())
        if not os.environ.get("MASTER_PORT"):
            # no silent shared default: two jobs on one host would meet in the same TCPStore
            raise RuntimeError("WORLD_SIZE > 1 but MASTER_PORT is unset: run under torchrun, "
                               "kubeflow_rm_amd.parallel.launch, or a multi-GPU notebook pod (injected env)")
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, timeout=_dt.timedelta(seconds=timeout_s), **kw)
    _ENV = DistEnv(rank=rank, world_size=world, local_rank=local_rank, device=device, backend=backend)
    return _ENV


def env() -> DistEnv:
    return _ENV if _ENV is not None else DistEnv()


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        if env().backend == "nccl":
            dist.barrier(device_ids=[env().device.index])
        else:
            dist.barrier()


def shutdown() -> None:
    global _ENV
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _ENV = None
