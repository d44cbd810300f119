"""K3 fast path for torch.distributed ranks (one process per GPU): one-shot all-reduce over HIP IPC.

Each rank registers an input buffer and a flag array (``kfamd_ipc_alloc``), the 64-byte IPC handles
are exchanged once over the process group, and every rank maps its peers' buffers
(``kfamd_ipc_open``). A call then copies the tensor into the rank's own buffer and launches
``kernels/allreduce_oneshot.hip`` on the current stream: every rank reads all peers over xGMI and
writes the sum into the tensor. For the latency-bound sizes of TP decode / small DP buckets this
replaces RCCL's 2(N-1) ring steps with one kernel. Mid-size tensors (``TWOSHOT_MIN_BYTES`` up to the
registered size) take the two-shot kernel: reduce-scatter + all-gather in one launch, every rank
pulling its slice from all peers at once (all xGMI links busy; 2(N-1)/N of the bytes instead of
N-1). :func:`all_reduce` routes larger tensors to ``torch.distributed.all_reduce`` (RCCL).

Failure model: the kernel's barriers wait at most ``timeout_ms`` (wall clock) for a peer. A missed
deadline NaN-poisons that call's output and sets a device flag; the flag protocol is then out of
step between ranks, so a timeout is fatal for this communicator. The flag is read back every
``check_every`` calls (one tiny D2H copy, so the hot path stays asynchronous) and by
:meth:`check`; once seen, every later call raises :class:`OneShotTimeout` — results between the
timeout and the check are NaN, never silently wrong. Re-create the object (collectively) to
recover.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from kubeflow_rm_amd.ops import _lib
from kubeflow_rm_amd.ops.allreduce import pick_algo

_DTYPES = {torch.float32: 0, torch.bfloat16: 1}
MAX_BLOCKS = 64


def agree(ok: bool, group=None) -> bool:
    """True on every rank iff ``ok`` on every rank (one tiny all-reduce; on the device for RCCL)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return ok
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


class OneShotTimeout(RuntimeError):
    """A peer missed the one-shot barrier deadline; this communicator is unusable."""


class IpcOneShotAllReduce:
    def __init__(self, group=None, max_bytes: int = 1 << 20, timeout_ms: int = 5000, check_every: int = 64):
        self.group = group
        self.timeout_ms, self.check_every = timeout_ms, max(1, check_every)
        self.broken = False
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if not 1 <= self.world <= 8:
            raise ValueError("one-shot all-reduce serves 1..8 ranks (one xGMI hive)")
        self.max_bytes = max_bytes
        L = _lib.lib()
        L.kfamd_allreduce_oneshot_set_timeout_ms(int(timeout_ms))
        fbytes = L.kfamd_allreduce_oneshot_flag_bytes(self.world, MAX_BLOCKS)
        self._own: list[int] = []
        mine = []
        for nbytes, uncached in ((max_bytes, 0), (fbytes, 1)):
            p = ctypes.c_void_p()
            h = ctypes.create_string_buffer(64)
            _lib.check(L.kfamd_ipc_alloc(nbytes, uncached, ctypes.byref(p), h), "kfamd_ipc_alloc")
            self._own.append(p.value)
            mine.append(h.raw)
        handles: list = [None] * self.world
        dist.all_gather_object(handles, mine, group=group)
        self._opened: list[int] = []
        bufs, flags = [], []
        err = None
        try:
            for r, (hb, hf) in enumerate(handles):
                if r == self.rank:
                    bufs.append(self._own[0])
                    flags.append(self._own[1])
                    continue
                pb, pf = ctypes.c_void_p(), ctypes.c_void_p()
                _lib.check(L.kfamd_ipc_open(hb, ctypes.byref(pb)), f"kfamd_ipc_open(buffer of rank {r})")
                self._opened.append(pb.value)
                _lib.check(L.kfamd_ipc_open(hf, ctypes.byref(pf)), f"kfamd_ipc_open(flags of rank {r})")
                self._opened.append(pf.value)
                bufs.append(pb.value)
                flags.append(pf.value)
        except RuntimeError as e:
            err = e
        # collective outcome: a rank that could not map a peer must not leave the others waiting in
        # the kernel's barrier or in the next collective; every rank raises together
        if not agree(err is None, group):
            self.close()
            raise err if err is not None else RuntimeError(f"one-shot all-reduce: a peer of rank {self.rank} "
                                                           "could not map the IPC buffers")
        arr = ctypes.c_void_p * 8
        self._in = arr(*bufs)
        self._flags = arr(*flags)
        self._out = arr(*([0] * 8))
        self.timeout = torch.zeros(1, dtype=torch.int32, device="cuda")
        self.epoch = 0
        dist.barrier(group=group)  # every rank mapped its peers before the first call

    def __call__(self, t: torch.Tensor, algo: str = "auto") -> torch.Tensor:
        """In-place sum of ``t`` (contiguous fp32 / bf16 CUDA tensor) over the group. ``algo``:
        "oneshot", "twoshot" or "auto" (by size; every rank must pick the same one)."""
        if t.dtype not in _DTYPES or not t.is_cuda or not t.is_contiguous():
            raise ValueError("contiguous fp32/bf16 CUDA tensor expected")
        nbytes = t.numel() * t.element_size()
        if nbytes > self.max_bytes:
            raise ValueError(f"{nbytes} B > registered {self.max_bytes} B (use RCCL)")
        if self.broken:
            raise OneShotTimeout(f"one-shot all-reduce (rank {self.rank}) timed out earlier; re-create it")
        L = _lib.lib()
        stream = torch.cuda.current_stream(t.device).cuda_stream
        # own registered input buffer <- t, stream-ordered before the kernel (whose entry barrier
        # publishes it to the peers); the result is written straight into t
        _lib.check(L.kfamd_copy_async(self._own[0], t.data_ptr(), nbytes, stream), "kfamd_copy_async")
        self.epoch += 1
        self._out[self.rank] = t.data_ptr()
        dt = _DTYPES[t.dtype]
        algo = pick_algo(nbytes, self.world, algo)
        if algo == "twoshot":  # reduces in place in the registered buffers, gathers into t
            fn, nb = L.kfamd_allreduce_twoshot, L.kfamd_allreduce_twoshot_blocks(t.numel(), dt, self.world)
        else:
            fn, nb = L.kfamd_allreduce_oneshot, L.kfamd_allreduce_oneshot_blocks(t.numel(), dt)
        nb = min(MAX_BLOCKS, nb)
        rc = fn(self._in, self._out, self._flags, self.world, self.rank, 1, t.numel(), dt,
                self.epoch, nb, self.timeout.data_ptr(), stream)
        _lib.check(rc, f"allreduce_{algo}[rank {self.rank}/{self.world}, {t.numel()}]")
        if self.epoch % self.check_every == 0:
            self.check()
        return t

    def timed_out(self) -> bool:
        return bool(self.timeout.item())

    def check(self) -> None:
        """Raise :class:`OneShotTimeout` if any call so far missed a peer (synchronises the stream)."""
        if self.broken or self.timed_out():
            self.broken = True
            raise OneShotTimeout(f"one-shot all-reduce: a peer of rank {self.rank} missed the "
                                 f"{self.timeout_ms} ms barrier deadline; outputs since the last check are NaN")

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """One-shot for registered-size fp32/bf16 tensors, RCCL (torch.distributed) otherwise."""
        if t.dtype in _DTYPES and t.is_contiguous() and t.numel() * t.element_size() <= self.max_bytes:
            return self(t)
        dist.all_reduce(t, group=self.group)
        return t

    def close(self) -> None:
        L = _lib.lib()
        torch.cuda.synchronize()
        if not getattr(self, "_own", None):
            return
        for p in self._opened:
            L.kfamd_ipc_close(p)
        for p in self._own:
            L.kfamd_ipc_free(p)
        self._opened, self._own = [], []
