"""K3 small-message all-reduce on the hand-written one-shot kernel (kernels/allreduce_oneshot.hip).

One kernel per rank reads every peer's registered buffer over xGMI and sums it (fp32, rank order,
so every rank's result is bit-identical); two block-pair flag barriers replace RCCL's 2(N-1) ring
hops, which is what bounds a KB-sized all-reduce. Mid-size messages take the two-shot kernel
(reduce-scatter + all-gather in one launch: 2(N-1)/N of the bytes per rank instead of N-1, pulled
from all peers at once so every xGMI link carries traffic). ``algo="auto"`` switches at
``TWOSHOT_MIN_BYTES``.

:class:`OneShotAllReduce` owns the registered buffers for a set of ranks that this process can
address: several devices of one process (peer access, the readiness op's layout) or, for tests on
a single GPU, several simulated ranks on one device, all served by ONE launch.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .gemm import _stream_ptr

_DTYPES = {torch.float32: 0, torch.bfloat16: 1}
TWOSHOT_MIN_BYTES = 256 << 10


def pick_algo(nbytes: int, nranks: int, algo: str = "auto") -> str:
    if algo != "auto":
        return algo
    return "twoshot" if nranks > 2 and nbytes >= TWOSHOT_MIN_BYTES else "oneshot"


class OneShotAllReduce:
    """Registered input/output/flag buffers for ``nranks`` ranks of up to ``max_numel`` elements.

    ``devices``: one device per rank (real peer ranks; peer access must be enabled between them)
    or a single device for every rank (simulation: the whole collective is one launch).
    """

    def __init__(self, nranks: int, max_numel: int, dtype: torch.dtype = torch.bfloat16,
                 devices: list[torch.device] | None = None):
        if not 1 <= nranks <= 8:
            raise ValueError("1..8 ranks")
        if dtype not in _DTYPES:
            raise ValueError(f"dtype {dtype}")
        self.nranks, self.max_numel, self.dtype = nranks, max_numel, dtype
        devs = devices or [torch.device("cuda", torch.cuda.current_device())]
        self.devices = devs if len(devs) == nranks else [devs[0]] * nranks
        self.simulated = len(set(self.devices)) == 1 and nranks > 1
        L = _lib.lib()
        self.max_blocks = 64
        fbytes = L.kfamd_allreduce_oneshot_flag_bytes(nranks, self.max_blocks)
        self.inputs = [torch.empty(max_numel, dtype=dtype, device=d) for d in self.devices]
        self.outputs = [torch.empty(max_numel, dtype=dtype, device=d) for d in self.devices]
        self.flags = [torch.zeros(fbytes // 4, dtype=torch.int32, device=d) for d in self.devices]
        self.timeout = [torch.zeros(1, dtype=torch.int32, device=d) for d in self.devices]
        self.epoch = 0
        arr = ctypes.c_void_p * 8
        self._in = arr(*[t.data_ptr() for t in self.inputs])
        self._out = arr(*[t.data_ptr() for t in self.outputs])
        self._flags = arr(*[t.data_ptr() for t in self.flags])

    def __call__(self, tensors: list[torch.Tensor], algo: str = "auto") -> list[torch.Tensor]:
        """All-reduce ``tensors`` (one per rank, same numel); returns views of the outputs.
        ``algo``: "oneshot", "twoshot" or "auto" (by message size)."""
        if len(tensors) != self.nranks:
            raise ValueError("one tensor per rank")
        n = tensors[0].numel()
        if n > self.max_numel or any(t.numel() != n or t.dtype != self.dtype for t in tensors):
            raise ValueError("shape/dtype mismatch")
        for r, t in enumerate(tensors):
            self.inputs[r][:n].copy_(t.reshape(-1), non_blocking=True)
        self.epoch += 1
        L = _lib.lib()
        dt = _DTYPES[self.dtype]
        algo = pick_algo(n * tensors[0].element_size(), self.nranks, algo)
        if algo == "twoshot":
            fn, nb = L.kfamd_allreduce_twoshot, L.kfamd_allreduce_twoshot_blocks(n, dt, self.nranks)
        elif algo == "oneshot":
            fn, nb = L.kfamd_allreduce_oneshot, L.kfamd_allreduce_oneshot_blocks(n, dt)
        else:
            raise ValueError(f"algo {algo}")
        nb = min(self.max_blocks, nb)
        self.last_algo = algo
        if self.simulated:
            rc = fn(self._in, self._out, self._flags, self.nranks, 0, self.nranks, n, dt,
                    self.epoch, nb, self.timeout[0].data_ptr(), _stream_ptr(tensors[0]))
            _lib.check(rc, f"allreduce_{algo}[{self.nranks}x{n}]")
        else:
            # inputs are copied on each device's current stream; the kernels then run concurrently,
            # one per device, meeting at the flag barriers
            for r, d in enumerate(self.devices):
                with torch.cuda.device(d):
                    rc = fn(self._in, self._out, self._flags, self.nranks, r, 1, n, dt,
                            self.epoch, nb, self.timeout[r].data_ptr(), torch.cuda.current_stream(d).cuda_stream)
                _lib.check(rc, f"allreduce_{algo}[rank {r}/{self.nranks}x{n}]")
        return [o[:n].view(tensors[r].shape) for r, o in enumerate(self.outputs)]

    def timed_out(self) -> bool:
        return any(int(t.item()) != 0 for t in self.timeout)
