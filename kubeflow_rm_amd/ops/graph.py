"""hipGraph capture of launch-bound loops built on the framework's kernels.

Every launcher in ``kernels/`` is asynchronous on the caller's stream and never allocates, syncs or
copies (kfamd_kernels.h), so a sequence of them — a decode step, a small-batch forward — can be
captured once into a HIP graph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and replayed with a
single launch, removing the per-kernel host/ctypes overhead that dominates small shapes.
"""
from __future__ import annotations

from typing import Callable

import torch


class GraphedCallable:
    """Capture ``fn(*static_inputs)`` into a HIP graph; ``__call__(*inputs)`` copies the inputs into
    the captured buffers, replays, and returns the captured outputs (valid until the next call)."""

    def __init__(self, fn: Callable, *static_inputs: torch.Tensor, warmup: int = 2):
        self.fn = fn
        self.static_inputs = tuple(static_inputs)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm up (allocator, lazy init) off the capture
            for _ in range(warmup):
                fn(*self.static_inputs)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_out = fn(*self.static_inputs)

    def __call__(self, *inputs: torch.Tensor):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not dst:
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out
