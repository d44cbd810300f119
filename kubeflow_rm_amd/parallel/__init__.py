"""Multi-GPU wiring for notebooks: one process per MI355X, RCCL (backend "nccl") over xGMI.

* :mod:`.dist` — process-group bring-up from the env the pod spec injects (xGMI ring order).
* :mod:`.dp` — bucketed gradient all-reduce overlapped with backward.
* :mod:`.tp` — column/row parallel linears on the hand-written MFMA GEMM.
* :mod:`.collectives` — all-reduce bandwidth sweep (busbw).
* :mod:`.oneshot` — K3 one-shot all-reduce over HIP IPC for small messages (``tp.enable_oneshot``).
* :mod:`.launch` — spawn N local ranks (torchrun-equivalent for notebooks / tests).
"""
from .collectives import allreduce_sweep  # noqa: F401
from .dist import DistEnv, barrier, device_for_local_rank, env, init, shutdown, xgmi_ring  # noqa: F401
from .dp import DataParallel, GradBucketer  # noqa: F401
from .tp import (ColumnParallelLinear, RowParallelLinear, copy_to_tp, enable_oneshot,  # noqa: F401
                 gather_from_tp, reduce_from_tp, scatter_to_tp)
