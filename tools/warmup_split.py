#!/usr/bin/env python3
"""Fine split of the torch-ready warmup's first-GEMM phase (one fresh process)."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    T = {}
    t = time.perf_counter()
    from kubeflow_rm_amd.images.notebook_server import _preinit_hip
    pre = _preinit_hip()
    import torch
    T["import_torch"] = time.perf_counter() - t
    t = time.perf_counter()
    if pre is not None:
        pre.join()
    T["preinit_join"] = time.perf_counter() - t
    t = time.perf_counter()
    from kubeflow_rm_amd import ops
    ops.lib()
    T["ops_lib_dlopen"] = time.perf_counter() - t
    t = time.perf_counter()
    torch.cuda.init()
    T["torch_cuda_init"] = time.perf_counter() - t
    t = time.perf_counter()
    dev = torch.device("cuda", 0)
    x = torch.empty(1024, 1024, dtype=torch.bfloat16, device=dev)
    T["first_alloc"] = time.perf_counter() - t
    import os
    if os.environ.get("GEMM_FIRST") == "1":  # our kernel before any copy: which one pays the ~100 ms?
        t = time.perf_counter()
        c = ops.gemm_nt(x, x)
        torch.cuda.synchronize()
        T["gemm_on_empty"] = time.perf_counter() - t
    t = time.perf_counter()
    ha = torch.rand(1024, 1024).to(torch.bfloat16)
    a = ha.to(dev)
    torch.cuda.synchronize()
    T["h2d"] = time.perf_counter() - t
    t = time.perf_counter()
    c = ops.gemm_nt(a, a)
    torch.cuda.synchronize()
    T["first_gemm"] = time.perf_counter() - t
    t = time.perf_counter()
    c = ops.gemm_nt(a, a)
    torch.cuda.synchronize()
    T["second_gemm"] = time.perf_counter() - t
    t = time.perf_counter()
    c.cpu()
    T["d2h"] = time.perf_counter() - t
    print(json.dumps({k: round(v * 1e3, 1) for k, v in T.items()}), flush=True)


if __name__ == "__main__":
    main()
