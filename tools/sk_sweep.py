#!/usr/bin/env python3
"""Stream-K A/B: time kfamd_w4_streamk_nt at several (grid, splits) plans against the plain kernel."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from kubeflow_rm_amd.ops import gemm  # noqa: E402


def timeit(fn, iters):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    for spec in sys.argv[1].split(","):
        M, N, K = map(int, spec.split("x"))
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        plans = [(256, s) for s in (1, 2, 3, 4, 5, 8)] + [(128, 1), (512, 1)]
        fns = {"plain": lambda: gemm.gemm_nt(a, b, out=c, variant="w4")}
        for p in plans:
            fns[f"sk{p[0]}x{p[1]}"] = (lambda p=p: gemm._streamk(a, b, c, M, N, K, K, K, N, p, bias=None, r_ptr=None,
                                                                ldr=0, aux=None, alpha=1.0, act="none"))
        for f in fns.values():
            f()
        res = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                res[k].append(timeit(f, 20))
        print(json.dumps({"shape": spec, **{k: round(min(v), 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
