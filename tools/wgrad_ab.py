#!/usr/bin/env python3
"""wgrad-shaped (TN: dW = gy^T x) GEMM A/B: ops.mm with the split-K plan and without split-K,
against torch. Usage: wgrad_ab.py MxNxK,..."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from kubeflow_rm_amd import ops  # noqa: E402
from kubeflow_rm_amd.ops import gemm as G  # noqa: E402


def t_us(fn, iters=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    for spec in sys.argv[1].split(","):
        M, N, K = map(int, spec.split("x"))
        gy = (torch.rand(K, M, device="cuda") * 2 - 1).to(torch.bfloat16)  # [T, out]
        x = (torch.rand(K, N, device="cuda") * 2 - 1).to(torch.bfloat16)   # [T, in]
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        cfgs = {"nosplit": False, "plan": True}

        def ours(cfg):
            G.SPLITK = cfgs[cfg]
            ops.mm(gy, x, trans_a=True, out=out)

        fns = {k: (lambda k=k: ours(k)) for k in cfgs}
        fns["torch"] = lambda: torch.matmul(gy.t(), x)
        for f in fns.values():
            f()
        res = {k: [] for k in fns}
        for _ in range(5):
            for k, f in fns.items():
                res[k].append(t_us(f))
        plans = {}
        for k, on in cfgs.items():
            G.SPLITK = on
            plans[k] = G.splitk_plan(M, N, K)
        G.SPLITK = True
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": spec, "plans": plans, **{f"{k}_us": round(min(v), 1) for k, v in res.items()},
                          **{f"{k}_tf": round(fl / min(v) / 1e6, 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
