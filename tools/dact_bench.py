#!/usr/bin/env python3
"""fc2 dgrad + fc1 activation backward at an MLP shape: the fused GEMM epilogue (ops.dgrad_act) vs
mm + act_grad, interleaved rounds, medians in µs. python tools/dact_bench.py --shape 8192x2048x8192
(M tokens x fc2 out x fc2 in)."""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    from kubeflow_rm_amd import ops
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8192x2048x8192,32768x768x3072")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--preact", default="8192x8192x2048,32768x3072x768",
                    help="MxNxK: the forward GEMM with bias + gelu + pre-activation output vs bias only")
    ap.add_argument("--res", default="8192x2048x2048,8192x2048x8192",
                    help="MxNxK: the forward GEMM with bias + residual epilogue vs bias only")
    a = ap.parse_args()
    for shp in [x for x in a.shapes.split(",") if x]:
        M, K, N = map(int, shp.split("x"))
        g = torch.Generator(device="cuda").manual_seed(0)
        gy = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        w = (torch.randn(K, N, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
        z = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
        fused = lambda: ops.dgrad_act(gy, w, z, "gelu_tanh", True, torch.bfloat16)  # noqa: E731
        fused_nodb = lambda: ops.dgrad_act(gy, w, z, "gelu_tanh", False)  # noqa: E731
        split = lambda: ops.act_grad(ops.mm(gy, w), z, "gelu_tanh", True, torch.bfloat16)  # noqa: E731
        gemm = lambda: ops.mm(gy, w)  # noqa: E731
        fns = {"fused": fused, "fused_nodb": fused_nodb, "split": split, "gemm_only": gemm}
        for f in fns.values():
            timeit(f, 2)
        res = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                res[k].append(timeit(f, a.iters))
        print(json.dumps({"shape": shp, **{k + "_us": round(statistics.median(v), 1) for k, v in res.items()}}),
              flush=True)

    for shp in [x for x in a.preact.split(",") if x]:
        M, N, K = map(int, shp.split("x"))
        g = torch.Generator(device="cuda").manual_seed(2)
        x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
        b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
        fns = {"gelu_preact": lambda: ops.gemm_nt_preact(x, w, b, "gelu_tanh"), "bias": lambda: ops.gemm_nt(x, w, bias=b)}
        for f in fns.values():
            timeit(f, 2)
        res = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                res[k].append(timeit(f, a.iters))
        print(json.dumps({"preact": shp, **{k + "_us": round(statistics.median(v), 1) for k, v in res.items()}}),
              flush=True)
    for shp in [x for x in a.res.split(",") if x]:
        M, N, K = map(int, shp.split("x"))
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
        b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
        r = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
        fns = {"bias_res": lambda: ops.gemm_nt(x, w, bias=b, residual=r), "bias": lambda: ops.gemm_nt(x, w, bias=b)}
        for f in fns.values():
            timeit(f, 2)
        res = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                res[k].append(timeit(f, a.iters))
        print(json.dumps({"gemm": shp, **{k + "_us": round(statistics.median(v), 1) for k, v in res.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
