#!/usr/bin/env python3
"""Split-K fixup A/B (gemm_w4.h SPLIT == 2) on wgrad-shaped problems (dW = gy^T x, mm trans_a):
the previous plan (FIXK off: the 128 tile, or the 128-tile split-K + reduce), the fixup at each
forced split count, and torch (hipBLASLt). Hot: 20 back-to-back calls on cache-resident operands;
cold: each call after a 512 MiB write that evicts L2 and MALL, timed alone (median of 20).

  python tools/fixk_ab.py 2048x2048x8192,3072x768x32768 --splits 2,3,4,6,8
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from kubeflow_rm_amd import ops  # noqa: E402
from kubeflow_rm_amd.ops import gemm as G  # noqa: E402


def hot_us(fn, iters=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def cold_us(fn, flush, iters=20):
    ts = []
    for _ in range(iters):
        flush.add_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes")
    ap.add_argument("--splits", default="2,3,4,6,8")
    a = ap.parse_args()
    flush = torch.zeros(128 * 1024 * 1024, dtype=torch.float32, device="cuda")
    for spec in a.shapes.split(","):
        M, N, K = map(int, spec.split("x"))
        gy = (torch.rand(K, M, device="cuda") * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(K, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = None
        cfgs = {"prev": (False, None)}
        for s in [int(v) for v in a.splits.split(",") if v]:
            if (K // 64) // s >= 4:
                cfgs[f"fix{s}"] = (True, s)
        cfgs["plan"] = (True, None)

        def ours(k):
            G.FIXK, G.FIXK_SPLITS = cfgs[k]
            ops.mm(gy, x, trans_a=True, out=out)

        res, same = {}, {}
        for k in cfgs:
            ours(k)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            same[k] = round((out.float() - ref).abs().max().item(), 4)
        fns = {k: (lambda k=k: ours(k)) for k in cfgs}
        fns["torch"] = lambda: torch.matmul(gy.t(), x)
        for k, f in fns.items():
            res[k] = {"hot": round(min(hot_us(f) for _ in range(3)), 1), "cold": round(cold_us(f, flush), 1)}
        G.FIXK, G.FIXK_SPLITS = True, None
        print(json.dumps({"shape": spec, "plan_now": G.fixk_plan(M, N, K), "max_diff_vs_prev": same, "us": res}),
              flush=True)
        del gy, x, out


if __name__ == "__main__":
    main()
