#!/usr/bin/env python3
"""Flash attention A/B: the in-tree gfx950 kernels (ops.flash_attention) vs torch SDPA (aotriton)
on the same random bf16 inputs, interleaved rounds in one process (cdna_hip_programming.md §5.4
rule 24). Prints one JSON line per (shape, pass) with medians in µs and TFLOP/s.

Causal FLOPs: fwd 4·B·H·T²·D / 2, bwd 2.5× that (five products with recompute of S: 10·B·H·T²·D/2).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

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
    p = argparse.ArgumentParser()
    p.add_argument("--shapes", default="4x16x2048x128,16x12x2048x64,1x16x4096x128")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--no-causal", action="store_true")
    a = p.parse_args()
    causal = not a.no_causal
    for shp in a.shapes.split(","):
        B, H, T, D = map(int, shp.split("x"))
        g = torch.Generator(device="cuda").manual_seed(0)
        q, k, v, do = (torch.randn(B, H, T, D, device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
        qs, ks, vs = (x.clone().requires_grad_(True) for x in (q, k, v))
        fl = 4.0 * B * H * T * T * D * (0.5 if causal else 1.0)

        def ours_f():
            return ops.flash_attention(qs, ks, vs, causal=causal)

        def sdpa_f():
            return F.scaled_dot_product_attention(qs, ks, vs, is_causal=causal)

        o1, o2 = ours_f(), sdpa_f()

        def ours_b():
            torch.autograd.grad(o1, (qs, ks, vs), do, retain_graph=True)

        def sdpa_b():
            torch.autograd.grad(o2, (qs, ks, vs), do, retain_graph=True)

        res = {"fwd": ([], []), "bwd": ([], [])}
        for f in (ours_f, sdpa_f, ours_b, sdpa_b):
            timeit(f, 2)
        for _ in range(a.rounds):
            res["fwd"][0].append(timeit(ours_f, a.iters))
            res["fwd"][1].append(timeit(sdpa_f, a.iters))
            res["bwd"][0].append(timeit(ours_b, a.iters))
            res["bwd"][1].append(timeit(sdpa_b, a.iters))
        for ph, (ours, theirs) in res.items():
            f = fl * (2.5 if ph == "bwd" else 1.0)
            mo, mt = statistics.median(ours), statistics.median(theirs)
            print(json.dumps({"shape": shp, "causal": causal, "pass": ph, "ours_us": round(mo, 1),
                              "sdpa_us": round(mt, 1), "ours_tflops": round(f / mo / 1e6, 1),
                              "sdpa_tflops": round(f / mt / 1e6, 1), "speedup": round(mt / mo, 3),
                              "ours_all": [round(x, 1) for x in ours], "sdpa_all": [round(x, 1) for x in theirs]}),
                  flush=True)


if __name__ == "__main__":
    main()
