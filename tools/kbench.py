#!/usr/bin/env python3
"""Kernel micro-benchmarks on one GPU: GEMM TFLOPS sweep (ours vs torch/hipBLASLt), LayerNorm GB/s.

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24); random operands.
Prints one JSON line per measurement; --out writes them to a file as well.
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(fn, iters, dev):
    import torch
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,2048,4096,8192,16384")
    ap.add_argument("--ln", default="8192x4096,8192x8192,32768x8192")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--variants", default="auto")
    args = ap.parse_args()
    import torch
    from kubeflow_rm_amd import ops
    dev = torch.device("cuda", 0)
    out = []

    def emit(d):
        print(json.dumps(d), flush=True)
        out.append(d)

    for s in [int(x) for x in args.sizes.split(",") if x]:
        a = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(s, s, device=dev, dtype=torch.bfloat16)
        iters = max(3, min(200, int(2e12 / (2 * s ** 3)) + 1))
        variants = args.variants.split(",")
        ours, theirs = {v: [] for v in variants}, []
        for _ in range(3):
            for v in variants:
                ops.gemm_nt(a, b, out=c, variant=v)
            if not args.no_torch:
                torch.matmul(a, b.t())
        for _ in range(args.rounds):
            for v in variants:
                ours[v].append(timeit(lambda: ops.gemm_nt(a, b, out=c, variant=v), iters, dev))
            if not args.no_torch:
                theirs.append(timeit(lambda: torch.matmul(a, b.t()), iters, dev))
        fl = 2.0 * s ** 3
        d = {"kind": "gemm_nt_bf16", "M": s, "N": s, "K": s}
        for v in variants:
            d[f"{v}_tflops"] = round(fl / min(ours[v]) / 1e12, 1)
            d[f"{v}_tflops_median"] = round(fl / sorted(ours[v])[len(ours[v]) // 2] / 1e12, 1)
        if theirs:
            d["torch_tflops"] = round(fl / min(theirs) / 1e12, 1)
        emit(d)
        del a, b, c
        torch.cuda.empty_cache()

    for spec in [x for x in args.ln.split(",") if x]:
        rows, H = map(int, spec.split("x"))
        x = torch.randn(rows, H, device=dev).to(torch.bfloat16)
        w = torch.randn(H, device=dev).to(torch.bfloat16)
        bb = torch.randn(H, device=dev).to(torch.bfloat16)
        for _ in range(3):
            ops.layer_norm_fwd(x, w, bb)
            torch.nn.functional.layer_norm(x, (H,), w, bb)
        ts, tt = [], []
        for _ in range(args.rounds):
            ts.append(timeit(lambda: ops.layer_norm_fwd(x, w, bb), 50, dev))
            tt.append(timeit(lambda: torch.nn.functional.layer_norm(x, (H,), w, bb), 50, dev))
        bytes_moved = 2 * rows * H * 2
        emit({"kind": "layernorm_fwd_bf16", "rows": rows, "hidden": H,
              "ours_GBps": round(bytes_moved / min(ts) / 1e9, 1),
              "torch_GBps": round(bytes_moved / min(tt) / 1e9, 1),
              "ours_us": round(min(ts) * 1e6, 1), "torch_us": round(min(tt) * 1e6, 1)})
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text("\n".join(json.dumps(d) for d in out) + "\n")


if __name__ == "__main__":
    main()
