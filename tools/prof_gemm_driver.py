#!/usr/bin/env python3
"""Profiling driver: N launches each of our GEMM variants and torch.matmul at one size (for
rocprofv3 --pmc / --kernel-trace; kernel names separate the variants)."""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="pipe_sched,w4")
    args = ap.parse_args()
    import torch
    from kubeflow_rm_amd import ops
    dev = torch.device("cuda", 0)
    s = args.size
    a = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
    c = torch.empty(s, s, device=dev, dtype=torch.bfloat16)
    for v in args.variants.split(","):
        for _ in range(args.iters):
            ops.gemm_nt(a, b, out=c, variant=v)
    for _ in range(args.iters):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
