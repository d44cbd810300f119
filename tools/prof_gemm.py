#!/usr/bin/env python3
"""Kernel-trace target: gemm_nt (ours) or torch.matmul on [M, K] x [N, K]^T, 20 iterations.
python tools/prof_gemm.py ours|torch MxNxK"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from kubeflow_rm_amd import ops
    which = sys.argv[1] if len(sys.argv) > 1 else "ours"
    M, N, K = (int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1500x1500x1500").split("x"))
    dev = torch.device("cuda", 0)
    a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    for _ in range(20):
        if which == "ours":
            ops.gemm_nt(a, b)
        else:
            torch.matmul(a, b.t())
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
