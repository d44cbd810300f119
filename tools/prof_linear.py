#!/usr/bin/env python3
"""Kernel-trace target: linear (gelu, bias) fwd+bwd on [T, K] x [N, K], ours or torch, N iterations."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from kubeflow_rm_amd import ops
    which = sys.argv[1] if len(sys.argv) > 1 else "ours"
    T, K, N = (int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "8192x4096x4096").split("x"))
    dev = torch.device("cuda", 0)
    x = ((torch.rand(T, K, device=dev) * 2 - 1).to(torch.bfloat16)).requires_grad_(True)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16).requires_grad_(True)
    b = torch.zeros(N, device=dev, dtype=torch.bfloat16).requires_grad_(True)
    gy = (torch.rand(T, N, device=dev) * 2 - 1).to(torch.bfloat16)
    F = torch.nn.functional
    for _ in range(20):
        x.grad = w.grad = b.grad = None
        if which == "ours":
            ops.linear(x, w, b, act="gelu_tanh").backward(gy)
        else:
            F.gelu(F.linear(x, w, b), approximate="tanh").backward(gy)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
