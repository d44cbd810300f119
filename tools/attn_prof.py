#!/usr/bin/env python3
"""rocprofv3 target: the flash attention kernels alone (fwd + bwd), a few iterations per shape.
python tools/attn_prof.py 4x16x2048x128 [iters]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from kubeflow_rm_amd import ops
    shp = sys.argv[1] if len(sys.argv) > 1 else "4x16x2048x128"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    B, H, T, D = map(int, shp.split("x"))
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v, do = (torch.randn(B, H, T, D, device="cuda", generator=g).to(torch.bfloat16) for _ in range(4))
    q, k, v = (x.requires_grad_(True) for x in (q, k, v))
    for _ in range(iters):
        o = ops.flash_attention(q, k, v, causal=True)
        torch.autograd.grad(o, (q, k, v), do)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
