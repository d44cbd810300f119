#!/usr/bin/env python3
"""Driver for rocprofv3 passes over K2 (LayerNorm fwd, 32768x8192 bf16) and K3 (one-shot
all-reduce, 8 ranks simulated on one device, 256 KiB fp32 per rank)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from kubeflow_rm_amd import ops
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    x = torch.randn(32768, 8192, device="cuda").to(torch.bfloat16)
    w = torch.randn(8192, device="cuda").to(torch.bfloat16)
    b = torch.randn(8192, device="cuda").to(torch.bfloat16)
    for _ in range(iters):
        ops.layer_norm_fwd(x, w, b)
    ar = ops.OneShotAllReduce(8, 65536, torch.float32)
    xs = [torch.randn(65536, device="cuda") for _ in range(8)]
    for _ in range(iters):
        ar(xs)
    torch.cuda.synchronize()
    assert not ar.timed_out()
    print("ok")


if __name__ == "__main__":
    main()
