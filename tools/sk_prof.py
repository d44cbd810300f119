#!/usr/bin/env python3
"""Stream-K profiling driver: a few launches of the plain kernel and of given stream-K plans on one
shape (for rocprofv3 kernel traces / counters). Usage: sk_prof.py MxNxK S1,S2,..."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from kubeflow_rm_amd.ops import gemm  # noqa: E402


def main():
    M, N, K = map(int, sys.argv[1].split("x"))
    splits = [int(x) for x in sys.argv[2].split(",")]
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        gemm.gemm_nt(a, b, out=c, variant="w4")
    torch.cuda.synchronize()
    for s in splits:
        for _ in range(5):
            gemm._streamk(a, b, c, M, N, K, K, K, N, (256, s), bias=None, r_ptr=None, ldr=0, aux=None, alpha=1.0,
                          act="none")
        torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
