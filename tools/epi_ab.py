#!/usr/bin/env python3
"""Fused-epilogue cost on the GPT-1b forward projections: ops.gemm_nt with no epilogue, bias,
bias + residual, bias + GELU (+ pre-activation output), against torch (hipBLASLt with its bias
epilogue, plus a separate residual add / GELU). Median of rounds, microseconds per call.

  python tools/epi_ab.py 8192x2048x2048,8192x2048x8192,8192x6144x2048,8192x8192x2048
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from kubeflow_rm_amd import ops  # noqa: E402


def t_us(fn, iters=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    for spec in sys.argv[1].split(","):
        M, N, K = map(int, spec.split("x"))
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        b = (torch.rand(N, device="cuda") * 2 - 1).to(torch.bfloat16)
        r = (torch.rand(M, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fns = {
            "ours_none": lambda: ops.gemm_nt(x, w, out=out),
            "ours_bias": lambda: ops.gemm_nt(x, w, bias=b, out=out),
            "ours_bias_res": lambda: ops.gemm_nt(x, w, bias=b, residual=r, out=out),
            "ours_bias_gelu_preact": lambda: ops.gemm_nt_preact(x, w, b, "gelu_tanh"),
            "torch_bias": lambda: F.linear(x, w, b),
            "torch_bias_res": lambda: F.linear(x, w, b).add_(r),
            "torch_bias_gelu": lambda: F.gelu(F.linear(x, w, b), approximate="tanh"),
        }
        ref = (x.float() @ w.float().t() + b.float() + r.float())
        got = ops.gemm_nt(x, w, bias=b, residual=r).float()
        err = ((got - ref).abs().max() / (ref.abs().max() + 1e-6)).item()
        res = {k: [] for k in fns}
        for _ in range(5):
            for k, f in fns.items():
                res[k].append(t_us(f))
        print(json.dumps({"shape": spec, "bias_res_rel_err": round(err, 5),
                          "us": {k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
