#!/usr/bin/env python3
"""kubeflow_rm_amd.optim.AdamW against torch's fused AdamW on a real model: the same init, the same
batches, the native kernels for the model in both runs; per-step losses of both runs, and the
optimizer step alone timed on gpt-1b's parameters.

  python tools/optim_check.py gpt-small 8 1024 20
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from kubeflow_rm_amd.models import gpt
    from kubeflow_rm_amd.optim import AdamW
    name, B, T, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    dev = torch.device("cuda", 0)
    losses = {}
    for which in ("ours", "torch"):
        torch.manual_seed(0)
        m = gpt.build(name, device=dev)
        opt = AdamW(m.parameters(), lr=3e-4, weight_decay=0.1) if which == "ours" else \
            torch.optim.AdamW(m.parameters(), lr=3e-4, weight_decay=0.1, fused=True)
        g = torch.Generator(device=dev).manual_seed(1)
        out = []
        for _ in range(n):
            idx = torch.randint(0, m.cfg.vocab_size, (B, T), generator=g, device=dev)
            opt.zero_grad(set_to_none=True)
            _, loss = m(idx, idx)
            loss.backward()
            opt.step()
            out.append(round(float(loss.item()), 4))
        losses[which] = out
        del m, opt
        torch.cuda.empty_cache()
    print(json.dumps({"model": name, "losses": losses}), flush=True)
    # the optimizer step alone on gpt-1b's parameters (bf16, grads set)
    m = gpt.build("gpt-1b", device=dev)
    for p in m.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    res = {}
    for which in ("ours", "torch"):
        opt = AdamW(m.parameters(), lr=1e-4) if which == "ours" else torch.optim.AdamW(m.parameters(), lr=1e-4,
                                                                                       fused=True)
        for _ in range(3):
            opt.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            opt.step()
        torch.cuda.synchronize()
        res[which + "_ms"] = round((time.perf_counter() - t0) / 10 * 1e3, 3)
        del opt
    print(json.dumps({"adamw_step_gpt1b": res, "params_M": round(sum(p.numel() for p in m.parameters()) / 1e6, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
