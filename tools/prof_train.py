#!/usr/bin/env python3
"""Kernel-trace target: a few GPT training steps (native kernels or torch ops).
python tools/prof_train.py native|torch gpt-1b 4 2048"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from kubeflow_rm_amd import ops
    from kubeflow_rm_amd.models import gpt
    which = sys.argv[1] if len(sys.argv) > 1 else "native"
    name = sys.argv[2] if len(sys.argv) > 2 else "gpt-1b"
    B, T = (int(sys.argv[3]) if len(sys.argv) > 3 else 4), (int(sys.argv[4]) if len(sys.argv) > 4 else 2048)
    dev = torch.device("cuda", 0)
    m = gpt.build(name, device=dev)
    if which == "torch":
        opt = torch.optim.AdamW(m.parameters(), lr=1e-4, fused=True)
    else:
        from kubeflow_rm_amd.optim import AdamW
        opt = AdamW(m.parameters(), lr=1e-4)
    idx = torch.randint(0, m.cfg.vocab_size, (B, T), device=dev)
    ctx = ops.torch_reference() if which == "torch" else open("/dev/null")
    with ctx:
        for _ in range(6):
            opt.zero_grad(set_to_none=True)
            _, loss = m(idx, idx)
            loss.backward()
            opt.step()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
