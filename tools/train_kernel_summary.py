#!/usr/bin/env python3
"""Group a rocprofv3 kernel-stats CSV of a GPT training run (tools/prof_train.py) by role: our w4 GEMM
by operand layout (forward NT, dgrad, wgrad, split-K partials + reduce), hipBLASLt kernels by their
Tensile layout tag, attention, LayerNorm, cross-entropy, optimizer, other. Prints JSON: total ms per
group and the top kernels.
python tools/train_kernel_summary.py gpurun_out/.../run_kernel_stats.csv"""
import csv
import json
import re
import sys


def group(name: str) -> str:
    n = name
    if "gemm_w4" in n:
        # gemm_w4<ACT, HAS_BIAS, HAS_RES, HAS_AUX, LA, LB, BM, SPLIT, ...>
        m = re.search(r"gemm_w4I(.*?)EEEv", n)
        args = re.findall(r"L([ib])(-?\d+)E", m.group(1)) if m else []
        vals = [int(v) for _, v in args]
        if len(vals) >= 8:
            la, lb, split = vals[4], vals[5], vals[7]
            if split:
                return "ours: split-K partials"
            if la == 0 and lb == 0:
                return "ours: forward (NT)"
            if la == 1:
                return "ours: wgrad (dY^T X)"
            return "ours: dgrad (dY W)"
        return "ours: gemm_w4 (other)"
    if "splitk_reduce" in n:
        return "ours: split-K reduce"
    if "Cijk" in n:
        tag = re.search(r"Cijk_(A\w{3})_(B\w{3})", n)
        return "hipBLASLt " + (f"{tag.group(1)}_{tag.group(2)}" if tag else "")
    if ("GLOBAL__N" in n or "anonymous namespace" in n) and ("attn_fwd" in n or "attn_bwd" in n):
        return "ours: attention (flash)"  # kernels/attention_bf16.hip (aotriton's is a bare "attn_fwd")
    if "attn" in n or "flash" in n.lower() or "bwd_kernel" in n:
        return "attention (torch SDPA / aotriton)"
    if "norm" in n.lower():
        return "layernorm"
    if "xent" in n or "cross_entropy" in n.lower() or "nll" in n.lower() or "softmax" in n.lower():
        return "cross-entropy / softmax"
    if "adam" in n.lower() or "multi_tensor" in n.lower():
        return "optimizer"
    if "act_grad" in n or "gelu" in n.lower():
        return "activation grad"
    return "other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    groups: dict[str, float] = {}
    for r in rows:
        ms = float(r.get("TotalDurationNs") or r.get("TotalDuration") or 0) / 1e6
        g = group(r["Name"])
        groups[g] = groups.get(g, 0.0) + ms
    tot = sum(groups.values())
    print(json.dumps({"total_ms": round(tot, 2),
                      "groups_ms": {k: round(v, 2) for k, v in sorted(groups.items(), key=lambda kv: -kv[1])}}, indent=1))


if __name__ == "__main__":
    main()
