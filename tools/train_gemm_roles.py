#!/usr/bin/env python3
"""Per-layer GEMM times of a GPT training-step kernel trace (rocprofv3 --kernel-trace CSV), by op
(qkv / out / fc1 / fc2 projections, lm head) and role (forward / dgrad / wgrad), from the order of
the launches: in each step's forward a layer runs qkv, attention, out, fc1, fc2; its backward runs
fc2, fc1, out (dgrad then wgrad each), attention backward, qkv. The two backends' GEMM kernels are
told apart from everything else by name (gemm_w4 / hipBLASLt Cijk), the attention kernels by the
flash-attention names. Output: one JSON object, mean microseconds per call.

  python tools/train_gemm_roles.py run_kernel_trace.csv
"""
import collections
import csv
import json
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = []
    for r in rows:
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "gemm_w4" in n or "Cijk" in n:
            ev.append(("G", d))
        elif "bwd_kernel_dk_dv" in n:
            ev.append(("AB", d))
        elif "attn_fwd" in n or ("fwd" in n and "attn" in n.lower()):
            ev.append(("AF", d))
    acc = collections.defaultdict(list)
    # forward: G(qkv) AF G(out) G(fc1) G(fc2) per layer; backward: G G(fc2) G G(fc1) G G(out) AB G G(qkv)
    for i, (k, d) in enumerate(ev):
        if k == "AF":
            before = [x for x in ev[max(0, i - 3):i] if x[0] == "G"]
            after = [x for x in ev[i + 1:i + 6] if x[0] != "G"][:1]
            g_after = []
            for x in ev[i + 1:]:
                if x[0] != "G":
                    break
                g_after.append(x)
            if before and len(g_after) >= 3:
                acc[("qkv", "fwd")].append(before[-1][1])
                for name, x in zip(("out", "fc1", "fc2"), g_after[:3]):
                    acc[(name, "fwd")].append(x[1])
        if k == "AB":
            g_before = []
            for x in reversed(ev[:i]):
                if x[0] != "G":
                    break
                g_before.append(x)
            g_before = g_before[::-1]
            g_after = []
            for x in ev[i + 1:]:
                if x[0] != "G":
                    break
                g_after.append(x)
            if len(g_before) >= 6 and len(g_after) >= 2:
                for name, role, x in zip(("fc2", "fc2", "fc1", "fc1", "out", "out"),
                                         ("dgrad", "wgrad") * 3, g_before[-6:]):
                    acc[(name, role)].append(x[1])
                acc[("qkv", "dgrad")].append(g_after[0][1])
                acc[("qkv", "wgrad")].append(g_after[1][1])
    out = {f"{op}.{role}": {"calls": len(v), "mean_us": round(sum(v) / len(v), 1)} for (op, role), v in sorted(acc.items())}
    per_layer = collections.Counter()
    for (op, role), v in acc.items():
        per_layer[role] += sum(v) / len(v)
    out["per_layer_us"] = {k: round(v, 1) for k, v in per_layer.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
