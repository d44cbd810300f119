#!/usr/bin/env python3
"""Summarize tools/runs/gpu_prof_gemm.sh output: per kernel, counter means, mean dispatch time, effective clock."""
import collections
import csv
import sys
from pathlib import Path

base = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_gemm")
res = collections.defaultdict(dict)
for f in sorted(base.glob("pmc*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = "hipBLASLt" if "Cijk" in k else ("w4" if ("256w4" in k or "gemm_w4" in k) else ("pipe_sched" if "256p" in k else None))
        if k is None:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg[(k, r["Counter_Name"])].append((float(r["Counter_Value"]), d))
    for (k, c), v in agg.items():
        vals = [x for x, _ in v]
        ds = [d for _, d in v]
        res[k][c] = sum(vals) / len(vals)
        if c == "GRBM_GUI_ACTIVE":
            res[k]["eff_clock_GHz"] = round(sum(vals) / 8 / sum(ds) / 1e3, 3)
            res[k]["pmc_dispatch_us"] = round(sum(ds) / len(ds), 1)
for r in csv.DictReader(open(base / "trace/run_kernel_stats.csv")):
    k = r["Name"]
    k = "hipBLASLt" if "Cijk" in k else ("w4" if ("256w4" in k or "gemm_w4" in k) else ("pipe_sched" if "256p" in k else None))
    if k:
        res[k]["trace_mean_us"] = round(float(r["AverageNs"]) / 1e3, 1)
        res[k]["trace_TFLOPs"] = round(2 * 8192 ** 3 / (float(r["AverageNs"]) * 1e-9) / 1e12, 1)
for k, v in res.items():
    if "TCC_HIT_sum" in v:
        v["L2_hit_rate"] = round(v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]), 4)
    print(k, {a: (round(b, 3) if isinstance(b, float) else b) for a, b in sorted(v.items())})
