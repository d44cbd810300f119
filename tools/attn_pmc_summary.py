#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc counter files (tools/runs/r5t_attn_pmc.sh): sums each
counter over the dispatches of every kernel whose name matches, then prints wave-cycle shares.

  python tools/attn_pmc_summary.py gpurun_out/r5t_attn_pmc/pmc1 gpurun_out/r5t_attn_pmc/pmc2 ...
"""
import collections
import csv
import json
import sys
from pathlib import Path


def load(dirs):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in dirs:
        for f in Path(d).rglob("*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                for key in ("attn_bwd_dq_split", "attn_bwd_dkdv8", "attn_bwd_delta", "attn_bwd_dq<", "attn_bwd", "attn_fwd"):
                    if key.rstrip("<") in name and (key != "attn_bwd" or ("dq" not in name and "delta" not in name and "dkdv" not in name)):
                        tot[key.rstrip("<")][r["Counter_Name"]] += float(r["Counter_Value"])
                        break
    return tot


def main():
    tot = load(sys.argv[1:])
    out = {}
    for k, c in tot.items():
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        row = {n: c[n] for n in sorted(c)}
        # SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES cycles
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM"):
            if n in c:
                row[n + "_share"] = round(c[n] / wc, 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            row["mfma_busy_of_gui_active"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] * 256 * 4 / 8), 3)
        out[k] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
