#!/usr/bin/env python3
"""Per-kernel time summary from a rocprofv3 rocpd sqlite database (the default --kernel-trace output
on this image): python tools/rocpd_stats.py <run_results.db> [--last N] [--csv out.csv]"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    m = re.search(r"(gemm_w4)I(Li\d+E)(Lb\d+E)(Lb\d+E)(Lb\d+E)(Li\d+E)(Li\d+E)(Li\d+E)(Lb\d+E)?", name)
    if m:
        v = [re.sub(r"L[ib](\d+)E", r"\1", g or "") for g in m.groups()[1:]]
        sk = ",splitK" if v[7] == "1" else ""
        return f"gemm_w4<act{v[0]},b{v[1]},r{v[2]},x{v[3]},LA{v[4]},LB{v[5]},BM{v[6]}{sk}>"
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default="")
    ap.add_argument("--gaps", action="store_true", help="also print the last 12 dispatches with idle gaps")
    args = ap.parse_args()
    con = sqlite3.connect(args.db)
    rows = con.execute("""
        select k.display_name, d.end - d.start, d.start, d.end from rocpd_kernel_dispatch d
        join rocpd_info_kernel_symbol k on d.kernel_id = k.id
        order by d.start""").fetchall()
    agg = {}
    for name, dur, _, _ in rows:
        a = agg.setdefault(short(name), [0, 0.0])
        a[0] += 1
        a[1] += dur
    tot = sum(v[1] for v in agg.values())
    lines = ["kernel,calls,total_us,avg_us,pct"]
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{k},{n},{t / 1e3:.1f},{t / n / 1e3:.2f},{100 * t / tot:.1f}")
    print("\n".join(lines))
    if args.csv:
        open(args.csv, "w").write("\n".join(lines) + "\n")
    if args.gaps:
        print("last dispatches: kernel,dur_us,gap_before_us")
        tail = rows[-13:]
        for prev, cur in zip(tail, tail[1:]):
            print(f"  {short(cur[0])[:70]},{cur[1] / 1e3:.2f},{(cur[2] - prev[3]) / 1e3:.2f}")


if __name__ == "__main__":
    main()
