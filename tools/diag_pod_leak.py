#!/usr/bin/env python3
"""Which processes outlive a LocalCluster? Runs the bench's cold-start variants back to back (as
bench.py does) and, after each cluster has stopped, lists every TCP listener on the pod address
range (127.20.x.y / 127.21.x.y) with its owning process: on nodes without per-pod network
namespaces a leftover listener makes the next cluster's pod at the same address fail to bind.

  python tools/diag_pod_leak.py [--runs 3]      (GPU box; prints one JSON line per variant)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import struct
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def _listeners() -> list[dict]:
    inodes = {}
    for line in Path("/proc/net/tcp").read_text().splitlines()[1:]:
        f = line.split()
        if f[3] != "0A":  # LISTEN
            continue
        ip_hex, port_hex = f[1].split(":")
        ip = socket.inet_ntoa(struct.pack("<I", int(ip_hex, 16)))
        if ip.startswith(("127.20.", "127.21.")):
            inodes[f[9]] = f"{ip}:{int(port_hex, 16)}"
    out = []
    if not inodes:
        return out
    for pid in os.listdir("/proc"):
        if not pid.isdigit():
            continue
        try:
            fds = os.listdir(f"/proc/{pid}/fd")
        except OSError:
            continue
        for fd in fds:
            try:
                link = os.readlink(f"/proc/{pid}/fd/{fd}")
            except OSError:
                continue
            if link.startswith("socket:[") and link[8:-1] in inodes:
                try:
                    cmd = Path(f"/proc/{pid}/cmdline").read_bytes().replace(b"\0", b" ").decode()[:200]
                    stat = Path(f"/proc/{pid}/stat").read_text().rsplit(")", 1)[1].split()
                    ppid, pgid, sid = int(stat[1]), int(stat[2]), int(stat[3])
                except OSError:
                    cmd, ppid, pgid, sid = "?", -1, -1, -1
                out.append({"addr": inodes[link[8:-1]], "pid": int(pid), "ppid": ppid, "pgid": pgid, "sid": sid,
                            "cmd": cmd})
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    args = ap.parse_args()
    from kubeflow_rm_amd.bench_coldstart import measure_cold_start
    variants = [
        ("default", dict(server="torch-ready", namespace="bench", zygote=True)),
        ("stub", dict(namespace="bench-stub")),
        ("torch_fresh", dict(server="torch-ready", namespace="bench-torch")),
        ("odh", dict(odh_oauth=True, namespace="bench-odh")),
    ]
    rc = 0
    for name, kw in variants:
        t0 = time.time()
        cs = measure_cold_start(runs=args.runs, gpus_per_notebook=1, timeout=30, **kw)
        after = []
        for wait in (0.0, 1.0, 5.0):
            time.sleep(wait)
            after.append({"after_s": round(time.time() - t0, 1), "listeners": _listeners()})
        print(json.dumps({"variant": name, "p50_s": cs.get("p50_s"), "failures": len(cs.get("failures") or []),
                          "left_over": after}), flush=True)
        if any(a["listeners"] for a in after[-1:]):
            rc = 1
    return rc


if __name__ == "__main__":
    sys.exit(main())
