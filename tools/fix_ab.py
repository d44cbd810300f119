#!/usr/bin/env python3
"""Where the split-K fixup's time goes: the wgrad kernel (LA = LB = 1) built with KFW4_FIX_AB
ablations (1 no partial stores, 2 no partial reads by the owner, 3 neither, 4 stores / loads
without sc1), timed against the production build at forced split counts.

  python tools/fix_ab.py --build           # host: kubeflow_rm_amd/lib/fixab/libfixab_<v>.so
  python tools/fix_ab.py 2048x2048x8192 --splits 3,4
"""
import argparse
import ctypes
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
OUT = ROOT / "kubeflow_rm_amd" / "lib" / "fixab"
VARIANTS = {"prod": 0, "nostore": 1, "noread": 2, "neither": 3, "nosc1": 4}


def build():
    from concurrent.futures import ThreadPoolExecutor
    OUT.mkdir(parents=True, exist_ok=True)

    def one(name):
        so = OUT / f"libfixab_{name}.so"
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               f"-I{ROOT / 'kernels'}", f"-DKFW4_FIX_AB={VARIANTS[name]}", str(ROOT / "tools" / "fix_ab.hip"),
               "-o", str(so)]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode:
            raise SystemExit(f"{name}: {p.stderr[-2000:]}")
        nm = subprocess.run(["nm", "-D", "--undefined-only", str(so)], capture_output=True, text=True).stdout
        if "device_stub" in nm:
            raise SystemExit(f"{name}: launch stubs missing")
        return name
    with ThreadPoolExecutor(5) as ex:
        for n in ex.map(one, VARIANTS):
            print("built", n, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="?", default="2048x2048x8192")
    ap.add_argument("--splits", default="3,4")
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    if a.build:
        build()
        return
    import torch
    vp, i, ll, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float
    libs = {}
    for n in VARIANTS:
        L = ctypes.CDLL(str(OUT / f"libfixab_{n}.so"))
        L.fixab_11.restype = i
        L.fixab_11.argtypes = [vp, vp, vp, vp, i, i, i, i, ll, ll, ll, ll, ll, ll, ll, ll, f, vp, vp, i, i, vp]
        libs[n] = L
    st = torch.cuda.current_stream().cuda_stream
    for spec in a.shapes.split(","):
        M, N, K = map(int, spec.split("x"))
        gy = (torch.rand(K, M, device="cuda") * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(K, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        tiles = -(-M // 256) * -(-N // 256)
        cnt = torch.zeros(tiles, dtype=torch.int32, device="cuda")
        for S in [int(v) for v in a.splits.split(",")]:
            kper = -(-(-(-K // S)) // 64) * 64
            W = torch.empty(S * tiles * 65536, dtype=torch.float32, device="cuda")
            res = {}
            for n, L in libs.items():
                def run(L=L):
                    assert L.fixab_11(gy.data_ptr(), x.data_ptr(), out.data_ptr(), None, M, N, K, 1, M, N, N, 0, 0, 0,
                                      0, 0, 1.0, W.data_ptr(), cnt.data_ptr(), S, kper, st) == 0
                for _ in range(3):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                best = 1e9
                for _ in range(3):
                    e0.record()
                    for _ in range(20):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
                res[n] = round(best, 1)
            from kubeflow_rm_amd import ops
            from kubeflow_rm_amd.ops import gemm as G
            G.FIXK = False
            ops.mm(gy, x, trans_a=True, out=out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.mm(gy, x, trans_a=True, out=out)
            e1.record()
            torch.cuda.synchronize()
            G.FIXK = True
            res["prev_plan"] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
            print(json.dumps({"shape": spec, "splits": S, "kper": kper, "us": res}), flush=True)


if __name__ == "__main__":
    main()
