#!/usr/bin/env python3
"""A/B of the w4 grouped-raster tile-row group (KFW4_GROUP_M) on square GEMMs: the production library
(group 4) against scratch builds lib/libkfamd_w4_gm{2,8,16}.so, interleaved rounds, plus torch."""
import ctypes
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from kubeflow_rm_amd import ops
    lib_dir = Path(__file__).resolve().parent.parent / "kubeflow_rm_amd" / "lib"
    libs = {"gm4": ops.lib()}
    for g in (2, 8, 16):
        p = lib_dir / f"libkfamd_w4_gm{g}.so"
        if p.exists():
            libs[f"gm{g}"] = ctypes.CDLL(str(p))
    vp, ll, i = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int
    for L in libs.values():
        L.kfamd_w4_launch_nt.restype = i
        L.kfamd_w4_launch_nt.argtypes = [i, vp, vp, vp, vp, vp, vp, i, i, i, i, ll, ll, ll, ll, ll, ll, ll, ll,
                                         ctypes.c_float, i, vp]
    dev = torch.device("cuda", 0)
    for s in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8192,16384").split(",")]:
        a = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(s, s, device=dev, dtype=torch.bfloat16)
        st = torch.cuda.current_stream(dev).cuda_stream
        iters = max(5, int(4e13 / (2 * s ** 3)))

        def run(L):
            rc = L.kfamd_w4_launch_nt(256, a.data_ptr(), b.data_ptr(), c.data_ptr(), None, None, None, s, s, s, 1,
                                      s, s, s, 0, 0, 0, 0, 0, 1.0, 0, st)
            assert rc == 0, rc
        best = {k: 0.0 for k in libs}
        best["torch"] = 0.0
        t_end = time.perf_counter() + 1.0
        while time.perf_counter() < t_end:  # settle the clock
            run(libs["gm4"])
        torch.cuda.synchronize()
        for _ in range(5):
            for k, L in list(libs.items()) + [("torch", None)]:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(iters):
                    if L is None:
                        torch.matmul(a, b.t())
                    else:
                        run(L)
                torch.cuda.synchronize()
                tf = 2 * s ** 3 * iters / (time.perf_counter() - t0) / 1e12
                best[k] = max(best[k], tf)
        print(json.dumps({"size": s, **{k: round(v, 1) for k, v in best.items()}}), flush=True)


if __name__ == "__main__":
    main()
