#!/usr/bin/env python3
"""A/B of the w4 GEMM schedule knobs (diagnostic library, kernels/gemm_bf16_w4.hip KN word) against
the production kernel and torch.matmul (hipBLASLt): interleaved rounds in ONE process
(cdna_hip_programming.md §5.4 rule 24), random operands, and every knob's output checked BITWISE
against the production kernel's (the knobs change only scheduling, never the arithmetic order).

Build the diagnostic library on the host first:
  python -c "from kubeflow_rm_amd import _build; _build.build_diag_kernels()"
"""
import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

KNOBS = {0: "base", 1: "dma2nd", 4: "nt_store", 8: "sc1_store", 16: "persist", 17: "persist+dma2nd",
         20: "persist+nt", 24: "persist+sc1"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,8192,16384")
    ap.add_argument("--knobs", default=",".join(str(k) for k in KNOBS))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    from kubeflow_rm_amd import _build, ops
    if not _build.DIAG_LIB.exists():
        raise SystemExit(f"{_build.DIAG_LIB} missing: build it with _build.build_diag_kernels()")
    L = ctypes.CDLL(str(_build.DIAG_LIB))
    f = L.kfamd_gemm_nt_bf16_w4_knob
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    knobs = [int(k) for k in args.knobs.split(",") if k]
    out = []
    for s in [int(x) for x in args.sizes.split(",") if x]:
        a = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
        ref = ops.gemm_nt(a, b)
        c = torch.empty_like(ref)
        stream = torch.cuda.current_stream(dev).cuda_stream
        bad = {}
        for k in knobs:
            c.zero_()
            rc = f(k, a.data_ptr(), b.data_ptr(), c.data_ptr(), s, s, s, stream)
            assert rc == 0, (k, rc)
            torch.cuda.synchronize()
            if not torch.equal(c, ref):
                bad[k] = int((c != ref).sum().item())
        iters = max(3, min(100, int(4e12 / (2 * s ** 3)) + 1))
        runs = {**{f"kn{k}": (lambda k=k: f(k, a.data_ptr(), b.data_ptr(), c.data_ptr(), s, s, s, stream)) for k in knobs},
                "prod": lambda: ops.gemm_nt(a, b, out=c), "torch": lambda: torch.matmul(a, b.t())}
        times = {n: [] for n in runs}
        for fn in runs.values():
            fn()
        for _ in range(args.rounds):
            for n, fn in runs.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(iters):
                    fn()
                torch.cuda.synchronize()
                times[n].append((time.perf_counter() - t0) / iters)
        fl = 2.0 * s ** 3
        d = {"size": s, "iters": iters, "rounds": args.rounds, "mismatch_vs_prod": bad}
        for n, ts in times.items():
            ts = sorted(ts)
            label = KNOBS.get(int(n[2:]), n) if n.startswith("kn") else n
            d[label] = {"best_tf": round(fl / ts[0] / 1e12, 1), "median_tf": round(fl / ts[len(ts) // 2] / 1e12, 1)}
        print(json.dumps(d), flush=True)
        out.append(d)
        del a, b, c, ref
        torch.cuda.empty_cache()
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text("\n".join(json.dumps(d) for d in out) + "\n")


if __name__ == "__main__":
    main()
