#!/usr/bin/env python3
"""A/B of w4 GEMM K-loop schedules (tools/w4_ab.hip built once per knob set) on one GPU.

  python tools/w4_ab.py --build            # on the host: compile every variant into kubeflow_rm_amd/lib/w4ab/
  python tools/w4_ab.py --sizes 4096,8192   # on the GPU: bitwise check vs production, interleaved timing
                                            # rounds vs the production kernel and torch.matmul, then the
                                            # variants' cheap K-loop stamps (cycles per 64-k tile by segment)

Prints one JSON line per measurement. Knobs: kernels/gemm_w4.h (KFW4_RG, KFW4_DMA_EVERY, KFW4_DMA_PHASE,
KFW4_PIN_MFMA, KFW4_PRIO); every variant also carries KFW4_CHEAP_STAMPS=1, which only touches its diag
kernel (s_memtime with no wait of its own, read after the loop's own lgkmcnt(0)).
"""
import argparse
import ctypes
import json
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
OUT = ROOT / "kubeflow_rm_amd" / "lib" / "w4ab"

VARIANTS = {
    "base": ["-DKFW4_FASTK=0", "-DKFW4_UNROLL5=0", "-DKFW4_ASM_DMA=0", "-DKFW4_PREBAR=0"],  # the round-3 K loop
    "unroll5": ["-DKFW4_FASTK=0", "-DKFW4_UNROLL5=1"],
    "f2u5": ["-DKFW4_FASTK=2", "-DKFW4_UNROLL5=1", "-DKFW4_ASM_DMA=0", "-DKFW4_PREBAR=0"],
    "r4": [],  # the production knobs
    "noful": ["-DKFW4_FULLLINE=0"],  # the half-line epilogue stores
    "asmdma": ["-DKFW4_ASM_DMA=1"],
    "prebar1": ["-DKFW4_PREBAR=1"],
    "prebar2": ["-DKFW4_PREBAR=2"],
    "asm_prebar1": ["-DKFW4_ASM_DMA=1", "-DKFW4_PREBAR=1"],
    "prev": ["-DKFW4_FASTK=2", "-DKFW4_UNROLL5=1"],
    "f2u5_rg4p0": ["-DKFW4_FASTK=2", "-DKFW4_UNROLL5=1", "-DKFW4_RG=4", "-DKFW4_DMA_PHASE=0"],
    "f2u5_e4p0": ["-DKFW4_FASTK=2", "-DKFW4_UNROLL5=1", "-DKFW4_DMA_EVERY=4", "-DKFW4_DMA_PHASE=0"],
    "u5_rg4p0": ["-DKFW4_FASTK=0", "-DKFW4_UNROLL5=1", "-DKFW4_RG=4", "-DKFW4_DMA_PHASE=0"],
    "rg4": ["-DKFW4_RG=4"],
    "dma_cluster": ["-DKFW4_DMA_EVERY=2", "-DKFW4_DMA_PHASE=1"],
    "dma_spread6": ["-DKFW4_DMA_EVERY=6", "-DKFW4_DMA_PHASE=1"],
    "nopin": ["-DKFW4_PIN_MFMA=0"],
    "noprio": ["-DKFW4_PRIO=0"],
    "gm2": ["-DKFW4_GROUP_M=2"],
    "gm8": ["-DKFW4_GROUP_M=8"],
    "gm16": ["-DKFW4_GROUP_M=16"],
    "phase3": ["-DKFW4_DMA_PHASE=3"],
    "gm32": ["-DKFW4_GROUP_M=32"],
    "rg4gm16": ["-DKFW4_RG=4", "-DKFW4_GROUP_M=16"],
    "nosuper": ["-DKFW4_SUPER=0"],  # the per-XCD row groups at every size (before r6zm_super)
    "rg4super": ["-DKFW4_RG=4"],
}


def build(names):
    from concurrent.futures import ThreadPoolExecutor
    OUT.mkdir(parents=True, exist_ok=True)

    def one(name):
        so = OUT / f"libw4ab_{name}.so"
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-mcode-object-version=5", f"-I{ROOT / 'kernels'}", "-DKFW4_CHEAP_STAMPS=1", *VARIANTS[name],
               str(ROOT / "tools" / "w4_ab.hip"), "-o", str(so)]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode:
            raise SystemExit(f"{name}: {p.stderr[-2000:]}")
        nm = subprocess.run(["nm", "-D", "--undefined-only", str(so)], capture_output=True, text=True).stdout
        if "device_stub" in nm:  # hipcc 7.2 dropped the launch stubs (gemm_w4.h notes)
            raise SystemExit(f"{name}: launch stubs missing")
        return name
    with ThreadPoolExecutor(4) as ex:
        for n in ex.map(one, names):
            print("built", n, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--sizes", default="4096,8192,16384")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--diag", default="8192")
    ap.add_argument("--po-grid", type=int, default=256, help="blocks of the persistent-overlapped (PO) launch")
    a = ap.parse_args()
    names = [v for v in a.variants.split(",") if v]
    if a.build:
        build(names)
        return
    import torch
    from kubeflow_rm_amd import ops
    vp, i = ctypes.c_void_p, ctypes.c_int
    libs = {}
    for n in names:
        L = ctypes.CDLL(str(OUT / f"libw4ab_{n}.so"))
        L.w4ab_nt.restype = i
        L.w4ab_nt.argtypes = [vp, vp, vp, i, i, i, vp]
        L.w4ab_diag.restype = i
        L.w4ab_diag.argtypes = [vp, vp, vp, i, i, i, vp, vp]
        L.w4ab_po.restype = i
        L.w4ab_po.argtypes = [vp, vp, vp, i, i, i, i, vp]
        libs[n] = L
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    for spec in [x for x in a.sizes.split(",") if x]:
        # s (s^3) or MxNxK
        M, N, K = (int(v) for v in spec.split("x")) if "x" in spec else (int(spec),) * 3
        s = spec
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        ref = ops.gemm_nt(A, B)
        C = torch.empty_like(ref)
        same = {}
        for n, L in libs.items():
            assert L.w4ab_nt(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, st) == 0
            torch.cuda.synchronize()
            same[n] = bool(torch.equal(C, ref))
            C.zero_()
            assert L.w4ab_po(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, a.po_grid, st) == 0
            torch.cuda.synchronize()
            same[n + "_po"] = bool(torch.equal(C, ref))
        flop = 2.0 * M * N * K
        iters = max(5, int(3e13 / flop))
        fns = {"prod": lambda: ops.gemm_nt(A, B, out=C), "torch": lambda: torch.matmul(A, B.t())}
        for n, L in libs.items():
            fns[n] = (lambda L=L: L.w4ab_nt(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, st))
            fns[n + "_po"] = (lambda L=L: L.w4ab_po(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, a.po_grid, st))
        t_end = time.perf_counter() + 1.0
        while time.perf_counter() < t_end:
            fns["prod"]()
        tf = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, fn in fns.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(iters):
                    fn()
                torch.cuda.synchronize()
                tf[k].append(flop * iters / (time.perf_counter() - t0) / 1e12)
        print(json.dumps({"size": s, "bitwise_equal_to_prod": same,
                          "median_tf": {k: round(statistics.median(v), 1) for k, v in tf.items()},
                          "best_tf": {k: round(max(v), 1) for k, v in tf.items()}}), flush=True)
        del A, B, C, ref
    for spec in [x for x in a.diag.split(",") if x]:
        # s (s^3) or MxNxK: e.g. 1024x1024x8192 puts 16 blocks on 16 CUs (no chip-wide store burst)
        M_, N_, K_ = (int(v) for v in spec.split("x")) if "x" in spec else (int(spec),) * 3
        A = (torch.rand(M_, K_, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N_, K_, device=dev) * 2 - 1).to(torch.bfloat16)
        C = torch.empty(M_, N_, device=dev, dtype=torch.bfloat16)
        nblk = (M_ // 256) * (N_ // 256)
        diag = torch.zeros(nblk * 4 * 16, dtype=torch.int64, device=dev)
        nk = K_ // 64
        s = spec
        for n, L in libs.items():
            for _ in range(3):
                assert L.w4ab_diag(A.data_ptr(), B.data_ptr(), C.data_ptr(), M_, N_, K_, diag.data_ptr(), st) == 0
            torch.cuda.synchronize()
            d = diag.view(nblk, 4, 16).double()
            seg = (d[..., :4].sum(dim=(0, 1)) / (nblk * 4 * (nk - 1))).tolist()  # cycles per 64-k tile
            clk = ((d[:, 0, 7]) / (d[:, 0, 9] - d[:, 0, 8]).clamp(min=1) * 100).median().item()
            print(json.dumps({"diag_size": s, "variant": n,
                              "cycles_per_ktile": {"substep0": round(seg[0]), "mid_wait_barrier": round(seg[1]),
                                                   "substep1": round(seg[2]), "end_wait_rotate": round(seg[3]),
                                                   "total": round(sum(seg))},
                              "prologue_cycles": round(d[..., 4].mean().item()),
                              "epilogue_cycles": round(d[..., 5].mean().item()),
                              "block_cycles": round(d[..., 7].mean().item()), "clock_mhz_median": round(clk)}),
                  flush=True)


if __name__ == "__main__":
    main()
