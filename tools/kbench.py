#!/usr/bin/env python3
"""Kernel micro-benchmarks on one GPU: GEMM TFLOPS sweep (ours vs torch/hipBLASLt), LayerNorm GB/s.

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24); random operands.
Prints one JSON line per measurement; --out writes them to a file as well.
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(fn, iters, dev):
    import torch
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,2048,4096,8192,16384")
    ap.add_argument("--ln", default="8192x4096,8192x8192,32768x8192")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--variants", default="auto")
    ap.add_argument("--layouts", default="", help="MxNxK list: mm() in all four operand layouts vs torch")
    ap.add_argument("--splitk", default="", help="MxNxK list: gemm_nt with and without split-K vs torch")
    ap.add_argument("--streamk", default="", help="MxNxK list: gemm_nt with and without stream-K vs torch")
    ap.add_argument("--linear", default="", help="TxKxN list: linear fwd+bwd (gelu, bias) vs torch autograd")
    args = ap.parse_args()
    import torch
    from kubeflow_rm_amd import ops
    dev = torch.device("cuda", 0)
    out = []

    def emit(d):
        print(json.dumps(d), flush=True)
        out.append(d)

    for s in [int(x) for x in args.sizes.split(",") if x]:
        a = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(s, s, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(s, s, device=dev, dtype=torch.bfloat16)
        iters = max(3, min(200, int(2e12 / (2 * s ** 3)) + 1))
        variants = args.variants.split(",")
        ours, theirs = {v: [] for v in variants}, []
        for _ in range(3):
            for v in variants:
                ops.gemm_nt(a, b, out=c, variant=v)
            if not args.no_torch:
                torch.matmul(a, b.t())
        for _ in range(args.rounds):
            for v in variants:
                ours[v].append(timeit(lambda: ops.gemm_nt(a, b, out=c, variant=v), iters, dev))
            if not args.no_torch:
                theirs.append(timeit(lambda: torch.matmul(a, b.t()), iters, dev))
        fl = 2.0 * s ** 3
        d = {"kind": "gemm_nt_bf16", "M": s, "N": s, "K": s}
        for v in variants:
            d[f"{v}_tflops"] = round(fl / min(ours[v]) / 1e12, 1)
            d[f"{v}_tflops_median"] = round(fl / sorted(ours[v])[len(ours[v]) // 2] / 1e12, 1)
        if theirs:
            d["torch_tflops"] = round(fl / min(theirs) / 1e12, 1)
        emit(d)
        del a, b, c
        torch.cuda.empty_cache()

    for spec in [x for x in args.splitk.split(",") if x]:
        from kubeflow_rm_amd.ops import gemm as G
        M, N, K = map(int, spec.split("x"))
        fl = 2.0 * M * N * K
        iters = max(10, min(200, int(2e12 / fl) + 1))
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = {}
        for tag, on in (("split", True), ("nosplit", False)):
            G.SPLITK = on
            for _ in range(3):
                ops.gemm_nt(a, b, out=c)
            res[tag] = min(timeit(lambda: ops.gemm_nt(a, b, out=c), iters, dev) for _ in range(args.rounds))
        G.SPLITK = True
        for _ in range(3):
            torch.matmul(a, b.t())
        res["torch"] = min(timeit(lambda: torch.matmul(a, b.t()), iters, dev) for _ in range(args.rounds))
        d = {"kind": "gemm_splitk_bf16", "M": M, "N": N, "K": K, "plan": G.splitk_plan(M, N, K)}
        for k, v in res.items():
            d[f"{k}_us"] = round(v * 1e6, 1)
            d[f"{k}_tflops"] = round(fl / v / 1e12, 1)
        emit(d)
        del a, b, c
        torch.cuda.empty_cache()

    for spec in [x for x in args.streamk.split(",") if x]:
        from kubeflow_rm_amd.ops import gemm as G
        M, N, K = map(int, spec.split("x"))
        fl = 2.0 * M * N * K
        iters = max(10, min(200, int(2e12 / fl) + 1))
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = torch.matmul(a, b.t())
        res, err = {}, {}
        for tag, on in (("sk", True), ("dp", False)):
            G.STREAMK = on
            for _ in range(3):
                ops.gemm_nt(a, b, out=c)
            err[tag] = float((c.float() - ref.float()).abs().max())
            res[tag] = []
        for _ in range(args.rounds):  # interleaved rounds
            for tag, on in (("sk", True), ("dp", False)):
                G.STREAMK = on
                res[tag].append(timeit(lambda: ops.gemm_nt(a, b, out=c), iters, dev))
            res.setdefault("torch", []).append(timeit(lambda: torch.matmul(a, b.t()), iters, dev))
        G.STREAMK = True  # (for the plan below; restored after)
        d = {"kind": "gemm_streamk_bf16", "M": M, "N": N, "K": K, "plan": G.streamk_plan(M, N, K),
             "max_err_vs_torch": err}
        for k, v in res.items():
            d[f"{k}_us"] = round(min(v) * 1e6, 1)
            d[f"{k}_tflops"] = round(fl / min(v) / 1e12, 1)
        G.STREAMK = False
        emit(d)
        del a, b, c, ref
        torch.cuda.empty_cache()

    for spec in [x for x in args.layouts.split(",") if x]:
        M, N, K = map(int, spec.split("x"))
        fl = 2.0 * M * N * K
        iters = max(3, min(200, int(2e12 / fl) + 1))
        d = {"kind": "mm_layouts_bf16", "M": M, "N": N, "K": K}
        for ta, tb in ((False, True), (False, False), (True, False), (True, True)):
            a = (torch.rand(*((K, M) if ta else (M, K)), device=dev) * 2 - 1).to(torch.bfloat16)
            b = (torch.rand(*((N, K) if tb else (K, N)), device=dev) * 2 - 1).to(torch.bfloat16)
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fa = (lambda: a.t()) if ta else (lambda: a)
            fb = (lambda: b.t()) if tb else (lambda: b)
            for _ in range(3):
                ops.mm(a, b, trans_a=ta, trans_b=tb, out=c)
                torch.matmul(fa(), fb())
            o, t = [], []
            for _ in range(args.rounds):
                o.append(timeit(lambda: ops.mm(a, b, trans_a=ta, trans_b=tb, out=c), iters, dev))
                t.append(timeit(lambda: torch.matmul(fa(), fb()), iters, dev))
            tag = ("T" if ta else "N") + ("T" if tb else "N")
            d[f"{tag}_tflops"] = round(fl / min(o) / 1e12, 1)
            d[f"{tag}_torch_tflops"] = round(fl / min(t) / 1e12, 1)
            del a, b, c
        emit(d)
        torch.cuda.empty_cache()

    for spec in [x for x in args.linear.split(",") if x]:
        T, K, N = map(int, spec.split("x"))
        x = ((torch.rand(T, K, device=dev) * 2 - 1).to(torch.bfloat16)).requires_grad_(True)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16).requires_grad_(True)
        bb = torch.zeros(N, device=dev, dtype=torch.bfloat16).requires_grad_(True)
        gy = (torch.rand(T, N, device=dev) * 2 - 1).to(torch.bfloat16)
        F = torch.nn.functional

        from kubeflow_rm_amd.ops import gemm as G

        def ours():
            ops.linear(x, w, bb, act="gelu_tanh").backward(gy)

        def ours_fwd():
            with torch.no_grad():
                ops.linear(x, w, bb, act="gelu_tanh")

        def theirs():
            F.gelu(F.linear(x, w, bb), approximate="tanh").backward(gy)

        def theirs_fwd():
            with torch.no_grad():
                F.gelu(F.linear(x, w, bb), approximate="tanh")
        res = {}
        for mode in ("fused", "split"):
            G.PREACT_MODE = mode
            for _ in range(3):
                ours()
            res[mode] = min(timeit(ours, 10, dev) for _ in range(args.rounds))
            res[mode + "_fwd"] = min(timeit(ours_fwd, 10, dev) for _ in range(args.rounds))
        G.PREACT_MODE = "auto"
        for _ in range(3):
            theirs()
        t = min(timeit(theirs, 10, dev) for _ in range(args.rounds))
        tf = min(timeit(theirs_fwd, 10, dev) for _ in range(args.rounds))
        fl = 3 * 2.0 * T * K * N
        best = min(res["fused"], res["split"])
        emit({"kind": "linear_gelu_fwd_bwd_bf16", "T": T, "K": K, "N": N, "ours_ms": round(best * 1e3, 3),
              "fused_ms": round(res["fused"] * 1e3, 3), "split_ms": round(res["split"] * 1e3, 3),
              "fused_fwd_ms": round(res["fused_fwd"] * 1e3, 3), "split_fwd_ms": round(res["split_fwd"] * 1e3, 3),
              "torch_ms": round(t * 1e3, 3), "torch_fwd_ms": round(tf * 1e3, 3),
              "ours_tflops": round(fl / best / 1e12, 1), "torch_tflops": round(fl / t / 1e12, 1)})
        del x, w, bb, gy
        torch.cuda.empty_cache()

    for spec in [x for x in args.ln.split(",") if x]:
        rows, H = map(int, spec.split("x"))
        x = torch.randn(rows, H, device=dev).to(torch.bfloat16)
        w = torch.randn(H, device=dev).to(torch.bfloat16)
        bb = torch.randn(H, device=dev).to(torch.bfloat16)
        for _ in range(3):
            ops.layer_norm_fwd(x, w, bb)
            torch.nn.functional.layer_norm(x, (H,), w, bb)
        ts, tt = [], []
        for _ in range(args.rounds):
            ts.append(timeit(lambda: ops.layer_norm_fwd(x, w, bb), 50, dev))
            tt.append(timeit(lambda: torch.nn.functional.layer_norm(x, (H,), w, bb), 50, dev))
        bytes_moved = 2 * rows * H * 2
        # the copy roof on this device and shape: a D2D copy of the same bytes (read + write)
        dst = torch.empty_like(x)
        tc = min(timeit(lambda: dst.copy_(x), 50, dev) for _ in range(args.rounds))
        emit({"kind": "layernorm_fwd_bf16", "rows": rows, "hidden": H,
              "ours_GBps": round(bytes_moved / min(ts) / 1e9, 1),
              "torch_GBps": round(bytes_moved / min(tt) / 1e9, 1),
              "copy_GBps": round(bytes_moved / tc / 1e9, 1),
              "ours_of_copy_roof": round(tc / min(ts), 3),
              "ours_us": round(min(ts) * 1e6, 1), "torch_us": round(min(tt) * 1e6, 1)})
        # backward: the dx pass alone (reads dy, x; writes dx), with the residual gradient folded in
        # (+ one read), the whole backward with dgamma / dbeta, and torch's autograd LayerNorm backward
        from kubeflow_rm_amd.ops import _lib as L
        _, mean, rstd = ops.layer_norm_fwd(x, w, bb, save_stats=True)
        gy = torch.randn(rows, H, device=dev).to(torch.bfloat16)
        gr = torch.randn(rows, H, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(x)
        dg = torch.empty(H, device=dev, dtype=torch.bfloat16)
        db = torch.empty(H, device=dev, dtype=torch.bfloat16)
        ws = torch.empty(L.lib().kfamd_layernorm_bwd_workspace(rows, H) // 4, device=dev, dtype=torch.float32)
        st = torch.cuda.current_stream(dev).cuda_stream

        def bwd(res, full):
            L.lib().kfamd_layernorm_bwd_bf16_v3(gy.data_ptr(), gr.data_ptr() if res else None, x.data_ptr(),
                                                w.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                                dg.data_ptr() if full else None, db.data_ptr() if full else None, 1,
                                                ws.data_ptr(), rows, H, st)
        xr = x.clone().requires_grad_(True)
        wr, br = w.clone().requires_grad_(True), bb.clone().requires_grad_(True)
        yr = torch.nn.functional.layer_norm(xr, (H,), wr, br)

        def torch_bwd():
            torch.autograd.grad(yr, (xr, wr, br), gy, retain_graph=True)
        res = {"dx": [], "dx_res": [], "full": [], "full_res": [], "torch": []}
        for _ in range(args.rounds):
            res["dx"].append(timeit(lambda: bwd(False, False), 50, dev))
            res["dx_res"].append(timeit(lambda: bwd(True, False), 50, dev))
            res["full"].append(timeit(lambda: bwd(False, True), 50, dev))
            res["full_res"].append(timeit(lambda: bwd(True, True), 50, dev))
            res["torch"].append(timeit(torch_bwd, 20, dev))
        b3, b4 = 3 * rows * H * 2, 4 * rows * H * 2
        emit({"kind": "layernorm_bwd_bf16", "rows": rows, "hidden": H,
              "dx_us": round(min(res["dx"]) * 1e6, 1), "dx_GBps": round(b3 / min(res["dx"]) / 1e9, 1),
              "dx_res_us": round(min(res["dx_res"]) * 1e6, 1), "dx_res_GBps": round(b4 / min(res["dx_res"]) / 1e9, 1),
              "full_us": round(min(res["full"]) * 1e6, 1), "full_res_us": round(min(res["full_res"]) * 1e6, 1),
              "torch_full_us": round(min(res["torch"]) * 1e6, 1),
              "copy_GBps": round(bytes_moved / tc / 1e9, 1)})
        del x, w, bb, gy, gr, dx, dst, ws, xr, yr
        torch.cuda.empty_cache()
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text("\n".join(json.dumps(d) for d in out) + "\n")


if __name__ == "__main__":
    main()
