#!/usr/bin/env python3
"""w4 GEMM K-loop stamps: shares of substep-0 issue (+F1 reads landing), DMA wait + barrier,
substep-1 issue, final read wait — per wave, averaged over the grid (diagnostic build only;
read shares, not the total). Also times the real kernel in the same process for reference."""
import ctypes
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from kubeflow_rm_amd import _build, ops
    # the stamped / ablation kernels live in their own library (never in libkfamd_kernels.so);
    # build it on the host first: python -c "from kubeflow_rm_amd import _build; _build.build_diag_kernels()"
    import os
    lib = Path(os.environ.get("KFAMD_DIAG_LIB", str(_build.DIAG_LIB)))  # A/B: another diag build
    if not lib.exists():
        raise SystemExit(f"{lib} missing: build it with _build.build_diag_kernels()")
    L = ctypes.CDLL(str(lib))
    f = L.kfamd_gemm_nt_bf16_w4_diag
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    for spec in (sys.argv[1] if len(sys.argv) > 1 else "4096,8192,16384").split(","):
        # a size s (s^3) or MxNxK (multiples of 256 / 256 / 64)
        M, N, K = (int(v) for v in spec.split("x")) if "x" in spec else (int(spec),) * 3
        s = K
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        nblk = (M // 256) * (N // 256)
        diag = torch.zeros(nblk * 4 * 16, dtype=torch.int64, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        abl_cycles = {}
        for abl in (1, 2, 0):
            for _ in range(3):
                rc = f(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, diag.data_ptr(), abl, stream)
                assert rc == 0, rc
            torch.cuda.synchronize()
            d8 = diag.view(nblk, 4, 16).double()
            draw = diag.view(nblk, 4, 16)
            d = d8[..., :4]
            abl_cycles[abl] = round(d.sum(-1).mean().item() / (s // 64))
        # in-kernel clock (MHz) = shader clocks / realtime ticks * 100, per block (wave 0)
        w0 = draw[:, 0, :]
        rt = (w0[:, 9] - w0[:, 8]).double()
        clk_mhz = (w0[:, 7].double() / rt.clamp(min=1) * 100.0)
        # per-CU timeline: gaps between consecutive blocks on the same CU (realtime ticks = 10 ns)
        hw = w0[:, 10]
        cu_key = ((hw >> 32) & 0xF) * 8192 + ((hw >> 13) & 0x7) * 1024 + ((hw >> 12) & 1) * 512 + ((hw >> 8) & 0xF)
        starts, ends = w0[:, 8], w0[:, 9]
        gaps, blocks_per_cu = [], []
        t_first, t_last = starts.min().item(), ends.max().item()
        for key in torch.unique(cu_key).tolist():
            sel = (cu_key == key).nonzero().flatten()
            order = sel[torch.argsort(starts[sel])]
            blocks_per_cu.append(len(order))
            for a_, b_ in zip(order[:-1].tolist(), order[1:].tolist()):
                gaps.append((starts[b_] - ends[a_]).item() * 10.0)  # ns
        gaps_t = torch.tensor(gaps, dtype=torch.float64) if gaps else torch.zeros(1, dtype=torch.float64)
        timeline = {"cus_used": len(blocks_per_cu), "blocks_per_cu_max": max(blocks_per_cu),
                    "inter_block_gap_ns_median": round(gaps_t.median().item(), 1),
                    "inter_block_gap_ns_mean": round(gaps_t.mean().item(), 1),
                    "kernel_span_us": round((t_last - t_first) * 0.01, 1),
                    "block_us_median": round((ends - starts).double().median().item() * 0.01, 2),
                    "clock_MHz_median": round(clk_mhz.median().item(), 1)}
        tot = d.sum(-1, keepdim=True)
        share = (d / tot).mean(dim=(0, 1)).tolist()
        cyc = d.mean(dim=(0, 1)).tolist()
        # real kernel time, same process
        for _ in range(3):
            ops.gemm_nt(a, b, out=c, variant="w4")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 10
        for _ in range(n):
            ops.gemm_nt(a, b, out=c, variant="w4")
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        print(json.dumps({"size": spec, "segments": ["substep0_issue+F1_land", "dma_wait+barrier", "substep1_issue",
                                                   "F0_land"], "share": [round(x, 4) for x in share],
                          "mean_cycles_per_wave": [round(x) for x in cyc], "w4_tflops": round(2 * M * N * K / dt / 1e12, 1),
                          "loop_cycles_per_ktile": round(sum(cyc) / (s // 64)),
                          "prologue_cycles": round(d8[..., 4].mean().item()), "epilogue_issue_cycles": round(d8[..., 5].mean().item()),
                          "kloop_cycles": round(d8[..., 6].mean().item()),
                          "block_cycles": round(d8[..., 7].mean().item()), "timeline": timeline,
                          "ablation_loop_cycles_per_ktile": {"no_dma": abl_cycles[1], "no_ds_read": abl_cycles[2],
                                                             "full": abl_cycles[0]}}), flush=True)


if __name__ == "__main__":
    main()
