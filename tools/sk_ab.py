#!/usr/bin/env python3
"""Stream-K ablation timing: kubeflow_rm_amd/lib/skab{0..3}.so (tools/sk_ab.hip built with
-DKFW4_SK_AB=0..3: 1 = no partial stores / adds, 2 = owners do not wait, 3 = both) at several splits."""
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from kubeflow_rm_amd import ops  # noqa: E402


def main():
    libs = {}
    for v in range(4):
        p = ROOT / "kubeflow_rm_amd" / "lib" / f"skab{v}.so"
        if p.exists():
            lib = ctypes.CDLL(str(p))
            lib.skab_launch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2 + \
                [ctypes.c_uint, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
            libs[v] = lib
    W = torch.empty(64 * 1024 * 1024, dtype=torch.float32, device="cuda")
    F = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    epoch = [0]
    for spec in sys.argv[1].split(","):
        M, N, K = map(int, spec.split("x"))
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        st = torch.cuda.current_stream().cuda_stream

        def run(v, s):
            epoch[0] += 1
            assert libs[v].skab_launch(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, W.data_ptr(), F.data_ptr(),
                                       epoch[0], 256, s, st) == 0

        fns = {"plain": lambda: ops.gemm_nt(a, b, out=c, variant="w4")}
        for v in libs:
            for s in (1, 3, 8):
                fns[f"ab{v}_s{s}"] = (lambda v=v, s=s: run(v, s))
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        res = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                for _ in range(20):
                    f()
                ev1.record()
                torch.cuda.synchronize()
                res[k].append(ev0.elapsed_time(ev1) / 20 * 1e3)
        print(json.dumps({"shape": spec, **{k: round(min(v), 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
