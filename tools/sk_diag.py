#!/usr/bin/env python3
"""Stream-K debugging aid: per 256x256 tile max error of gemm_nt_preact (y, z) and gemm_nt against fp32."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from kubeflow_rm_amd.ops import gemm  # noqa: E402


def tiles_bad(out, ref, tag):
    M, N = ref.shape
    bad = []
    for tm in range(0, M, 256):
        for tn in range(0, N, 256):
            e = (out[tm:tm + 256, tn:tn + 256].float() - ref[tm:tm + 256, tn:tn + 256]).abs().max().item()
            s = ref[tm:tm + 256, tn:tn + 256].abs().max().item()
            if e > 1e-2 * s + 1e-2:
                bad.append((tm // 256, tn // 256, round(e, 3)))
    print(tag, "bad tiles", len(bad), bad[:12], flush=True)
    for tm, tn, _ in bad[:3]:  # where inside the tile
        d = (out[tm * 256:tm * 256 + 256, tn * 256:tn * 256 + 256].float()
             - ref[tm * 256:tm * 256 + 256, tn * 256:tn * 256 + 256]).abs()
        thr = 1e-2 * ref.abs().max().item() + 1e-2
        rows = (d > thr).any(1).nonzero().flatten().tolist()
        cols = (d > thr).any(0).nonzero().flatten().tolist()
        print("   tile", (tm, tn), "bad elems", int((d > thr).sum()), "rows", len(rows), rows[:20], "cols", len(cols),
              cols[:40], flush=True)


def fit_segments(z, a, b, bias, M, N, K, G=256, show=6):
    """Least-squares coefficients of each stream-K segment's contribution in the SK tiles' output
    (1 = added once; 0 = missing; 2 = doubled)."""
    tiles_m, tiles_n = -(-M // 256), -(-N // 256)
    nwg, KT = tiles_m * tiles_n, -(-K // 64)
    T_dp = nwg - nwg % G
    units = (nwg - T_dp) * KT
    q = -(-units // G)
    per_group = 4 * tiles_n
    koff = K - KT * 64
    shown = 0
    for t in range(nwg - T_dp):
        w = T_dp + t
        gg = w // per_group
        fm = gg * 4
        gmm = min(tiles_m - fm, 4)
        tm, tn = fm + (w % per_group) % gmm, (w % per_group) // gmm
        m0, n0 = min(tm * 256, M - 256), min(tn * 256, N - 256)
        segs = []
        v = t * KT
        while v < (t + 1) * KT:
            blk = v // q
            ve = min((blk + 1) * q, (t + 1) * KT)
            segs.append((blk, v - t * KT, ve - t * KT))
            v = ve
        cols = []
        for blk, k0, k1 in segs:
            lo, hi = max(0, koff + 64 * k0), koff + 64 * k1
            cols.append((a[m0:m0 + 256, lo:hi].float() @ b[n0:n0 + 256, lo:hi].float().t()).flatten())
        X = torch.stack(cols, 1)
        y = (z[m0:m0 + 256, n0:n0 + 256].float() - bias[n0:n0 + 256].float()).flatten()
        c = torch.linalg.lstsq(X.cpu(), y.cpu().unsqueeze(1)).solution.flatten()
        print("tile", t, (tm, tn), "segs", segs, "coef", [round(x, 3) for x in c.tolist()], flush=True)
        shown += 1
        if shown >= show:
            break


def main():
    M, N, K = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "3072x3072x4096").split("x"))
    g = torch.Generator(device="cuda").manual_seed(0)
    a = ((torch.rand(M, K, generator=g, device="cuda") * 2 - 1)).to(torch.bfloat16)
    b = ((torch.rand(N, K, generator=g, device="cuda") * 2 - 1) * 0.1).to(torch.bfloat16)
    bias = ((torch.rand(N, generator=g, device="cuda") * 2 - 1)).to(torch.bfloat16)
    z_ref = a.float() @ b.float().t() + bias.float()
    y_ref = torch.nn.functional.gelu(z_ref, approximate="tanh")
    print("plan", gemm.streamk_plan(M, N, K), flush=True)
    for sk in (True, False):
        gemm.STREAMK = sk
        y, z = gemm.gemm_nt_preact(a, b, bias, "gelu_tanh")
        torch.cuda.synchronize()
        tiles_bad(z, z_ref, f"sk={sk} z")
        if sk:
            fit_segments(z, a, b, bias, M, N, K)
        tiles_bad(y, y_ref, f"sk={sk} y")
        c = gemm.gemm_nt(a, b, bias=bias, act="gelu_tanh")
        tiles_bad(c, y_ref, f"sk={sk} gemm_nt")


if __name__ == "__main__":
    main()
