#!/usr/bin/env python3
"""Flash-attention build A/B: the kernel library re-linked with kernels/attention_bf16.hip compiled
under other flags / -D knobs, one library per variant (kubeflow_rm_amd/lib/attnab/).

  python tools/attn_ab.py --build [--variants a,b]   # host: compile + link every variant
  KFAMD_KERNEL_LIB=kubeflow_rm_amd/lib/attnab/libkfamd_kernels_<v>.so python tools/attn_bench.py ...

The GPU side is the ordinary tooling with ``KFAMD_KERNEL_LIB`` pointing at a variant (ops/_lib.py), so
a variant runs the same numerics tests and the same interleaved bench as production
(tools/runs/r5n_attn_ab.sh).
"""
from __future__ import annotations

import argparse
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
OUT = ROOT / "kubeflow_rm_amd" / "lib" / "attnab"


def _variants():
    from kubeflow_rm_amd import _build as B
    prod = B.TU_FLAGS.get("attention_bf16.hip", [])
    return {
        "prod": prod,  # the production flags and knob defaults
        "head": prod,  # git HEAD's attention source with the production flags
        "sepdelta": [*prod, "-DKFATT_DQ_DELTA=0"],  # the separate delta prologue kernel
        "dkdv4_64": [*prod, "-DKFATT_DKDV8_64=0"],  # D = 64 with the 4-wave dK / dV kernel
        "dkdv4": [*prod, "-DKFATT_DKDV8=0"],  # D = 128 dK / dV with the 4-wave kernel (one wave per SIMD)
        # the compiler's default AGPR form: S / dP shuttled through v_accvgpr moves
        "agprform": [],
        "guarded": [*prod, "-DKFATT_BUF=0", "-DKFATT_DMA=0", "-DKFATT_DQ_SPLIT=0"],  # per-row guards, atomics
        "atomics": [*prod, "-DKFATT_DQ_SPLIT=0"],  # dQ by fp32 atomics inside the dK / dV kernel
        "atomics_regstage": [*prod, "-DKFATT_DQ_SPLIT=0", "-DKFATT_DMA=0"],  # ... Q / dO register-staged
        "atomics_dropped": [*prod, "-DKFATT_DQ_SPLIT=0", "-DKFATT_ABL=1"],  # timing only: atomics dropped
        "fwd_dma": [*prod, "-DKFATT_FWD_DMA=1"],  # forward K / V by LDS-DMA
        "nolpt": [*prod, "-DKFATT_LPT=0"],  # head-major block order (no longest-first across heads)
        "nofpair": [*prod, "-DKFATT_FWD_PAIR=0"],  # causal forward: one query block per workgroup
        "dqpair": [*prod, "-DKFATT_DQ_PAIR=1"],  # dQ kernel: heavy + light query block per workgroup
        "fwd8": [*prod, "-DKFATT_FWD_PP=0", "-DKFATT_FWD_NW=8"],  # forward: the unstaggered 8-wave attn_fwd
        "fwdold": [*prod, "-DKFATT_FWD_PP=0"],  # forward: attn_fwd (4 waves, two workgroups per CU)
        "fabl1": [*prod, "-DKFATT_FWD_ABL=1"],  # timing only: attn_fwd_pp without K / V staging
        "fabl2": [*prod, "-DKFATT_FWD_ABL=2"],  # timing only: attn_fwd_pp without the per-tile barrier
        "fabl3": [*prod, "-DKFATT_FWD_ABL=3"],  # timing only: neither
        "pf1": [*prod, "-DKFATT_FWD_PF2=0"],  # attn_fwd_pp with K / V loads one tile ahead
        "nofence": [*prod, "-DKFATT_FWD_FENCE=0"],  # attn_fwd_pp without the phase fences
        "nowide": [*prod, "-DKFATT_FWD_WIDE=0"],  # attn_fwd_pp with 8-B O stores
        "bnowide": [*prod, "-DKFATT_BWD_WIDE=0"],  # dQ / dK / dV with 8-B stores
        "nopxp": [*prod, "-DKFATT_FWD_PXP=0"],  # attn_fwd_pp pairs without the cross-pass prefetch
        "prio": [*prod, "-DKFATT_FWD_PRIO=1"],  # attn_fwd_pp with waves 4-7 at priority 1
        "babl1": [*prod, "-DKFATT_DKDV_ABL=1"],  # timing only: dK / dV kernel without Q / dO staging
        "babl2": [*prod, "-DKFATT_DKDV_ABL=2"],  # timing only: ... without the per-tile barrier
        "babl4": [*prod, "-DKFATT_DKDV_ABL=4"],  # timing only: ... one K / V fragment read per tile
        "babl7": [*prod, "-DKFATT_DKDV_ABL=7"],  # timing only: all three
        "nopp": [*prod, "-DKFATT_FWD_PP=0"],  # forward by attn_fwd everywhere
        "ra4": [*prod, "-DKFATT_FWD_RA=4"],  # attn_fwd_pp: LDS reads pinned 4 MFMAs ahead (r6v_ra)
        "split": [*prod, "-DKFATT_FWD_SPLIT=1"],  # attn_fwd_pp softmax max / sum as 4 chains
        "fra0": [*prod, "-DKFATT_FWD_RA=0"],  # attn_fwd_pp reads in the compiler's order
        "fra1": [*prod, "-DKFATT_FWD_RA=1"],
        "fra3": [*prod, "-DKFATT_FWD_RA=3"],
        "f4ra1": [*prod, "-DKFATT_FWD4_RA=1"],  # attn_fwd (4 waves: D = 64, small grids) with pinned reads
        "f4ra2": [*prod, "-DKFATT_FWD4_RA=2"],
        "dra1": [*prod, "-DKFATT_DQ_RA=1"],  # attn_bwd_dq_split (D = 128): reads pinned 1 MFMA ahead
        "dra2": [*prod, "-DKFATT_DQ_RA=2"],
        "bra1": [*prod, "-DKFATT_BWD_RA=1"],  # attn_bwd_dkdv8 (D = 128): reads pinned 1 MFMA ahead
        "bra2": [*prod, "-DKFATT_BWD_RA=2"],  # ... 2 MFMAs ahead
    }


VARIANTS = _variants()


def build(names):
    from kubeflow_rm_amd import _build as B
    B.build_kernels()
    # the objects of the current sources (build/kernels also keeps objects of retired ones)
    srcs = sorted(B.KERNEL_DIR.glob("*.hip")) + sorted((B.KERNEL_DIR / "tu").glob("*.hip"))
    others = [B.BUILD_DIR / "kernels" / (s.stem + ".o") for s in srcs if s.stem != "attention_bf16"]
    OUT.mkdir(parents=True, exist_ok=True)
    for n in names:
        obj = OUT / f"attention_bf16_{n}.o"
        src = B.KERNEL_DIR / "attention_bf16.hip"
        if n == "head":  # the committed source (git HEAD), for an A/B against the working tree
            src = OUT / "attention_bf16_head.hip"
            src.write_text(subprocess.run(["git", "-C", str(ROOT), "show", "HEAD:kernels/attention_bf16.hip"],
                                          capture_output=True, text=True, check=True).stdout)
        subprocess.run([B.HIPCC, *B.HIP_FLAGS, *VARIANTS[n], "-I", str(B.KERNEL_DIR), "-c", str(src), "-o", str(obj)],
                       check=True)
        lib = OUT / f"libkfamd_kernels_{n}.so"
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib), str(obj),
                        *map(str, others)], check=True)
        B.check_kernel_library(lib)
        print("built", lib.relative_to(ROOT), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    a = ap.parse_args()
    names = [v for v in a.variants.split(",") if v]
    if a.build:
        build(names)


if __name__ == "__main__":
    main()
