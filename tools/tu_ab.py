#!/usr/bin/env python3
"""Build A/B of any kernel translation units: the kernel library re-linked with the named TUs compiled
under extra flags (-D knobs), one library per variant (kubeflow_rm_amd/lib/tuab/).

  python tools/tu_ab.py --name pd0 --tus tu/w4_dgrad_act,tu/w4_nt_none --flags=-DKFW4_RES_PD=0
  KFAMD_KERNEL_LIB=kubeflow_rm_amd/lib/tuab/libkfamd_kernels_pd0.so python tools/dact_bench.py

(tools/attn_ab.py is the attention-specific form with named variants.)
"""
from __future__ import annotations

import argparse
import shlex
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
OUT = ROOT / "kubeflow_rm_amd" / "lib" / "tuab"


def build(name: str, tus: list[str], flags: list[str]) -> Path:
    from kubeflow_rm_amd import _build as B
    B.build_kernels()
    srcs = {str(s.relative_to(B.KERNEL_DIR).with_suffix("")): s
            for s in sorted(B.KERNEL_DIR.glob("*.hip")) + sorted((B.KERNEL_DIR / "tu").glob("*.hip"))}
    missing = [t for t in tus if t not in srcs]
    if missing:
        raise SystemExit(f"unknown translation units {missing}; have {sorted(srcs)}")
    OUT.mkdir(parents=True, exist_ok=True)
    objs = []
    for rel, src in srcs.items():
        if rel in tus:
            obj = OUT / f"{rel.replace('/', '_')}_{name}.o"
            tu_flags = B.TU_FLAGS.get(src.name, [])
            subprocess.run([B.HIPCC, *B.HIP_FLAGS, *tu_flags, *flags, "-I", str(B.KERNEL_DIR), "-c", str(src), "-o",
                            str(obj)], check=True)
            objs.append(obj)
        else:
            objs.append(B.BUILD_DIR / "kernels" / (src.stem + ".o"))
    lib = OUT / f"libkfamd_kernels_{name}.so"
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib), *map(str, objs)],
                   check=True)
    B.check_kernel_library(lib)
    print("built", lib.relative_to(ROOT), flush=True)
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", required=True)
    ap.add_argument("--tus", required=True, help="comma list of TUs relative to kernels/, no suffix")
    ap.add_argument("--flags", default="", help="extra hipcc flags for those TUs")
    a = ap.parse_args()
    build(a.name, [t for t in a.tus.split(",") if t], shlex.split(a.flags))


if __name__ == "__main__":
    main()
