"""One HIP runtime per process: the kernel library must resolve ``libamdhip64`` to the file torch mapped.

``ops/_lib.py`` loads ``libkfamd_kernels.so`` after torch so its ``NEEDED libamdhip64.so.7`` binds to
the runtime torch already mapped (same SONAME). A torch wheel built for another ROCm major bundles
``libamdhip64.so.6`` instead; the loader would then map a second runtime from /opt/rocm and torch's
``hipStream_t`` values would be handed to a runtime that never created them. Loading libraries does
not initialise the GPU, so this check runs at image build time (no GPU) and in the CPU test suite:

    python -m kubeflow_rm_amd.ops.runtime_check

exits non-zero, naming the files, when more than one ``libamdhip64`` is mapped after both loads.
Counterpart of the reference's CUDA-matched wheel pin
(/root/reference/components/example-notebook-servers/jupyter-pytorch-cuda/Dockerfile:9-23).
"""
from __future__ import annotations

import json
import sys


def hip_runtime_files() -> list[str]:
    """Distinct ``libamdhip64`` files mapped into this process."""
    out = set()
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and "libamdhip64" in parts[-1]:
                out.add(parts[-1])
    return sorted(out)


def check() -> dict:
    import torch
    from kubeflow_rm_amd.ops import _lib
    _lib.lib()  # torch first, then the kernel library (raises if it cannot load)
    files = hip_runtime_files()
    return {"torch": torch.__version__, "torch_hip": getattr(torch.version, "hip", None),
            "libamdhip64": files, "ok": len(files) == 1}


def main() -> int:
    rep = check()
    print(json.dumps(rep))
    if not rep["ok"]:
        print(f"error: {len(rep['libamdhip64'])} HIP runtimes mapped after torch + libkfamd_kernels.so: "
              f"{rep['libamdhip64']} (torch wheel and kernel build target different ROCm majors)", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
