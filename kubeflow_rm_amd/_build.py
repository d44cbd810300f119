"""In-tree build of every native artefact of the framework.

* ``libkfamd_kernels.so`` — the hand-written gfx950 HIP kernels (``kernels/*.hip``), compiled with
  ``hipcc --offload-arch=gfx950`` and loaded by :mod:`kubeflow_rm_amd.ops` through ctypes (one HIP
  runtime shared with torch: both resolve the ``libamdhip64.so.7`` SONAME).
* ``native/`` — the C++17 control plane (API server, controllers, admission, KFAM, kubelet, GPU
  topology/allocator) and the in-pod readiness op, built with CMake + Ninja into ``build/native``
  and installed into ``kubeflow_rm_amd/bin``.

Everything is built in-tree so that the artefacts travel with a ``gpurun`` snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNEL_DIR = ROOT / "kernels"
PKG_DIR = ROOT / "kubeflow_rm_amd"
LIB_DIR = PKG_DIR / "lib"
BIN_DIR = PKG_DIR / "bin"
BUILD_DIR = ROOT / "build"
KERNEL_LIB = LIB_DIR / "libkfamd_kernels.so"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KFAMD_OFFLOAD_ARCH", "gfx950")
HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-mcode-object-version=5",
    "-Wall",
    "-Wno-unused-variable",
    "-Wno-unused-function",
]


def _run(cmd: list[str], cwd: Path | None = None) -> None:
    proc = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(
            f"command failed ({proc.returncode}): {' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}"
        )


def _newer(target: Path, sources: list[Path]) -> bool:
    if not target.exists():
        return False
    t = target.stat().st_mtime
    return all(s.stat().st_mtime <= t for s in sources)


DIAG_LIB = LIB_DIR / "libkfamd_kernels_diag.so"


def build_diag_kernels() -> Path:
    """Diagnostic GEMM build (in-kernel s_memtime stamps + ablation switches: tools/w4_diag.py).
    Kept out of libkfamd_kernels.so: compiled only on request, with -DKFAMD_DIAG."""
    src = KERNEL_DIR / "gemm_bf16_w4.hip"
    obj = BUILD_DIR / "kernels" / "gemm_bf16_w4_diag.o"
    obj.parent.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    _run([HIPCC, *HIP_FLAGS, "-DKFAMD_DIAG", "-I", str(KERNEL_DIR), "-c", str(src), "-o", str(obj)])
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(DIAG_LIB), str(obj)])
    return DIAG_LIB


# per-translation-unit compiler flags. attention_bf16.hip: MFMA results in VGPRs unless the budget
# forces AGPRs — the default AGPR form shuttled S / dP through 972 v_accvgpr moves per backward
# iteration at D = 128 (329 with this); gpt-1b backward 665 -> 636 us, the forward ~1 % faster, the
# D = 64 backward level (profiles/r5n_attn_ab, tools/attn_ab.py)
TU_FLAGS = {"attention_bf16.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def build_kernels(force: bool = False, jobs: int = 8) -> Path:
    """Compile kernels/*.hip and kernels/tu/*.hip (one template variant per translation unit, so the
    slow ones build in parallel) for gfx950 and link libkfamd_kernels.so (incremental)."""
    srcs = sorted(KERNEL_DIR.glob("*.hip")) + sorted((KERNEL_DIR / "tu").glob("*.hip"))
    headers = sorted(KERNEL_DIR.glob("*.h"))
    obj_dir = BUILD_DIR / "kernels"
    obj_dir.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)

    # kfamd_build_info() names the kernel sources it was built from (content hash), so a loaded
    # library identifies itself even when only other translation units were recompiled
    src_hash = hashlib.sha256(b"".join(p.read_bytes() for p in [*srcs, *headers])).hexdigest()[:12]
    stamp = obj_dir / "src_hash"
    hash_changed = not stamp.exists() or stamp.read_text().strip() != src_hash

    def compile_one(src: Path) -> Path:
        obj = obj_dir / (src.stem + ".o")
        info = src.name == "kfamd_info.hip"
        deps = [src, *headers, *([Path(__file__)] if src.name in TU_FLAGS else [])]
        if force or not _newer(obj, deps) or (info and hash_changed):
            extra = [f'-DKFAMD_SRC_HASH="{src_hash}"'] if info else []
            extra += TU_FLAGS.get(src.name, [])
            _run([HIPCC, *HIP_FLAGS, *extra, "-I", str(KERNEL_DIR), "-c", str(src), "-o", str(obj)])
            check_object_kernels(src, obj)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs)))) as ex:
        objs = list(ex.map(compile_one, srcs))
    stamp.write_text(src_hash)
    if force or not _newer(KERNEL_LIB, objs):
        tmp = KERNEL_LIB.with_suffix(".so.tmp")
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)])
        check_kernel_library(tmp)
        os.replace(tmp, KERNEL_LIB)
    return KERNEL_LIB


# kernel families every production library must carry (kernel-descriptor symbols of the embedded
# gfx950 code object). A host compile that drops a template's kernel stubs still links and still
# exits 0, leaving a library whose launches fail at run time: refuse to install it.
REQUIRED_KERNELS = ("gemm_w4", "gemm_nt_256p", "gemm_nt_128", "norm_fwd_wave", "ln_bwd_dx_wave",
                    "allreduce_oneshot")


def kernel_descriptors(lib: Path) -> set[str]:
    import re
    data = Path(lib).read_bytes()
    return {m.group(1).decode() for m in re.finditer(rb"([A-Za-z0-9_]+)\.kd\x00", data)}


def check_object_kernels(src: Path, obj: Path) -> None:
    """A translation unit that defines __global__ kernels must carry their gfx950 descriptors.
    hipcc 7.2 can drop a TU's launch stubs AND its whole device bundle with exit status 0 (seen with
    a struct member as a buffer builtin's soffset, kernels/gemm_w4.h): catch it per object."""
    import re
    text = src.read_text()
    if not re.search(r"^\s*(template\s*<[^;{]*>\s*)?__global__", text, re.M) and \
            not any(k in text for k in ("gemm_w4<", "KFW4_NT_ENTRY(", "KFW4_SK_ENTRY(", "KFW4_FIX_ENTRY(")):
        return
    if not kernel_descriptors(obj):
        raise RuntimeError(f"{obj}: compiled from {src.name} but holds no gfx950 kernel descriptors "
                           "(device bundle dropped by the compiler)")


def check_kernel_library(lib: Path) -> None:
    names = kernel_descriptors(lib)
    missing = [k for k in REQUIRED_KERNELS if not any(k in n for n in names)]
    if missing:
        raise RuntimeError(f"{lib}: no gfx950 kernel descriptors for {missing} ({len(names)} kernels found)")
    # the other face of the dropped-stub bug: a host pass that lost a kernel's launch stub leaves an
    # undefined __device_stub__ reference, and the library fails to load (gemm_w4.h FASTK notes)
    nm = subprocess.run(["nm", "-D", "--undefined-only", str(lib)], capture_output=True, text=True)
    stubs = [ln.split()[-1] for ln in nm.stdout.splitlines() if "__device_stub__" in ln]
    if stubs:
        raise RuntimeError(f"{lib}: undefined kernel launch stubs (host pass dropped them): {stubs[:3]}")


SANITIZER_CXX = "/opt/rocm/lib/llvm/bin/clang++"


def build_native(force: bool = False, jobs: int = 8, build_type: str = "Release",
                 sanitize: str = "") -> Path:
    """Configure + build the C++ control plane with CMake/Ninja; install binaries into bin/."""
    src = ROOT / "native"
    if not (src / "CMakeLists.txt").exists():
        return BIN_DIR
    bdir = BUILD_DIR / ("native" if not sanitize else f"native-{sanitize}")
    if force and bdir.exists():
        shutil.rmtree(bdir)
    bdir.mkdir(parents=True, exist_ok=True)
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    cfg = ["cmake", *gen, str(src), f"-DCMAKE_BUILD_TYPE={build_type}",
           f"-DKFAMD_SANITIZE={sanitize}", f"-DKFAMD_BIN_DIR={BIN_DIR if not sanitize else bdir / 'bin'}",
           f"-DKFAMD_KERNEL_DIR={KERNEL_DIR}", f"-DKFAMD_OFFLOAD_ARCH={ARCH}"]
    if sanitize and Path(SANITIZER_CXX).exists():
        # GCC 11's libtsan has no pthread_cond_clockwait interceptor, which libstdc++ 11 uses for
        # every condition_variable::wait_for: it then reports "double lock" + phantom races on
        # every queue. ROCm's LLVM ships current tsan/asan/ubsan runtimes that intercept it.
        cfg.append(f"-DCMAKE_CXX_COMPILER={SANITIZER_CXX}")
    if not (bdir / "CMakeCache.txt").exists():
        _run(cfg, cwd=bdir)
    _run(["cmake", "--build", str(bdir), "-j", str(jobs)], cwd=bdir)
    return BIN_DIR if not sanitize else bdir / "bin"


def build_all(force: bool = False) -> None:
    build_kernels(force=force)
    build_native(force=force)


if __name__ == "__main__":  # python -m kubeflow_rm_amd._build [--force] [kernels|native]
    args = sys.argv[1:]
    force = "--force" in args
    what = [a for a in args if not a.startswith("--")] or ["kernels", "native"]
    if "kernels" in what:
        print(build_kernels(force=force))
    if "native" in what:
        print(build_native(force=force))
