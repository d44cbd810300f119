"""Image family: Dockerfile chains resolve inside images/ or to pinned upstream bases,
the Makefile builds every image in dependency order, s6 scripts are executable bash that parses,
and nothing CUDA/NVIDIA remains (MI355X-only family)."""
import re
import stat
import subprocess
from pathlib import Path

import pytest

IMAGES = Path(__file__).resolve().parent.parent / "images"
UPSTREAM = {"ubuntu:22.04", "python:3.11-slim"}


def _dockerfiles():
    return sorted(IMAGES.glob("*/Dockerfile"))


def _froms(df: Path):
    out = []
    for line in df.read_text().splitlines():
        m = re.match(r"FROM\s+(\S+)", line.strip())
        if m:
            out.append(m.group(1))
    return out


def test_every_image_dir_has_dockerfile_and_make_target():
    mk = (IMAGES / "Makefile").read_text()
    dirs = sorted(p.name for p in IMAGES.iterdir() if p.is_dir())
    for d in dirs:
        assert (IMAGES / d / "Dockerfile").is_file(), d
        assert re.search(rf"^{re.escape(d)}:", mk, re.M), f"no make target for {d}"


@pytest.mark.parametrize("df", _dockerfiles(), ids=lambda p: p.parent.name)
def test_from_chain_resolves(df):
    stages = set()
    for ref in _froms(df):
        name = ref.split(":")[0]
        if ref.startswith("${BASE_IMG_REGISTRY}/"):
            parent = name.split("/", 1)[1]
            assert (IMAGES / parent / "Dockerfile").is_file(), f"{df}: FROM {ref}"
            mk = (IMAGES / "Makefile").read_text()
            assert re.search(rf"^{re.escape(df.parent.name)}:.*\b{re.escape(parent)}\b", mk, re.M), \
                f"{df.parent.name} must depend on {parent} in the Makefile"
        elif ref.startswith("rocm/") or ref in UPSTREAM or name in stages:
            pass
        else:
            raise AssertionError(f"{df}: unexpected base {ref}")
        text = df.read_text()
        for m in re.finditer(r"FROM\s+\S+\s+AS\s+(\S+)", text, re.I):
            stages.add(m.group(1))


def test_no_cuda_anywhere():
    for p in IMAGES.rglob("*"):
        if p.is_file():
            t = p.read_text(errors="ignore").lower()
            assert "cuda" not in t and "nvidia" not in t, p


def test_s6_scripts_are_executable_bash():
    scripts = [p for p in IMAGES.rglob("*") if p.is_file() and ("/s6/" in str(p))]
    assert len(scripts) >= 6
    for p in scripts:
        assert p.stat().st_mode & stat.S_IXUSR, f"{p} not executable"
        assert p.read_text().startswith("#!/command/with-contenv bash"), p
        subprocess.run(["bash", "-n", str(p)], check=True)


# --- one ROCm release per image (VERDICT r4 missing #2) ----------------------------------------
_ROCM_REFS = [
    re.compile(r"download\.pytorch\.org/whl/(?:nightly/)?rocm(\d+)\.(\d+)"),  # torch wheel index
    re.compile(r"repo\.radeon\.com/rocm/manylinux/rocm-rel-(\d+)\.(\d+)"),    # AMD's TF / torch wheels
    re.compile(r"repo\.radeon\.com/rocm/apt/(\d+)\.(\d+)"),                   # ROCm apt repo
    re.compile(r"rocm/dev-ubuntu-\d+\.\d+:(\d+)\.(\d+)"),                     # builder stages
    re.compile(r"\+rocm(\d+)\.(\d+)"),                                        # pinned local versions
]


def _resolve_args(text: str) -> tuple[dict, str]:
    """ARG defaults with ${VAR} expanded in order, and the text with every ${VAR} expanded."""
    args: dict[str, str] = {}

    def sub(s: str) -> str:
        return re.sub(r"\$\{(\w+)\}", lambda m: args.get(m.group(1), m.group(0)), s)

    for line in text.splitlines():
        m = re.match(r"\s*ARG\s+(\w+)=(\S+)", line)
        if m:
            args[m.group(1)] = sub(m.group(2))
    return args, sub(text)


def rocm_mismatches(text: str) -> list[str]:
    """Every ROCm release a Dockerfile pulls from whose major differs from its ROCM_VERSION."""
    args, expanded = _resolve_args(text)
    want = args.get("ROCM_VERSION")
    if want is None:
        return []
    major = want.split(".")[0]
    bad = []
    for rx in _ROCM_REFS:
        for m in rx.finditer(expanded):
            if m.group(1) != major:
                bad.append(f"{m.group(0)} (ROCM_VERSION={want})")
    return sorted(set(bad))


@pytest.mark.parametrize("df", _dockerfiles(), ids=lambda p: p.parent.name)
def test_wheel_indexes_match_the_image_rocm_release(df):
    """A torch / TF wheel index or builder stage of another ROCm major than the image's
    ROCM_VERSION would map a second HIP runtime next to the kernels' libamdhip64.so.7."""
    assert rocm_mismatches(df.read_text()) == [], df


def test_rocm_mismatch_check_catches_the_round4_recipe():
    bad = ("ARG ROCM_VERSION=7.0\nFROM rocm/dev-ubuntu-22.04:${ROCM_VERSION}-complete AS builder\n"
           "ARG TORCH_INDEX=https://download.pytorch.org/whl/rocm6.4\nRUN pip install --index-url ${TORCH_INDEX} torch\n")
    assert rocm_mismatches(bad) == ["download.pytorch.org/whl/rocm6.4 (ROCM_VERSION=7.0)"]
    good = bad.replace("rocm6.4", "rocm${ROCM_VERSION}")
    assert rocm_mismatches(good) == []


def test_pytorch_image_smoke_loads_the_kernel_library():
    """The build-time smoke must load libkfamd_kernels.so (not only import Python modules) and run
    the one-runtime check."""
    text = (IMAGES / "jupyter-pytorch-rocm" / "Dockerfile").read_text()
    assert "ops.lib()" in text and "kubeflow_rm_amd.ops.runtime_check" in text


def test_one_hip_runtime_mapped_after_torch_and_kernels():
    """The same check on this machine's torch: exactly one libamdhip64 after both loads."""
    import subprocess
    import sys
    root = IMAGES.parent
    p = subprocess.run([sys.executable, "-m", "kubeflow_rm_amd.ops.runtime_check"], cwd=root,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
