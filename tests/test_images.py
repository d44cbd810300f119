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
