import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X / gfx950) and the built HIP kernels")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu() -> bool:
    if not os.path.exists("/dev/kfd"):
        return False
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


HAS_GPU = _has_gpu()


def pytest_collection_modifyitems(config, items):
    if HAS_GPU:
        return
    skip = pytest.mark.skip(reason="no AMD GPU visible (/dev/kfd absent)")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def _ensure_native() -> None:
    """Build the native control plane (and the kernel library it links) when missing."""
    lib = ROOT / "kubeflow_rm_amd" / "lib"
    bin_dir = ROOT / "kubeflow_rm_amd" / "bin"
    if (lib / "libkfcore_capi.so").exists() and (bin_dir / "kflite").exists():
        return
    from kubeflow_rm_amd import _build
    if not (lib / "libkfamd_kernels.so").exists():
        _build.build_kernels()
    _build.build_native()


@pytest.fixture(scope="session")
def native():
    _ensure_native()
    from kubeflow_rm_amd import native as nat
    return nat


@pytest.fixture(scope="module")
def cluster():
    """One kube-lite control plane (all controllers, synthetic 8x MI355X node) per test module."""
    _ensure_native()
    from kubeflow_rm_amd.cluster import LocalCluster
    cl = LocalCluster(env={"ENABLE_CULLING": "false", "USE_ISTIO": "true"})
    cl.start()
    yield cl
    cl.stop()
