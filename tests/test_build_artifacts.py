"""The built gfx950 kernel library carries every kernel family (kernel-descriptor symbols of its
embedded code object): a host compile that silently drops a kernel template's stubs still links,
so the build checks this too (kubeflow_rm_amd._build.check_kernel_library)."""
import pytest

from kubeflow_rm_amd import _build


@pytest.mark.skipif(not _build.KERNEL_LIB.exists(), reason="kernel library not built")
def test_kernel_library_has_every_kernel_family():
    _build.check_kernel_library(_build.KERNEL_LIB)
    names = _build.kernel_descriptors(_build.KERNEL_LIB)
    assert len(names) >= 40, len(names)
