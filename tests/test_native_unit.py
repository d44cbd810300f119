"""Native C++ unit tests (native/tests/*.cc on the tests/harness.h macro harness), run by CTest:
one ctest entry per suite (json, yaml, util, selector, gpu, http) — JSON merge / RFC 6902 /
strategic patches, YAML documents, quantities and time, label / field selectors, xGMI placement
and quota accounting, HTTP streaming, Upgrade hand-over and TLS with an in-process certificate."""
import shutil
import subprocess
from pathlib import Path

import pytest

BUILD = Path(__file__).resolve().parent.parent / "build" / "native"


@pytest.fixture(scope="module")
def built():
    from tests.conftest import _ensure_native
    _ensure_native()
    if not (BUILD / "tests" / "kfamd_native_tests").exists():
        from kubeflow_rm_amd import _build
        _build.build_native()
    return BUILD


@pytest.mark.skipif(shutil.which("ctest") is None, reason="ctest not installed")
def test_ctest_suites(built):
    r = subprocess.run(["ctest", "--output-on-failure"], cwd=built, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "100% tests passed" in r.stdout


def test_harness_reports_every_case(built):
    r = subprocess.run([str(built / "tests" / "kfamd_native_tests")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout and r.stdout.count("ok   ") >= 14
