"""Frontend unit tests (the reference's Karma/Jasmine specs for kubeflow-common-lib) run on node."""
import shutil
import subprocess
from pathlib import Path

import pytest

NODE = shutil.which("node") or shutil.which("nodejs")


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_common_frontend_runtime():
    script = Path(__file__).parent / "js" / "test_kf.js"
    r = subprocess.run([NODE, str(script)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(NODE is None, reason="node not installed")
@pytest.mark.parametrize("app", ["jupyter", "tensorboards", "volumes", "dashboard"])
def test_frontend_sources_parse(app):
    root = Path(__file__).resolve().parent.parent / "kubeflow_rm_amd" / "webapps" / app / "static"
    for js in root.rglob("*.js"):
        r = subprocess.run([NODE, "-e", "require('vm').createScript(require('fs').readFileSync(process.argv[1], 'utf8'))",
                            str(js)], capture_output=True, text=True, timeout=30)
        assert r.returncode == 0, f"{js}: {r.stderr}"


@pytest.mark.skipif(NODE is None, reason="node not installed")
@pytest.mark.skipif(not Path("/root/reference/components/crud-web-apps").exists(), reason="reference fixtures absent")
def test_jwa_dom_wiring():
    """DOM-level: the JWA page on a fake DOM (tests/js/fakedom.js) — table action buttons, confirm
    dialogs, the spawner's GPU vendor select and the POSTed body (tests/js/test_dom.js)."""
    script = Path(__file__).parent / "js" / "test_dom.js"
    r = subprocess.run([NODE, str(script), "/root/reference/components/crud-web-apps"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
