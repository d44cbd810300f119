"""``kfctl apply`` = kubectl's client-side apply: last-applied-configuration,
three-way strategic merge patch, "unchanged" without a request, ``--dry-run`` from a real diff.

End to end on the ODH integration workflow's own Notebook
(/root/reference/.github/workflows/odh_notebook_controller_integration_test.yaml:228-271): apply it,
let the ODH webhook inject the oauth-proxy sidecar, re-apply the identical manifest — a no-op — then
remove one env var and change the image: exactly those fields change, the sidecar stays.
"""
import copy
import json
from pathlib import Path

import pytest
import yaml

from kubeflow_rm_amd.apply import LAST_APPLIED, three_way_patch, with_last_applied

FIX = Path(__file__).parent / "fixtures" / "odh_ci_minimal_notebook.yaml"
NB = "kubeflow.org/v1"


# ---- the patch computation ------------------------------------------------------------------------
def _pod(containers, **extra):
    return {"spec": {"template": {"spec": {"containers": containers, **extra}}}}


def test_unchanged_manifest_gives_an_empty_patch_despite_webhook_additions():
    man = _pod([{"name": "nb", "image": "a", "env": [{"name": "X", "value": "1"}]}])
    live = _pod([{"name": "nb", "image": "a", "env": [{"name": "X", "value": "1"}], "volumeMounts": [{"mountPath": "/ca"}]},
                 {"name": "oauth-proxy", "image": "p"}], volumes=[{"name": "ca"}])
    assert three_way_patch(man, man, live) == {}


def test_removed_env_var_is_deleted_by_key():
    old = _pod([{"name": "nb", "env": [{"name": "A", "value": "1"}, {"name": "B", "value": "2"}]}])
    new = _pod([{"name": "nb", "env": [{"name": "A", "value": "1"}]}])
    live = copy.deepcopy(old)
    live["spec"]["template"]["spec"]["containers"].append({"name": "oauth-proxy"})
    p = three_way_patch(old, new, live)
    assert p == {"spec": {"template": {"spec": {"containers": [{"name": "nb", "env": [{"name": "B", "$patch": "delete"}]}]}}}}


def test_changed_image_patches_only_that_container():
    old = _pod([{"name": "nb", "image": "a"}, {"name": "side", "image": "s"}])
    new = _pod([{"name": "nb", "image": "b"}, {"name": "side", "image": "s"}])
    assert three_way_patch(old, new, old) == {"spec": {"template": {"spec": {"containers": [{"name": "nb", "image": "b"}]}}}}


def test_field_removed_from_manifest_is_deleted_but_server_fields_are_kept():
    old = {"metadata": {"labels": {"a": "1", "b": "2"}}, "spec": {"x": 1, "y": 2}}
    new = {"metadata": {"labels": {"a": "1"}}, "spec": {"x": 1}}
    live = {"metadata": {"labels": {"a": "1", "b": "2", "server": "s"}, "uid": "u"}, "spec": {"x": 1, "y": 2, "z": 3},
            "status": {"ready": True}}
    assert three_way_patch(old, new, live) == {"metadata": {"labels": {"b": None}}, "spec": {"y": None}}


def test_service_ports_merge_by_port_and_plain_lists_replace():
    old = {"spec": {"ports": [{"port": 80, "targetPort": 8080}], "args": ["a"]}}
    new = {"spec": {"ports": [{"port": 80, "targetPort": 9090}], "args": ["b"]}}
    assert three_way_patch(old, new, old) == {"spec": {"ports": [{"port": 80, "targetPort": 9090}], "args": ["b"]}}


def test_last_applied_annotation_is_the_bare_manifest():
    m = with_last_applied({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x"}, "data": {"k": "v"}})
    assert json.loads(m["metadata"]["annotations"][LAST_APPLIED]) == {
        "apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x"}, "data": {"k": "v"}}


# ---- end to end: the ODH CI notebook -------------------------------------------------------------
@pytest.fixture(scope="module")
def cl():
    from kubeflow_rm_amd.cluster import LocalCluster
    from tests.conftest import _ensure_native
    _ensure_native()
    cluster = LocalCluster(env={"ENABLE_CULLING": "false", "USE_ISTIO": "false"})
    cluster.start()
    yield cluster
    cluster.stop()


def _kfctl(cl, path, *extra):
    import contextlib
    import io
    from kubeflow_rm_amd import kfctl
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = kfctl.main(["apply", "-f", str(path), "--server", cl.url, *extra])
    assert rc == 0
    return buf.getvalue()


def _containers(o):
    return o["spec"]["template"]["spec"]["containers"]


def _settled(c, timeout=20.0, quiet=1.5):
    """The Notebook once its controllers stopped writing it (status updates bump resourceVersion)."""
    import time
    deadline = time.time() + timeout
    last = c.get(NB, "Notebook", "minimal-notebook", "default")
    since = time.time()
    while time.time() < deadline:
        time.sleep(0.25)
        o = c.get(NB, "Notebook", "minimal-notebook", "default")
        if o["metadata"]["resourceVersion"] != last["metadata"]["resourceVersion"]:
            last, since = o, time.time()
        elif time.time() - since >= quiet:
            break
    return last


def test_reapplying_the_odh_ci_notebook_is_a_noop(cl, tmp_path):
    c = cl.client
    out = _kfctl(cl, FIX)
    assert "Notebook/minimal-notebook -n default created" in out, out
    nb = c.wait_for(NB, "Notebook", "minimal-notebook", "default",
                    lambda o: [x["name"] for x in _containers(o)] == ["minimal-notebook", "oauth-proxy"]
                    and "kubeflow-resource-stopped" not in (o["metadata"].get("annotations") or {}), timeout=30)
    assert LAST_APPLIED in nb["metadata"]["annotations"]
    nb = _settled(c)
    rv, gen, containers = nb["metadata"]["resourceVersion"], nb["metadata"].get("generation"), _containers(nb)
    out = _kfctl(cl, FIX)
    assert "Notebook/minimal-notebook -n default unchanged" in out, out
    again = c.get(NB, "Notebook", "minimal-notebook", "default")
    assert again["metadata"]["resourceVersion"] == rv and again["metadata"].get("generation") == gen
    assert _containers(again) == containers
    assert "notebooks.opendatahub.io/update-pending" not in again["metadata"]["annotations"]
    # a server-side dry run of the same manifest reports the same from a real diff
    assert "unchanged (server dry run)" in _kfctl(cl, FIX, "--dry-run")

    # one env var added, then removed again: exactly that env var goes
    docs = list(yaml.safe_load_all(FIX.read_text()))
    man = docs[0]
    plus = copy.deepcopy(man)
    plus["spec"]["template"]["spec"]["containers"][0]["env"].append({"name": "EXTRA", "value": "1"})
    (tmp_path / "plus.yaml").write_text(yaml.safe_dump(plus))
    assert "configured" in _kfctl(cl, tmp_path / "plus.yaml", "--dry-run")
    assert c.get(NB, "Notebook", "minimal-notebook", "default")["metadata"].get("generation") == gen  # dry run
    assert "configured" in _kfctl(cl, tmp_path / "plus.yaml")
    env = [e["name"] for e in _containers(c.get(NB, "Notebook", "minimal-notebook", "default"))[0]["env"]]
    assert "EXTRA" in env and "NOTEBOOK_ARGS" in env
    assert "configured" in _kfctl(cl, FIX)
    after = c.get(NB, "Notebook", "minimal-notebook", "default")
    assert [e["name"] for e in _containers(after)[0]["env"]] == [e for e in env if e != "EXTRA"]
    assert [x["name"] for x in _containers(after)] == ["minimal-notebook", "oauth-proxy"]

    # a changed image updates only that container; the injected sidecar is untouched
    proxy = [x for x in _containers(after) if x["name"] == "oauth-proxy"][0]
    img = copy.deepcopy(man)
    img["spec"]["template"]["spec"]["containers"][0]["image"] = "quay.io/thoth-station/s2i-minimal-notebook:v0.3.1"
    (tmp_path / "img.yaml").write_text(yaml.safe_dump(img))
    assert "configured" in _kfctl(cl, tmp_path / "img.yaml")
    final = c.get(NB, "Notebook", "minimal-notebook", "default")
    assert _containers(final)[0]["image"].endswith(":v0.3.1")
    assert [x for x in _containers(final) if x["name"] == "oauth-proxy"][0] == proxy
