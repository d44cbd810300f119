"""Frontend <-> backend contract.

1. The pages' pure parts run on node against the reference's Cypress fixtures and the assertions of
   its Cypress specs (tests/js/test_apps.js; fixtures read in place from
   /root/reference/components/crud-web-apps/*/frontend/cypress/fixtures).
2. Our JWA / TWA / VWA backends answer with the JSON shapes those fixtures record (same envelope,
   same row keys, same nested status / gpus objects), checked against live kube-lite objects.
3. The request body the JWA spawner builds in JS (JWA.buildBody over JWA.formDefaults of OUR
   /api/config) is accepted by the backend and produces the requested Notebook (CPU / memory
   limits from the form-cpu-ram fields, MI355X GPUs, workspace PVC).

Known fixture drift: jupyter's config.json has a top-level ``storageClass`` that the reference's
spawner_ui_config.yaml does not define; volumes' pvcs.json stores ``viewer`` as a bare string while the reference
backend returns ``{status, url}`` (volumes/backend/apps/default/routes/get.py:24-27); our backend
follows the backend, the page accepts both (tests/js/test_apps.js).
"""
import json
import os
import shutil
import subprocess
import time
from pathlib import Path

import pytest

FIXTURES = Path("/root/reference/components/crud-web-apps")
NODE = shutil.which("node") or shutil.which("nodejs")
ROOT = Path(__file__).resolve().parent.parent
USER = "contract-owner@example.com"
NS = "contract-owner"

needs_fixtures = pytest.mark.skipif(not FIXTURES.exists(), reason="reference Cypress fixtures not present")
needs_node = pytest.mark.skipif(NODE is None, reason="node not installed")


def _fixture(app, name):
    return json.loads((FIXTURES / app / "frontend/cypress/fixtures" / f"{name}.json").read_text())


@needs_fixtures
@needs_node
def test_pages_against_cypress_fixtures():
    r = subprocess.run([NODE, str(ROOT / "tests/js/test_apps.js"), str(FIXTURES)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


def _h(token=None):
    h = {"kubeflow-userid": USER}
    if token:
        h["X-XSRF-TOKEN"] = token
    return h


def _client(app):
    app.testing = True
    tc = app.test_client()
    assert tc.get("/", headers=_h()).status_code == 200
    return tc, tc.get_cookie("XSRF-TOKEN").value


@pytest.fixture(scope="module")
def apps(cluster):
    os.environ["APP_SECURE_COOKIES"] = "false"
    from kubeflow_rm_amd.webapps import jupyter, tensorboards, volumes
    from kubeflow_rm_amd.webapps.crud_backend import config, k8s

    c = cluster.client
    c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": NS},
              "spec": {"owner": {"kind": "User", "name": USER}}})
    c.wait_for("rbac.authorization.k8s.io/v1", "RoleBinding", "namespaceAdmin", NS, lambda o: True, timeout=15)
    k8s.set_client(c)
    yield {"jwa": _client(jupyter.create_app(config.Config(mode="prod"))),
           "twa": _client(tensorboards.create_app(config.Config(mode="prod"))),
           "vwa": _client(volumes.create_app(config.Config(mode="prod"))), "c": c}
    os.environ.pop("APP_SECURE_COOKIES", None)


def _shape(v):
    """Key structure of a JSON value (dict keys recursively; list -> shape of its first item)."""
    if isinstance(v, dict):
        return {k: _shape(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_shape(v[0])] if v and isinstance(v[0], (dict, list)) else []
    return None


def _keys(d):
    return set(d) if isinstance(d, dict) else set()


def _poll(fn, pred, timeout=40):
    deadline = time.time() + timeout
    while True:
        v = fn()
        if pred(v) or time.time() > deadline:
            return v
        time.sleep(0.3)


@needs_fixtures
def test_jwa_config_shape_matches_fixture(apps):
    tc, _ = apps["jwa"]
    ours = tc.get("/api/config", headers=_h()).get_json()
    ref = _fixture("jupyter", "config")
    assert _keys(ours) >= _keys(ref)
    # the fixture's top-level "storageClass" is not in the reference's spawner_ui_config.yaml (the
    # class is per volume: newPvc.spec.storageClassName, spawner_ui_config.yaml:160)
    assert _keys(ours["config"]) >= _keys(ref["config"]) - {"storageClass"}, _keys(ref["config"]) - _keys(ours["config"])
    for k, v in ref["config"].items():
        if isinstance(v, dict):
            assert _keys(ours["config"][k]) >= _keys(v) - {"readOnly"}, k
    ws = ours["config"]["workspaceVolume"]["value"]
    assert set(ws) >= {"mount", "newPvc"}
    assert ours["config"]["gpus"]["value"]["vendors"][0]["limitsKey"] == "amd.com/gpu"


@needs_fixtures
def test_jwa_notebook_rows_and_poddefaults_match_fixture_shapes(apps):
    tc, token = apps["jwa"]
    c = apps["c"]
    c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "PodDefault", "metadata": {"name": "access-ml-pipeline", "namespace": NS},
              "spec": {"desc": "Allow access to Kubeflow Pipelines", "selector": {"matchLabels": {"access-ml-pipeline": "true"}},
                       "env": [{"name": "KF_PIPELINES_SA_TOKEN_PATH", "value": "/var/run/secrets/t"}]}})
    cfg = tc.get("/api/config", headers=_h()).get_json()["config"]
    body = {"name": "shape", "namespace": NS, "image": cfg["image"]["value"], "imagePullPolicy": "IfNotPresent",
            "serverType": "jupyter", "cpu": "0.5", "memory": "1Gi", "gpus": {"num": "none"}, "tolerationGroup": "none",
            "affinityConfig": "none", "configurations": ["access-ml-pipeline"], "shm": True, "datavols": []}
    r = tc.post(f"/api/namespaces/{NS}/notebooks", json=body, headers=_h(token))
    assert r.status_code == 200, r.get_json()
    ours = _poll(lambda: tc.get(f"/api/namespaces/{NS}/notebooks", headers=_h()).get_json(),
                 lambda v: any(n["name"] == "shape" for n in v["notebooks"]))
    ref = _fixture("jupyter", "notebooks")
    assert _keys(ours) == _keys(ref)
    row = [n for n in ours["notebooks"] if n["name"] == "shape"][0]
    ref_row = ref["notebooks"][0]
    # MI355X additions to a row (the in-pod readiness op result, the xGMI placement) are additive
    assert _keys(row) - {"gpuReadiness", "gpuPlacement"} == _keys(ref_row), _keys(row) ^ _keys(ref_row)
    assert _keys(row["status"]) == _keys(ref_row["status"])
    assert _keys(row["gpus"]) == _keys(ref_row["gpus"])
    assert row["status"]["phase"] in {"ready", "waiting", "warning", "stopped", "terminating", "unavailable", "error"}
    pds = tc.get(f"/api/namespaces/{NS}/poddefaults", headers=_h()).get_json()
    ref_pd = _fixture("jupyter", "poddefaults")
    assert _keys(pds) == _keys(ref_pd)
    assert _keys(ref_pd["poddefaults"][0]) - _keys(pds["poddefaults"][0]) == set()
    assert pds["poddefaults"][0]["label"] == "access-ml-pipeline" and pds["poddefaults"][0]["desc"]


@needs_fixtures
def test_vwa_and_twa_rows_match_fixture_shapes(apps):
    vtc, vtok = apps["vwa"]
    ttc, ttok = apps["twa"]
    r = vtc.post(f"/api/namespaces/{NS}/pvcs", json={"name": "shape-pvc", "size": "1Gi", "mode": "ReadWriteOnce",
                                                   "class": "{empty}", "type": "empty"}, headers=_h(vtok))
    assert r.status_code == 200, r.get_json()
    ours = vtc.get(f"/api/namespaces/{NS}/pvcs", headers=_h()).get_json()
    ref = _fixture("volumes", "pvcs")
    assert _keys(ours) == _keys(ref)
    row = [p for p in ours["pvcs"] if p["name"] == "shape-pvc"][0]
    assert _keys(row) == _keys(ref["pvcs"][0])
    assert _keys(row["status"]) == _keys(ref["pvcs"][0]["status"])
    assert set(row["viewer"]) == {"status", "url"}  # the reference backend's shape (see module doc)
    r = ttc.post(f"/api/namespaces/{NS}/tensorboards", json={"name": "shape-tb", "logspath": "pvc://shape-pvc/logs",
                                                           "configurations": []}, headers=_h(ttok))
    assert r.status_code == 200, r.get_json()
    ours = ttc.get(f"/api/namespaces/{NS}/tensorboards", headers=_h()).get_json()
    ref = _fixture("tensorboards", "tensorboards")
    assert _keys(ours) == _keys(ref)
    row = [t for t in ours["tensorboards"] if t["name"] == "shape-tb"][0]
    assert _keys(row) == _keys(ref["tensorboards"][0])
    assert _keys(row["status"]) == _keys(ref["tensorboards"][0]["status"])


@needs_node
def test_spawner_body_built_in_js_is_accepted_by_the_backend(apps):
    tc, token = apps["jwa"]
    c = apps["c"]
    cfg = tc.get("/api/config", headers=_h()).get_json()["config"]
    script = """
      global.window = global; global.document = {cookie: ""}; global.location = {search: ""};
      global.localStorage = {getItem: () => null, setItem: () => {}}; global.addEventListener = () => {}; global.parent = global;
      const path = require("path"); const W = path.join(process.argv[1], "kubeflow_rm_amd/webapps");
      global.kf = require(path.join(W, "crud_backend/static/kf.js"));
      const JWA = require(path.join(W, "jupyter/static/assets/app.js"));
      const cfg = JSON.parse(process.argv[2]);
      const f = JWA.formDefaults(cfg, "jsform");
      f.cpu = "1"; f.cpuLimit = "2"; f.memory = "2Gi"; f.memoryLimit = "3Gi";
      f.gpus = {num: "1", vendor: "amd.com/gpu"};
      f.workspace.size = "1"; f.workspace.accessMode = "ReadWriteOnce";
      f.datavols = [JWA.renameDataVolume(JWA.newDataVolume("jsform", 1), "jsform-data")];
      const errs = JWA.validate(f);
      if (errs.length) { console.error(errs.join("; ")); process.exit(2); }
      console.log(JSON.stringify(JWA.buildBody(f, cfg, process.argv[3])));
    """
    r = subprocess.run([NODE, "-e", script, str(ROOT), json.dumps(cfg), NS], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    body = json.loads(r.stdout)
    resp = tc.post(f"/api/namespaces/{NS}/notebooks", json=body, headers=_h(token))
    assert resp.status_code == 200, resp.get_json()
    nb = c.get("kubeflow.org/v1beta1", "Notebook", "jsform", NS)
    ctr = nb["spec"]["template"]["spec"]["containers"][0]
    assert ctr["resources"]["requests"]["cpu"] == "1" and ctr["resources"]["limits"]["cpu"] == "2"
    assert ctr["resources"]["requests"]["memory"] == "2Gi" and ctr["resources"]["limits"]["memory"] == "3Gi"
    assert ctr["resources"]["limits"]["amd.com/gpu"] == "1"
    assert {"name": "jsform-data", "mountPath": "/home/jovyan/jsform-data"} in ctr["volumeMounts"]
    assert c.get("v1", "PersistentVolumeClaim", "jsform-workspace", NS)["spec"]["accessModes"] == ["ReadWriteOnce"]


@needs_node
def test_custom_yaml_volumes_and_storage_class_accepted_by_the_backend(apps):
    """Custom (Advanced) volumes: the PVC / volume source the user typed as YAML (parsed by kf.parseYaml
    in node) and an explicit storage class reach the backend, which creates the PVC and mounts the
    source as written."""
    tc, token = apps["jwa"]
    c = apps["c"]
    cfg = tc.get("/api/config", headers=_h()).get_json()["config"]
    script = """
      global.window = global; global.document = {cookie: ""}; global.location = {search: ""};
      global.localStorage = {getItem: () => null, setItem: () => {}}; global.addEventListener = () => {}; global.parent = global;
      const path = require("path"); const W = path.join(process.argv[1], "kubeflow_rm_amd/webapps");
      global.kf = require(path.join(W, "crud_backend/static/kf.js"));
      const JWA = require(path.join(W, "jupyter/static/assets/app.js"));
      const cfg = JSON.parse(process.argv[2]);
      const f = JWA.formDefaults(cfg, "yamlform");
      f.workspace = Object.assign(f.workspace, {size: "1", accessMode: "ReadWriteOnce", useDefaultSC: false, storageClass: "standard"});
      let custom = JWA.toCustom(JWA.renameDataVolume(JWA.newDataVolume("yamlform", 1), "x"));
      custom = JWA.editCustom(custom, "metadata:\\n  name: yamlform-big\\nspec:\\n  accessModes: [ReadWriteOnce]\\n" +
                                      "  resources:\\n    requests:\\n      storage: 2Gi  # typed by hand\\n");
      let src = JWA.toCustom(Object.assign(JWA.newDataVolume("yamlform", 2), {type: "existing", existing: "x", mount: "/data/cfg"}));
      src = JWA.editCustom(src, "configMap:\\n  name: team-config\\n");
      f.datavols = [custom, src];
      const errs = JWA.validate(f);
      if (errs.length) { console.error(errs.join("; ")); process.exit(2); }
      console.log(JSON.stringify(JWA.buildBody(f, cfg, process.argv[3])));
    """
    r = subprocess.run([NODE, "-e", script, str(ROOT), json.dumps(cfg), NS], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    body = json.loads(r.stdout)
    resp = tc.post(f"/api/namespaces/{NS}/notebooks", json=body, headers=_h(token))
    assert resp.status_code == 200, resp.get_json()
    assert c.get("v1", "PersistentVolumeClaim", "yamlform-big", NS)["spec"]["resources"]["requests"]["storage"] == "2Gi"
    assert c.get("v1", "PersistentVolumeClaim", "yamlform-workspace", NS)["spec"]["storageClassName"] == "standard"
    vols = c.get("kubeflow.org/v1beta1", "Notebook", "yamlform", NS)["spec"]["template"]["spec"]["volumes"]
    assert any(v.get("configMap") == {"name": "team-config"} for v in vols), vols


DASH_FIXTURES = Path("/root/reference/components/centraldashboard-angular/frontend/cypress/fixtures")


@pytest.mark.skipif(not DASH_FIXTURES.exists(), reason="reference Cypress fixtures not present")
@needs_node
def test_dashboard_against_reference_specs():
    """cdb.js (namespace selection, URL mirroring, menu state, pages) vs the angular dashboard's
    namespace-selector / url-syncing Cypress specs and the Polymer dashboard's unit specs."""
    r = subprocess.run([NODE, str(ROOT / "tests/js/test_dashboard.js"), str(DASH_FIXTURES.parents[3])],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(not DASH_FIXTURES.exists(), reason="reference Cypress fixtures not present")
def test_dashboard_env_info_has_the_fixture_shape(monkeypatch):
    """/api/workgroup/env-info answers with envinfo.json's keys (the shell's only input besides links)."""
    from kubeflow_rm_amd.webapps import dashboard as dash
    want = json.loads((DASH_FIXTURES / "envinfo.json").read_text())

    class FakeKfam:
        def __init__(self, *_a, **_k):
            pass

        def is_cluster_admin(self, _u):
            return False

        def read_bindings(self, **_k):
            return [{"user": {"kind": "User", "name": "user"}, "referredNamespace": "kubeflow-user",
                     "roleRef": {"kind": "ClusterRole", "name": "admin"}}]

    class FakeK8s:
        def __init__(self, *_a, **_k):
            pass

        def get_platform_info(self):
            return {"provider": "other://", "providerName": "other", "kubeflowVersion": "mi355x"}

    monkeypatch.setattr(dash, "KfamClient", FakeKfam)
    monkeypatch.setattr(dash, "KubernetesService", FakeK8s)
    app = dash.create_app(k8s_client=object(), kfam_url="http://unused", metrics=None)
    got = app.test_client().get("/api/workgroup/env-info", headers={"kubeflow-userid": "user"}).get_json()
    assert set(got) == set(want)
    assert set(got["namespaces"][0]) == set(want["namespaces"][0])
    assert got["namespaces"][0]["role"] == "owner"
    shell = app.test_client().get("/")
    assert b"/cdb.js" in shell.data
    assert app.test_client().get("/cdb.js").status_code == 200


@needs_node
def test_gpu_vendor_contract_with_backend(apps):
    """T2: the spawner's vendor select is built from OUR /api/config vendor list and OUR /api/gpus
    (configured vendors some node reports capacity for: the kube-lite node advertises amd.com/gpu),
    so the MI355X vendor carries no "no GPUs in your cluster" tooltip, and a count without a vendor
    is refused in JS before it reaches the backend."""
    tc, _ = apps["jwa"]
    cfg = tc.get("/api/config", headers=_h()).get_json()["config"]
    vendors = tc.get("/api/gpus", headers=_h()).get_json()["vendors"]
    assert vendors == ["amd.com/gpu"]
    script = """
      global.window = global; global.document = {cookie: ""}; global.location = {search: ""};
      global.localStorage = {getItem: () => null, setItem: () => {}}; global.addEventListener = () => {}; global.parent = global;
      const path = require("path"); const W = path.join(process.argv[1], "kubeflow_rm_amd/webapps");
      global.kf = require(path.join(W, "crud_backend/static/kf.js"));
      const JWA = require(path.join(W, "jupyter/static/assets/app.js"));
      const cfg = JSON.parse(process.argv[2]), installed = new Set(JSON.parse(process.argv[3]));
      const f = JWA.formDefaults(cfg, "g");
      console.log(JSON.stringify({opts: JWA.vendorOptions(cfg, {num: "1", vendor: f.gpus.vendor}, installed),
                                  err: JWA.vendorError({num: "1", vendor: ""}), vendor: f.gpus.vendor}));
    """
    r = subprocess.run([NODE, "-e", script, str(ROOT), json.dumps(cfg), json.dumps(vendors)], capture_output=True,
                       text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out["vendor"] == "amd.com/gpu"
    assert 'value="amd.com/gpu" title="" selected>AMD Instinct MI355X' in out["opts"]
    assert out["err"] == "You must also specify the GPU Vendor for the assigned GPUs"
