"""Deployment manifests and the kustomize-lite renderer that builds them.

* renderer semantics: strategic merge by name, JSON patch, generators with content-hash names and
  rewritten references, namespace / prefix / labels / images, overlay ``behavior: merge``;
* every base and overlay under manifests/ renders, without duplicate object ids;
* every container image resolves to a kube-lite kubelet recipe other than the catch-all (so the
  manifests are runnable on kube-lite as well as documenting a real deployment);
* manifests/crds equals the native CRD registry (no drift);
* the full example applies to a kube-lite API server (server-side dry run: schema, defaulting,
  admission) in dependency order.
"""
import json
import re
from pathlib import Path

import pytest
import yaml

from kubeflow_rm_amd import kfctl, kustomize

ROOT = Path(__file__).resolve().parent.parent
MANIFESTS = ROOT / "manifests"


def _kust_dirs():
    return sorted(p.parent for p in MANIFESTS.rglob("kustomization.yaml"))


def test_strategic_merge_and_json_patch():
    base = {"spec": {"containers": [{"name": "a", "image": "x", "env": [{"name": "K", "value": "1"}]},
                                    {"name": "b", "image": "y"}], "replicas": 1}}
    patch = {"spec": {"containers": [{"name": "a", "env": [{"name": "K", "value": "2"}, {"name": "L", "value": "3"}]},
                                     {"name": "b", "$patch": "delete"}], "replicas": None}}
    out = kustomize.strategic_merge(base, patch)
    assert out == {"spec": {"containers": [{"name": "a", "image": "x", "env": [{"name": "K", "value": "2"},
                                                                               {"name": "L", "value": "3"}]}]}}
    out = kustomize.json_patch(base, [{"op": "add", "path": "/spec/containers/0/args", "value": ["--x"]},
                                      {"op": "replace", "path": "/spec/replicas", "value": 3},
                                      {"op": "remove", "path": "/spec/containers/1"}])
    assert out["spec"]["replicas"] == 3 and len(out["spec"]["containers"]) == 1
    assert out["spec"]["containers"][0]["args"] == ["--x"]


def test_generators_prefix_namespace_images(tmp_path):
    (tmp_path / "base").mkdir()
    (tmp_path / "base" / "app.yaml").write_text(yaml.safe_dump_all([
        {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web"},
         "spec": {"selector": {"matchLabels": {"app": "web"}}, "template": {"metadata": {"labels": {"app": "web"}},
                  "spec": {"serviceAccountName": "sa", "containers": [{"name": "c", "image": "kfamd/web:1",
                                                                       "envFrom": [{"configMapRef": {"name": "cfg"}}]}]}}}},
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "sa"}},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding", "metadata": {"name": "crb"},
         "roleRef": {"kind": "ClusterRole", "name": "r", "apiGroup": "rbac.authorization.k8s.io"},
         "subjects": [{"kind": "ServiceAccount", "name": "sa"}]}]))
    (tmp_path / "base" / "kustomization.yaml").write_text(yaml.safe_dump({
        "namePrefix": "p-", "resources": ["app.yaml"], "configMapGenerator": [{"name": "cfg", "literals": ["A=1"]}]}))
    (tmp_path / "ov").mkdir()
    (tmp_path / "ov" / "kustomization.yaml").write_text(yaml.safe_dump({
        "namespace": "team", "resources": ["../base"], "commonLabels": {"tier": "x"},
        "images": [{"name": "kfamd/web", "newName": "reg.local/web", "newTag": "2"}],
        "configMapGenerator": [{"name": "cfg", "behavior": "merge", "literals": ["B=2"]}]}))
    objs = {o["kind"]: o for o in kustomize.build(tmp_path / "ov")}
    cm, dep = objs["ConfigMap"], objs["Deployment"]
    assert cm["data"] == {"A": "1", "B": "2"} and re.fullmatch(r"p-cfg-[0-9a-z]{10}", cm["metadata"]["name"])
    assert cm["metadata"]["namespace"] == "team" and "annotations" not in cm["metadata"]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["envFrom"][0]["configMapRef"]["name"] == cm["metadata"]["name"]
    assert c["image"] == "reg.local/web:2"
    assert dep["spec"]["template"]["spec"]["serviceAccountName"] == "p-sa"
    assert dep["spec"]["selector"]["matchLabels"] == {"app": "web", "tier": "x"}
    crb = objs["ClusterRoleBinding"]
    assert "namespace" not in crb["metadata"] and crb["subjects"][0] == {"kind": "ServiceAccount", "name": "p-sa",
                                                                          "namespace": "team"}
    # a data change changes the hash
    (tmp_path / "ov" / "kustomization.yaml").write_text((tmp_path / "ov" / "kustomization.yaml").read_text()
                                                         .replace("B=2", "B=3"))
    cm2 = [o for o in kustomize.build(tmp_path / "ov") if o["kind"] == "ConfigMap"][0]
    assert cm2["metadata"]["name"] != cm["metadata"]["name"]


@pytest.mark.parametrize("d", _kust_dirs(), ids=lambda p: str(p.relative_to(MANIFESTS)))
def test_every_kustomization_renders(d):
    objs = kustomize.build(d)
    assert objs
    ids = [(o["apiVersion"].split("/")[0] if "/" in o["apiVersion"] else "", o["kind"],
            o["metadata"].get("namespace"), o["metadata"]["name"]) for o in objs]
    assert len(ids) == len(set(ids)), [i for i in ids if ids.count(i) > 1]
    for o in objs:
        assert o.get("apiVersion") and o.get("kind") and o["metadata"].get("name"), o
        if o["kind"] in kustomize.CLUSTER_SCOPED:
            assert "namespace" not in o["metadata"], o["metadata"]


def _recipes():
    src = (ROOT / "native" / "node" / "kubelet.cc").read_text()
    body = src[src.index('kDefaultRecipes = R"(') + len('kDefaultRecipes = R"('):]
    return json.loads(body[:body.index(')";')])


def test_images_resolve_to_kubelet_recipes():
    recipes = _recipes()
    objs = kustomize.build(MANIFESTS / "example")
    seen = 0
    for o in objs:
        ps = kustomize._pod_spec(o)
        if ps is None:
            continue
        for c in list(kustomize._containers(ps)):
            key = " ".join(["cmd:" + x for x in c.get("command", [])] + [c["image"]])
            hit = next(r for r in recipes if re.search(r["match"], key, re.I))
            assert hit["match"] != ".*", (o["metadata"]["name"], c["image"])
            seen += 1
    assert seen >= 10


def test_crd_manifests_match_native_registry(native):
    by_name = {c["metadata"]["name"]: c for c in native.call("builtin_crds")}
    files = list((MANIFESTS / "crds").rglob("*_*.yaml"))
    assert len(files) == len(by_name)
    for f in files:
        doc = yaml.safe_load(f.read_text())
        assert doc["spec"] == by_name[doc["metadata"]["name"]]["spec"], f


def test_example_applies_server_side_dry_run(cluster):
    objs = kustomize.build(MANIFESTS / "example")
    ordered = kfctl.apply_order(objs)
    assert ordered[0]["kind"] == "Namespace" and ordered[-1]["kind"].endswith("WebhookConfiguration")
    # the namespaces must exist for namespaced dry runs: apply the Namespace objects for real
    kfctl.apply(cluster.client, [o for o in objs if o["kind"] == "Namespace"], log=None)
    lines = kfctl.apply(cluster.client, objs, dry_run=True, log=None)
    assert len(lines) == len(objs)
    assert any("Deployment/notebook-controller-deployment -n kubeflow" in x for x in lines)
    # nothing but the namespace was stored
    assert not cluster.client.exists("apps/v1", "Deployment", "notebook-controller-deployment", "kubeflow")


def test_kfctl_build_cli(capsys):
    assert kfctl.main(["build", str(MANIFESTS / "centraldashboard" / "base")]) == 0
    docs = [d for d in yaml.safe_load_all(capsys.readouterr().out) if d]
    cm = [d for d in docs if d["kind"] == "ConfigMap"][0]
    assert cm["metadata"]["name"] == "centraldashboard-config"
    assert json.loads(cm["data"]["links"])["menuLinks"][0]["link"] == "/jupyter/"
