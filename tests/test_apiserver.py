"""kube-lite API server semantics (the envtest equivalent).

Covers what the reference's envtest suites rely on from a real kube-apiserver: CRUD with
resourceVersion concurrency, generation, status subresource, merge / JSON / strategic patches,
dry-run, finalizers, ownerReference GC, namespace lifecycle, CRD schema validation + multi-version
("None" conversion), label / field selectors, watch, RBAC SubjectAccessReview.
"""
import threading
import time

import pytest

from kubeflow_rm_amd.client import ApiException


@pytest.fixture(scope="module")
def c(cluster):
    cl = cluster.client
    for ns in ("t-api", "t-gc"):
        cl.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    return cl


def _cm(name, ns="t-api", data=None, **md):
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": ns, **md}, "data": data or {"a": "1"}}


def test_create_get_conflict_and_rv(c):
    o = c.create(_cm("cm1"))
    assert o["metadata"]["uid"] and o["metadata"]["resourceVersion"]
    with pytest.raises(ApiException) as e:
        c.create(_cm("cm1"))
    assert e.value.status == 409
    stale = dict(o)
    o["data"] = {"a": "2"}
    o2 = c.update(o)
    assert int(o2["metadata"]["resourceVersion"]) > int(stale["metadata"]["resourceVersion"])
    stale["data"] = {"a": "3"}
    with pytest.raises(ApiException) as e:
        c.update(stale)
    assert e.value.status == 409
    assert c.get("v1", "ConfigMap", "cm1", "t-api")["data"] == {"a": "2"}


def test_not_found_and_namespace_required(c):
    with pytest.raises(ApiException) as e:
        c.get("v1", "ConfigMap", "nope", "t-api")
    assert e.value.status == 404
    with pytest.raises(ApiException) as e:
        c.create(_cm("x", ns="no-such-ns"))
    assert e.value.status == 404


def test_patches(c):
    c.create(_cm("cm-p", data={"a": "1", "b": "2"}))
    o = c.patch("v1", "ConfigMap", "cm-p", {"data": {"b": None, "c": "3"}}, "t-api", "merge")
    assert o["data"] == {"a": "1", "c": "3"}
    o = c.patch("v1", "ConfigMap", "cm-p", [{"op": "replace", "path": "/data/a", "value": "9"}], "t-api", "json")
    assert o["data"]["a"] == "9"
    with pytest.raises(ApiException) as e:
        c.patch("v1", "ConfigMap", "cm-p", [{"op": "test", "path": "/data/a", "value": "0"}], "t-api", "json")
    assert e.value.status in (409, 422)


def test_strategic_merge_patch_containers(c):
    dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d1", "namespace": "t-api"},
           "spec": {"replicas": 0, "selector": {"matchLabels": {"app": "d1"}},
                    "template": {"metadata": {"labels": {"app": "d1"}},
                                 "spec": {"containers": [{"name": "a", "image": "x:1"}, {"name": "b", "image": "y:1"}]}}}}
    c.create(dep)
    o = c.patch("apps/v1", "Deployment", "d1", {"spec": {"template": {"spec": {"containers": [{"name": "b", "image": "y:2"}]}}}},
                "t-api", "strategic")
    imgs = {x["name"]: x["image"] for x in o["spec"]["template"]["spec"]["containers"]}
    assert imgs == {"a": "x:1", "b": "y:2"}


def test_dry_run_does_not_persist(c):
    c.create(_cm("cm-dry"), dry_run=True)
    assert not c.exists("v1", "ConfigMap", "cm-dry", "t-api")


WIDGET_CRD = {
    "apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
    "metadata": {"name": "widgets.example.com"},
    "spec": {"group": "example.com", "scope": "Namespaced",
             "names": {"kind": "Widget", "plural": "widgets", "singular": "widget", "listKind": "WidgetList"},
             "versions": [{"name": "v1", "served": True, "storage": True, "subresources": {"status": {}},
                           "schema": {"openAPIV3Schema": {"type": "object", "properties": {
                               "spec": {"type": "object", "required": ["size"],
                                        "properties": {"size": {"type": "integer", "minimum": 1}}},
                               "status": {"type": "object", "properties": {"ready": {"type": "boolean"}}}}}}}]}}


def test_dynamic_crd_generation_and_status_subresource(c):
    c.create(WIDGET_CRD)
    w = {"apiVersion": "example.com/v1", "kind": "Widget", "metadata": {"name": "w1", "namespace": "t-api"}, "spec": {"size": 1}}
    deadline = time.time() + 5
    while True:  # the new resource is served as soon as the CRD is established
        try:
            o = c.create(w)
            break
        except ApiException as e:
            if e.status != 404 or time.time() > deadline:
                raise
            time.sleep(0.05)
    assert o["metadata"]["generation"] == 1
    o["metadata"]["labels"] = {"x": "y"}
    o = c.update(o)
    assert o["metadata"]["generation"] == 1  # metadata-only change
    o["spec"]["size"] = 2
    o = c.update(o)
    assert o["metadata"]["generation"] == 2
    # spec changes through /status are ignored, status changes through the main resource too
    o["status"] = {"ready": True}
    o["spec"]["size"] = 3
    s = c.update_status(o)
    assert s["status"]["ready"] is True and s["spec"]["size"] == 2
    s["status"] = {"ready": False}
    s = c.update(s)
    assert s["status"]["ready"] is True
    with pytest.raises(ApiException) as e:
        c.create({**w, "metadata": {"name": "w2", "namespace": "t-api"}, "spec": {"size": 0}})
    assert e.value.status == 422


def test_crd_schema_validation_and_versions(c):
    bad = {"apiVersion": "kubeflow.org/v1beta1", "kind": "Notebook", "metadata": {"name": "bad", "namespace": "t-api"},
           "spec": {"template": {"spec": {"containers": []}}}}
    with pytest.raises(ApiException) as e:
        c.create(bad)
    assert e.value.status == 422
    good = {"apiVersion": "kubeflow.org/v1beta1", "kind": "Notebook", "metadata": {"name": "vb", "namespace": "t-api",
                                                                                    "annotations": {"kubeflow-resource-stopped": "x"}},
            "spec": {"template": {"spec": {"containers": [{"name": "vb", "image": "i"}]}}}}
    c.create(good)
    # the same object served at every version ("None" conversion)
    for v in ("v1", "v1beta1", "v1alpha1"):
        o = c.get(f"kubeflow.org/{v}", "Notebook", "vb", "t-api")
        assert o["apiVersion"] == f"kubeflow.org/{v}"
    tb = {"apiVersion": "tensorboard.kubeflow.org/v1alpha1", "kind": "Tensorboard",
          "metadata": {"name": "tb", "namespace": "t-api"}, "spec": {}}
    with pytest.raises(ApiException) as e:
        c.create(tb)
    assert e.value.status == 422


def test_label_and_field_selectors(c):
    for i in range(4):
        c.create(_cm(f"sel-{i}", labels={"grp": "a" if i % 2 else "b", "i": str(i)}))
    names = lambda r: sorted(x["metadata"]["name"] for x in r["items"])  # noqa: E731
    assert names(c.list("v1", "ConfigMap", "t-api", label_selector="grp=a")) == ["sel-1", "sel-3"]
    assert names(c.list("v1", "ConfigMap", "t-api", label_selector="grp in (a,b),i notin (0,1)")) == ["sel-2", "sel-3"]
    assert names(c.list("v1", "ConfigMap", "t-api", field_selector="metadata.name=sel-2")) == ["sel-2"]


def test_list_pagination(c):
    for i in range(5):
        c.create(_cm(f"page-{i}", labels={"page": "y"}))
    r = c.list("v1", "ConfigMap", "t-api", label_selector="page=y", limit=2)
    assert len(r["items"]) == 2 and r["metadata"].get("continue")


def test_finalizers_block_deletion(c):
    c.create(_cm("fin", finalizers=["example.com/hold"]))
    c.delete("v1", "ConfigMap", "fin", "t-api")
    o = c.get("v1", "ConfigMap", "fin", "t-api")
    assert o["metadata"]["deletionTimestamp"]
    o["metadata"]["finalizers"] = []
    c.update(o)
    c.wait_gone("v1", "ConfigMap", "fin", "t-api", timeout=5)


def test_owner_reference_garbage_collection(c):
    owner = c.create(_cm("owner", ns="t-gc"))
    ref = {"apiVersion": "v1", "kind": "ConfigMap", "name": "owner", "uid": owner["metadata"]["uid"], "controller": True,
           "blockOwnerDeletion": True}
    c.create(_cm("child1", ns="t-gc", ownerReferences=[ref]))
    c.create(_cm("child2", ns="t-gc", ownerReferences=[ref]))
    c.delete("v1", "ConfigMap", "owner", "t-gc")
    c.wait_gone("v1", "ConfigMap", "child1", "t-gc", timeout=10)
    c.wait_gone("v1", "ConfigMap", "child2", "t-gc", timeout=10)
    # orphan propagation keeps dependents
    owner = c.create(_cm("owner2", ns="t-gc"))
    ref["uid"], ref["name"] = owner["metadata"]["uid"], "owner2"
    c.create(_cm("child3", ns="t-gc", ownerReferences=[ref]))
    c.delete("v1", "ConfigMap", "owner2", "t-gc", propagation_policy="Orphan")
    c.wait_gone("v1", "ConfigMap", "owner2", "t-gc", timeout=10)
    time.sleep(0.3)
    assert "ownerReferences" not in c.get("v1", "ConfigMap", "child3", "t-gc")["metadata"] or \
        not c.get("v1", "ConfigMap", "child3", "t-gc")["metadata"]["ownerReferences"]


def test_namespace_deletion_cascades(c):
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "t-doomed"}})
    c.create(_cm("x", ns="t-doomed"))
    c.delete("v1", "Namespace", "t-doomed")
    c.wait_gone("v1", "Namespace", "t-doomed", None, timeout=15)
    with pytest.raises(ApiException):
        c.get("v1", "ConfigMap", "x", "t-doomed")


def test_watch_streams_events(c):
    rv = c.list("v1", "ConfigMap", "t-api")["metadata"]["resourceVersion"]
    seen = []

    def reader():
        for ev in c.watch("v1", "ConfigMap", "t-api", resource_version=rv, timeout_seconds=5):
            seen.append((ev["type"], ev["object"]["metadata"]["name"]))
            if len(seen) >= 3:
                return

    t = threading.Thread(target=reader)
    t.start()
    time.sleep(0.2)
    o = c.create(_cm("w1"))
    o["data"] = {"z": "1"}
    c.update(o)
    c.delete("v1", "ConfigMap", "w1", "t-api")
    t.join(10)
    assert seen == [("ADDED", "w1"), ("MODIFIED", "w1"), ("DELETED", "w1")]


def test_rbac_subject_access_review(c):
    rb = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
          "metadata": {"name": "bob-edit", "namespace": "t-api"},
          "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "kubeflow-edit"},
          "subjects": [{"kind": "User", "name": "bob@example.com", "apiGroup": "rbac.authorization.k8s.io"}]}
    c.create(rb)
    r = c.subject_access_review("bob@example.com", "create", "kubeflow.org", "notebooks", "t-api")
    assert r["status"]["allowed"] is True
    r = c.subject_access_review("bob@example.com", "create", "kubeflow.org", "notebooks", "t-gc")
    assert r["status"]["allowed"] is False
    r = c.subject_access_review("mallory@example.com", "list", "", "pods", "t-api")
    assert r["status"]["allowed"] is False
