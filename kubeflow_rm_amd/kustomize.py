"""kustomize-lite: render the repo's ``manifests/`` trees (the subset of kustomize they use).

The reference ships kustomize bases/overlays per component; ``kustomize`` itself is
not available here, so this module implements the fields those trees need:

* ``resources`` (YAML files, or directories holding a kustomization — bases and overlays)
* ``namespace`` (namespaced kinds only; ClusterRoleBinding / webhook service refs follow it)
* ``namePrefix`` / ``nameSuffix`` (with references in pod specs, RBAC and webhook configs updated)
* ``commonLabels`` (metadata, Deployment selectors and pod templates), ``commonAnnotations``
* ``images`` (``name`` -> ``newName`` / ``newTag`` / ``digest``)
* ``configMapGenerator`` / ``secretGenerator`` (``files``, ``literals``, ``envs``, ``behavior``),
  content-hash name suffixes unless ``generatorOptions.disableNameSuffixHash``, references rewritten
* ``patchesStrategicMerge`` / ``patches`` (strategic merge: maps merged, lists of named items merged
  by ``name``; RFC 6902 lists when the patch is a JSON-patch list with a ``target``)
* ``replicas`` (``name`` / ``count``)

``build(path)`` returns the objects in order; ``dump(objs)`` renders a multi-document YAML.
"""
from __future__ import annotations

import base64
import copy
import hashlib
import json
import os
from pathlib import Path
from typing import Any

import yaml

CLUSTER_SCOPED = {
    "Namespace", "ClusterRole", "ClusterRoleBinding", "CustomResourceDefinition", "MutatingWebhookConfiguration",
    "ValidatingWebhookConfiguration", "Profile", "StorageClass", "PersistentVolume", "Node", "APIService",
    "PriorityClass", "PodSecurityPolicy",
}
POD_TEMPLATE_KINDS = {"Deployment", "StatefulSet", "DaemonSet", "ReplicaSet", "Job"}


class KustomizeError(RuntimeError):
    pass


def _load_docs(path: Path) -> list[dict]:
    with open(path) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def _kustomization_file(d: Path) -> Path | None:
    for n in ("kustomization.yaml", "kustomization.yml", "Kustomization"):
        if (d / n).is_file():
            return d / n
    return None


def _hash(obj: dict) -> str:
    body = json.dumps({"kind": obj["kind"], "name": obj["metadata"]["name"], "data": obj.get("data", {})},
                      sort_keys=True, separators=(",", ":"))
    h = hashlib.sha256(body.encode()).hexdigest()
    return "".join(c for c in h if c not in "aeiou013")[:10]


def _pod_spec(obj: dict) -> dict | None:
    if obj.get("kind") == "Pod":
        return obj.get("spec")
    if obj.get("kind") in POD_TEMPLATE_KINDS:
        spec = obj.get("spec") or {}
        if obj["kind"] == "Job":
            return ((spec.get("template") or {}).get("spec"))
        return (spec.get("template") or {}).get("spec")
    if obj.get("kind") == "CronJob":
        return ((((obj.get("spec") or {}).get("jobTemplate") or {}).get("spec") or {}).get("template") or {}).get("spec")
    return None


def _containers(ps: dict):
    for key in ("initContainers", "containers"):
        for c in ps.get(key) or []:
            yield c


# ---- strategic merge ----------------------------------------------------------------------------
def strategic_merge(base: Any, patch: Any) -> Any:
    if isinstance(base, dict) and isinstance(patch, dict):
        out = dict(base)
        for k, v in patch.items():
            if v is None:
                out.pop(k, None)
            elif k in out:
                out[k] = strategic_merge(out[k], v)
            else:
                out[k] = copy.deepcopy(v)
        return out
    if isinstance(base, list) and isinstance(patch, list) and all(isinstance(x, dict) and "name" in x for x in base + patch):
        out = [copy.deepcopy(x) for x in base]
        idx = {x["name"]: i for i, x in enumerate(out)}
        for p in patch:
            if p.get("$patch") == "delete":
                out = [x for x in out if x["name"] != p["name"]]
                idx = {x["name"]: i for i, x in enumerate(out)}
            elif p["name"] in idx:
                out[idx[p["name"]]] = strategic_merge(out[idx[p["name"]]], p)
            else:
                out.append(copy.deepcopy(p))
                idx[p["name"]] = len(out) - 1
        return out
    return copy.deepcopy(patch)


def _json_pointer(path: str) -> list[str]:
    return [p.replace("~1", "/").replace("~0", "~") for p in path.lstrip("/").split("/")] if path else []


def json_patch(obj: dict, ops: list[dict]) -> dict:
    obj = copy.deepcopy(obj)
    for op in ops:
        parts = _json_pointer(op["path"])
        parent = obj
        for p in parts[:-1]:
            parent = parent[int(p)] if isinstance(parent, list) else parent.setdefault(p, {})
        last = parts[-1] if parts else None
        kind = op["op"]
        if kind in ("add", "replace"):
            if isinstance(parent, list):
                if last == "-":
                    parent.append(copy.deepcopy(op["value"]))
                elif kind == "add":
                    parent.insert(int(last), copy.deepcopy(op["value"]))
                else:
                    parent[int(last)] = copy.deepcopy(op["value"])
            else:
                parent[last] = copy.deepcopy(op["value"])
        elif kind == "remove":
            if isinstance(parent, list):
                parent.pop(int(last))
            else:
                parent.pop(last, None)
        else:
            raise KustomizeError(f"unsupported JSON patch op {kind!r}")
    return obj


# ---- generators ---------------------------------------------------------------------------------
def _generate(spec: dict, kind: str, base: Path, opts: dict) -> dict:
    data: dict[str, str] = {}
    for lit in spec.get("literals") or []:
        k, v = lit.split("=", 1)
        data[k] = v
    for f in spec.get("files") or []:
        key, _, rel = f.partition("=") if "=" in f else (os.path.basename(f), "", f)
        data[key] = (base / rel).read_text()
    for env in spec.get("envs") or spec.get(("env"), []) or []:
        for line in (base / env).read_text().splitlines():
            line = line.strip()
            if line and not line.startswith("#") and "=" in line:
                k, v = line.split("=", 1)
                data[k] = v
    obj = {"apiVersion": "v1", "kind": kind, "metadata": {"name": spec["name"]}}
    if kind == "Secret":
        obj["type"] = spec.get("type", "Opaque")
        obj["data"] = {k: base64.b64encode(v.encode()).decode() for k, v in data.items()}
    else:
        obj["data"] = data
    if spec.get("namespace"):
        obj["metadata"]["namespace"] = spec["namespace"]
    labels = {**(opts.get("labels") or {}), **((spec.get("options") or {}).get("labels") or {})}
    if labels:
        obj["metadata"]["labels"] = labels
    return obj


# ---- reference rewriting -------------------------------------------------------------------------
def _rename_refs(objs: list[dict], kind: str, old: str, new: str) -> None:
    for o in objs:
        ps = _pod_spec(o)
        if ps is not None:
            for v in ps.get("volumes") or []:
                if kind == "ConfigMap" and (v.get("configMap") or {}).get("name") == old:
                    v["configMap"]["name"] = new
                if kind == "Secret" and (v.get("secret") or {}).get("secretName") == old:
                    v["secret"]["secretName"] = new
                for src in ((v.get("projected") or {}).get("sources") or []):
                    key = "configMap" if kind == "ConfigMap" else "secret"
                    if (src.get(key) or {}).get("name") == old:
                        src[key]["name"] = new
            for c in _containers(ps):
                for ef in c.get("envFrom") or []:
                    key = "configMapRef" if kind == "ConfigMap" else "secretRef"
                    if (ef.get(key) or {}).get("name") == old:
                        ef[key]["name"] = new
                for e in c.get("env") or []:
                    key = "configMapKeyRef" if kind == "ConfigMap" else "secretKeyRef"
                    ref = (e.get("valueFrom") or {}).get(key)
                    if ref and ref.get("name") == old:
                        ref["name"] = new
            if kind == "ServiceAccount" and ps.get("serviceAccountName") == old:
                ps["serviceAccountName"] = new
        if kind == "ServiceAccount" and o.get("kind") in ("RoleBinding", "ClusterRoleBinding"):
            for s in o.get("subjects") or []:
                if s.get("kind") == "ServiceAccount" and s.get("name") == old:
                    s["name"] = new
        if kind in ("Role", "ClusterRole") and o.get("kind") in ("RoleBinding", "ClusterRoleBinding"):
            rr = o.get("roleRef") or {}
            if rr.get("kind") == kind and rr.get("name") == old:
                rr["name"] = new
        if kind == "Service" and o.get("kind") in ("MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"):
            for w in o.get("webhooks") or []:
                svc = (w.get("clientConfig") or {}).get("service")
                if svc and svc.get("name") == old:
                    svc["name"] = new


def _set_namespace(objs: list[dict], ns: str) -> None:
    for o in objs:
        if o.get("kind") in CLUSTER_SCOPED:
            if o.get("kind") in ("ClusterRoleBinding", "RoleBinding"):
                for s in o.get("subjects") or []:
                    if s.get("kind") == "ServiceAccount":
                        s["namespace"] = ns
            if o.get("kind") in ("MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"):
                for w in o.get("webhooks") or []:
                    svc = (w.get("clientConfig") or {}).get("service")
                    if svc is not None:
                        svc["namespace"] = ns
            continue
        o.setdefault("metadata", {})["namespace"] = ns
        if o.get("kind") == "RoleBinding":
            for s in o.get("subjects") or []:
                if s.get("kind") == "ServiceAccount":
                    s["namespace"] = ns


def _apply_images(objs: list[dict], images: list[dict]) -> None:
    def rewrite(img: str) -> str:
        name, tag, digest = img, None, None
        if "@" in name:
            name, digest = name.split("@", 1)
        elif ":" in name.rsplit("/", 1)[-1]:
            name, tag = name.rsplit(":", 1)
        for rule in images:
            if rule["name"] != name:
                continue
            name = rule.get("newName", name)
            if "digest" in rule:
                return f"{name}@{rule['digest']}"
            tag = rule.get("newTag", tag)
        if digest:
            return f"{name}@{digest}"
        return f"{name}:{tag}" if tag else name

    for o in objs:
        ps = _pod_spec(o)
        if ps is None:
            continue
        for c in _containers(ps):
            if "image" in c:
                c["image"] = rewrite(c["image"])


def _apply_labels(objs: list[dict], labels: dict) -> None:
    for o in objs:
        md = o.setdefault("metadata", {})
        md["labels"] = {**(md.get("labels") or {}), **labels}
        if o.get("kind") in ("Deployment", "StatefulSet", "DaemonSet", "ReplicaSet"):
            spec = o.setdefault("spec", {})
            sel = spec.setdefault("selector", {}).setdefault("matchLabels", {})
            sel.update(labels)
            tmd = spec.setdefault("template", {}).setdefault("metadata", {})
            tmd["labels"] = {**(tmd.get("labels") or {}), **labels}
        if o.get("kind") == "Service":
            spec = o.setdefault("spec", {})
            if spec.get("selector") is not None or spec.get("type") != "ExternalName":
                spec["selector"] = {**(spec.get("selector") or {}), **labels}


def _matches(o: dict, target: dict) -> bool:
    for key in ("kind", "name", "namespace"):
        if key in target:
            val = o.get("kind") if key == "kind" else o.get("metadata", {}).get(key)
            if val != target[key]:
                return False
    if "group" in target or "version" in target:
        g, _, v = o.get("apiVersion", "").rpartition("/")
        if target.get("group", g) != g or target.get("version", v) != v:
            return False
    return True


# ---- build ---------------------------------------------------------------------------------------
ORIG = "kfamd.io/generator-name"
PENDING_HASH = "kfamd.io/generated"


def build(path: str | os.PathLike) -> list[dict]:
    """Render a kustomization directory (or a plain YAML file)."""
    objs = _build(path, ())
    # content-hash suffixes last (after every overlay's data change), once per generated object
    for o in objs:
        ann = (o.get("metadata") or {}).get("annotations") or {}
        ann.pop(ORIG, None)
        if ann.pop(PENDING_HASH, None) == "true":
            old = o["metadata"]["name"]
            o["metadata"]["name"] = f"{old}-{_hash(o)}"
            _rename_refs(objs, o["kind"], old, o["metadata"]["name"])
        if not ann and "annotations" in (o.get("metadata") or {}):
            o["metadata"].pop("annotations")
    return objs


def _build(path: str | os.PathLike, _stack: tuple) -> list[dict]:
    d = Path(path).resolve()
    if d.is_file():
        return _load_docs(d)
    kf = _kustomization_file(d)
    if kf is None:
        raise KustomizeError(f"{d}: no kustomization.yaml")
    if d in _stack:
        raise KustomizeError(f"kustomization cycle through {d}")
    k = yaml.safe_load(kf.read_text()) or {}
    objs: list[dict] = []
    for r in (k.get("resources") or []) + (k.get("bases") or []) + (k.get("crds") or []):
        p = (d / r).resolve()
        if not p.exists():
            raise KustomizeError(f"{kf}: resource {r} not found")
        objs.extend(_build(p, _stack + (d,)) if p.is_dir() else _load_docs(p))

    gen_opts = k.get("generatorOptions") or {}
    renames: list[tuple[str, str, str]] = []
    for kind, key in (("ConfigMap", "configMapGenerator"), ("Secret", "secretGenerator")):
        for spec in k.get(key) or []:
            gen = _generate(spec, kind, d, gen_opts)
            behavior = spec.get("behavior", "create")
            existing = [o for o in objs if o.get("kind") == kind and
                        ((o["metadata"].get("annotations") or {}).get(ORIG) or o["metadata"].get("name")) == spec["name"]]
            if behavior in ("merge", "replace") and existing:
                tgt = existing[0]
                tgt["data"] = {**(tgt.get("data") or {}), **gen["data"]} if behavior == "merge" else gen["data"]
                gen = tgt
            elif behavior in ("merge", "replace"):
                raise KustomizeError(f"{kf}: {behavior} of missing {kind} {spec['name']}")
            else:
                objs.append(gen)
            no_hash = gen_opts.get("disableNameSuffixHash") or (spec.get("options") or {}).get("disableNameSuffixHash")
            ann = gen.setdefault("metadata", {}).setdefault("annotations", {})
            ann.setdefault(ORIG, spec["name"])
            if not no_hash and behavior == "create":
                ann[PENDING_HASH] = "true"
    # patches
    for pf in k.get("patchesStrategicMerge") or []:
        for patch in _load_docs(d / pf):
            hit = False
            for i, o in enumerate(objs):
                if o.get("kind") == patch.get("kind") and o["metadata"].get("name") == patch["metadata"].get("name"):
                    objs[i] = strategic_merge(o, patch)
                    hit = True
            if not hit:
                raise KustomizeError(f"{kf}: patch {pf} matches no resource")
    for p in k.get("patches") or []:
        body = yaml.safe_load((d / p["path"]).read_text()) if "path" in p else yaml.safe_load(p["patch"])
        target = p.get("target")
        for i, o in enumerate(objs):
            if isinstance(body, list):
                if target and _matches(o, target):
                    objs[i] = json_patch(o, body)
            elif (target and _matches(o, target)) or (not target and o.get("kind") == body.get("kind")
                                                    and o["metadata"].get("name") == body["metadata"].get("name")):
                objs[i] = strategic_merge(o, body)
    for rep in k.get("replicas") or []:
        for o in objs:
            if o["metadata"].get("name") == rep["name"] and o.get("kind") in ("Deployment", "StatefulSet", "ReplicaSet"):
                o.setdefault("spec", {})["replicas"] = rep["count"]

    # names, namespace, labels, images
    prefix, suffix = k.get("namePrefix", ""), k.get("nameSuffix", "")
    if prefix or suffix:
        for o in objs:
            if o.get("kind") in ("CustomResourceDefinition", "Namespace"):
                continue
            old = o["metadata"]["name"]
            new = f"{prefix}{old}{suffix}"
            o["metadata"]["name"] = new
            renames.append((o["kind"], old, new))
    if k.get("namespace"):
        _set_namespace(objs, k["namespace"])
    if k.get("commonLabels"):
        _apply_labels(objs, k["commonLabels"])
    if k.get("commonAnnotations"):
        for o in objs:
            md = o.setdefault("metadata", {})
            md["annotations"] = {**(md.get("annotations") or {}), **k["commonAnnotations"]}
    if k.get("images"):
        _apply_images(objs, k["images"])
    for kind, old, new in renames:
        _rename_refs(objs, kind, old, new)
    return objs


def dump(objs: list[dict]) -> str:
    return "---\n".join(yaml.safe_dump(o, sort_keys=False, default_flow_style=False) for o in objs)
