"""The writing half of kfctl's kubectl subset: create / patch / annotate / label / scale.

    kfctl create namespace|ns NAME
    kfctl create secret tls NAME --cert=FILE --key=FILE [-n NS]
    kfctl create secret generic NAME [--from-literal=K=V ...] [--from-file=[K=]PATH ...] [-n NS]
    kfctl create configmap|cm NAME [--from-literal=K=V ...] [--from-file=[K=]PATH ...] [-n NS]
    kfctl create serviceaccount|sa NAME [-n NS]
    kfctl create -f FILE|-                      (AlreadyExists is an error, unlike apply)
    kfctl patch TYPE NAME | TYPE/NAME -p PATCH [--type strategic|merge|json] [--subresource status] [-n NS]
    kfctl annotate TYPE NAME | TYPE/NAME KEY=VAL ... KEY- ... [--overwrite] [-n NS] [-l SEL | --all]
    kfctl label    (same form as annotate)
    kfctl scale TYPE NAME | TYPE/NAME --replicas=N [--current-replicas=M] [-n NS]

These are the verbs the reference's CI drives kubectl with: ``kubectl create ns``
(.github/workflows/notebook_controller_integration_test.yaml:86,
odh_notebook_controller_integration_test.yaml:132,168), ``kubectl create secret tls`` (:195,198),
``kubectl patch MutatingWebhookConfiguration/... --type=json -p=...`` (:212), and the annotation
protocol of SURVEY §2.9.3 (``kubeflow-resource-stopped`` stops a notebook,
``notebooks.opendatahub.io/notebook-restart`` restarts it). Output and conflict rules follow kubectl:
``<kind>[.<group>]/<name> created|patched|annotated|labeled|scaled`` (``(no change)`` when the
object did not change), and an existing annotation / label with a different value is an error
unless ``--overwrite``.
"""
from __future__ import annotations

import base64
import json
import os
import sys

from .client import ApiException, KubeClient
from .kubectl import KubectlError, Resource, _parse_target, load_docs, resolve


def _ref(res: Resource, name: str) -> str:
    return f"{res.kind.lower()}{'.' + res.group if res.group else ''}/{name}"


def _ns(res: Resource, a) -> str | None:
    return (a.namespace or "default") if res.namespaced else None


def _created(kind: str, group: str, name: str, out) -> None:
    out.write(f"{kind.lower()}{'.' + group if group else ''}/{name} created\n")


def _from_sources(a) -> dict[str, str]:
    data: dict[str, str] = {}
    for kv in a.from_literal or []:
        if "=" not in kv:
            raise KubectlError(f"error: invalid literal source {kv}, expected key=value")
        k, v = kv.split("=", 1)
        data[k] = v
    for spec in a.from_file or []:
        k, _, path = spec.partition("=") if "=" in spec else (os.path.basename(spec), "", spec)
        with open(path, "rb") as f:
            data[k] = f.read().decode("utf-8", "surrogateescape")
    return data


def cmd_create(client: KubeClient, a, out=sys.stdout) -> int:
    if a.filename:
        for o in load_docs(a.filename):
            ns = (o.get("metadata") or {}).get("namespace") or a.namespace
            res = resolve(client, f"{o['kind'].lower()}")
            made = client.create(o, namespace=ns if res.namespaced else None)
            out.write(_ref(res, made["metadata"]["name"]) + " created\n")
        return 0
    if not a.args:
        raise KubectlError("error: must specify one of -f and -k, or a resource type to create")
    what, rest = a.args[0].lower(), a.args[1:]
    ns = a.namespace or "default"
    if what in ("namespace", "ns"):
        if len(rest) != 1:
            raise KubectlError("error: exactly one NAME is required")
        client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": rest[0]}})
        _created("Namespace", "", rest[0], out)
        return 0
    if what in ("serviceaccount", "sa"):
        client.create({"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": rest[0], "namespace": ns}})
        _created("ServiceAccount", "", rest[0], out)
        return 0
    if what in ("configmap", "cm"):
        if len(rest) != 1:
            raise KubectlError("error: exactly one NAME is required")
        client.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": rest[0], "namespace": ns},
                       "data": _from_sources(a)})
        _created("ConfigMap", "", rest[0], out)
        return 0
    if what == "secret":
        if len(rest) != 2:
            raise KubectlError("error: usage: create secret tls|generic NAME")
        sub, name = rest
        if sub == "tls":
            if not a.cert or not a.key:
                raise KubectlError("error: --cert and --key are required for a tls secret")
            with open(a.cert, "rb") as f:
                crt = f.read()
            with open(a.key, "rb") as f:
                key = f.read()
            if b"-----BEGIN" not in crt or b"-----BEGIN" not in key:
                raise KubectlError("error: failed to load key pair: the --cert / --key files are not PEM")
            data = {"tls.crt": base64.b64encode(crt).decode(), "tls.key": base64.b64encode(key).decode()}
            typ = "kubernetes.io/tls"
        elif sub == "generic":
            data = {k: base64.b64encode(v.encode("utf-8", "surrogateescape")).decode() for k, v in _from_sources(a).items()}
            typ = a.type or "Opaque"
        else:
            raise KubectlError(f"error: unknown secret type {sub} (tls, generic)")
        client.create({"apiVersion": "v1", "kind": "Secret", "metadata": {"name": name, "namespace": ns},
                       "type": typ, "data": data})
        _created("Secret", "", name, out)
        return 0
    raise KubectlError(f'error: unknown resource type "{what}" for create '
                       "(namespace, secret tls|generic, configmap, serviceaccount, or -f FILE)")


def cmd_patch(client: KubeClient, a, out=sys.stdout) -> int:
    res, names = _parse_target(client, a.target)
    if len(names) != 1:
        raise KubectlError("error: patch takes exactly one resource NAME")
    if a.patch is None:
        raise KubectlError("error: must specify -p to patch")
    try:
        body = json.loads(a.patch)
    except ValueError:
        import yaml
        body = yaml.safe_load(a.patch)
    ptype = a.type or "strategic"
    if ptype not in ("strategic", "merge", "json"):
        raise KubectlError(f'error: --type must be one of [json merge strategic], not "{ptype}"')
    ns = _ns(res, a)
    before = client.get(res.api_version, res.kind, names[0], ns)
    after = client.patch(res.api_version, res.kind, names[0], body, ns, ptype, subresource=a.subresource)
    same = (after.get("metadata") or {}).get("resourceVersion") == before["metadata"].get("resourceVersion")
    out.write(_ref(res, names[0]) + (" patched (no change)\n" if same else " patched\n"))
    return 0


def _kv_args(items: list[str]) -> tuple[dict[str, str], list[str]]:
    sets, removes = {}, []
    for it in items:
        if it.endswith("-") and "=" not in it:
            removes.append(it[:-1])
        elif "=" in it:
            k, v = it.split("=", 1)
            if not k:
                raise KubectlError(f"error: invalid {it!r}: the key is empty")
            sets[k] = v
        else:
            raise KubectlError(f"error: invalid {it!r}: expected KEY=VALUE or KEY-")
    return sets, removes


def _meta_verb(field: str, done: str, client: KubeClient, a, out) -> int:
    """annotate / label: merge-patch metadata.<field>, kubectl's --overwrite rule."""
    # kubectl form: TYPE NAME... KEY=VAL ... KEY-  or  TYPE/NAME ... KEY=VAL ...
    targets = [x for x in a.items if "=" not in x and not x.endswith("-")]
    kvs = [x for x in a.items if x not in targets]
    sets, removes = _kv_args(kvs)
    if not sets and not removes:
        raise KubectlError(f"error: at least one {field[:-1]} update is required")
    res, names = _parse_target(client, targets)
    ns = _ns(res, a)
    if not names:
        if not (a.all or a.selector):
            raise KubectlError("error: one or more resources must be specified as <resource> <name> or <resource>/<name>")
        names = [o["metadata"]["name"] for o in client.list(res.api_version, res.kind, ns, label_selector=a.selector or "")
                 .get("items", [])]
    for name in names:
        cur = client.get(res.api_version, res.kind, name, ns)
        have = (cur.get("metadata") or {}).get(field) or {}
        if not a.overwrite:
            clash = [k for k, v in sets.items() if k in have and have[k] != v]
            if clash:
                raise KubectlError(f"error: --overwrite is false but found the following declared {field[:-1]}(s): " +
                                   ", ".join(f"'{k}' already has a value ({have[k]})" for k in clash))
        patch = {k: v for k, v in sets.items() if have.get(k) != v}
        patch.update({k: None for k in removes if k in have})
        if not patch:
            out.write(_ref(res, name) + (" not labeled\n" if field == "labels" else " annotated\n"))
            continue
        client.patch(res.api_version, res.kind, name, {"metadata": {field: patch}}, ns, "merge")
        out.write(_ref(res, name) + f" {done}\n")
    return 0


def cmd_annotate(client: KubeClient, a, out=sys.stdout) -> int:
    return _meta_verb("annotations", "annotated", client, a, out)


def cmd_label(client: KubeClient, a, out=sys.stdout) -> int:
    return _meta_verb("labels", "labeled", client, a, out)


def cmd_scale(client: KubeClient, a, out=sys.stdout) -> int:
    if a.replicas is None or a.replicas < 0:
        raise KubectlError("error: The --replicas=COUNT flag is required, and COUNT must be greater than or equal to 0")
    res, names = _parse_target(client, a.target)
    if not names:
        raise KubectlError("error: resource(s) were provided, but no name was specified")
    ns = _ns(res, a)
    for name in names:
        path = client.path(res.api_version, res.kind, ns, name, "scale")
        try:
            sc = client._req("GET", path)
        except ApiException as e:
            if e.status == 404 and "scale" not in str(e.body or ""):
                raise
            raise KubectlError(f"error: no scale subresource for {_ref(res, name)}: {e.message}")
        if a.current_replicas is not None and (sc.get("spec") or {}).get("replicas") != a.current_replicas:
            raise KubectlError(f"error: Expected replicas to be {a.current_replicas}, was {(sc.get('spec') or {}).get('replicas')}")
        sc.setdefault("spec", {})["replicas"] = a.replicas
        client._req("PUT", path, sc)
        out.write(_ref(res, name) + " scaled\n")
    return 0


def add_parsers(sub, common) -> None:
    c = sub.add_parser("create", help="create a namespace / secret / configmap / serviceaccount, or -f FILE")
    c.add_argument("args", nargs="*")
    c.add_argument("-f", "--filename", default=None)
    c.add_argument("--cert", default=None)
    c.add_argument("--key", default=None)
    c.add_argument("--type", default=None, help="secret generic: the Secret type (default Opaque)")
    c.add_argument("--from-literal", action="append", default=None)
    c.add_argument("--from-file", action="append", default=None)
    common(c, selector=False)
    p = sub.add_parser("patch", help="patch a resource (strategic / merge / json)")
    p.add_argument("target", nargs="+")
    p.add_argument("-p", "--patch", default=None)
    p.add_argument("--type", default=None)
    p.add_argument("--subresource", default=None)
    common(p, selector=False)
    for name in ("annotate", "label"):
        m = sub.add_parser(name, help=f"update the {name}s on resources (KEY=VAL, KEY- removes)")
        m.add_argument("items", nargs="+")
        m.add_argument("--overwrite", action="store_true")
        m.add_argument("--all", action="store_true")
        common(m)
    s = sub.add_parser("scale", help="set the replicas of a StatefulSet / Deployment / ReplicaSet")
    s.add_argument("target", nargs="+")
    s.add_argument("--replicas", type=int, default=None)
    s.add_argument("--current-replicas", type=int, default=None)
    common(s, selector=False)


VERBS = {"create": cmd_create, "patch": cmd_patch, "annotate": cmd_annotate, "label": cmd_label, "scale": cmd_scale}
