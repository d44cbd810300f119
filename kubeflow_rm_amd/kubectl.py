"""kubectl-subset verbs of ``kfctl`` against the kube-lite API server (or any Kubernetes API).

    kfctl get <resource> [name ...] [-n NS | -A] [-l SELECTOR] [-o wide|yaml|json|name|jsonpath=EXPR]
    kfctl describe <resource> [name ...] [-n NS | -A] [-l SELECTOR]
    kfctl wait <resource>[/name] [name ...] --for=condition=C[=V] | --for=jsonpath='{.path}'=V | --for=delete
               [--timeout=100s] [-n NS] [-l SELECTOR | --all]
    kfctl rollout status [--watch] statefulset|deployment <name> [--timeout=300s] [-n NS]
    kfctl logs <pod> [-c CONTAINER] [-n NS] [--tail N] [-f]
    kfctl apply -f FILE|-     kfctl delete -f FILE|- | <resource> <name>
    kfctl create / patch / annotate / label / scale          (kubectl_mutate.py)

What the reference's own acceptance flow runs (``.github/workflows/odh_notebook_controller_integration_test.yaml:275-289``,
``notebook_controller_integration_test.yaml:106``) and what its load test drives
(``components/notebook-controller/loadtest/start_notebooks.py:50-96``). Resources resolve the way
kubectl resolves them, from API discovery: plural, singular, kind, short names (``po``, ``sts``,
``nb`` ...) and ``plural.group`` (``notebooks.kubeflow.org``). Exit codes follow kubectl: 0 on
success, 1 on an error or a wait that timed out.
"""
from __future__ import annotations

import argparse
import datetime as _dt
import json
import re
import sys
import time
from typing import Any, Callable

from .client import ApiException, KubeClient, print_warning

# short names kubectl knows for kinds whose discovery here carries none
_EXTRA_SHORT = {"statefulsets": ["sts"], "deployments": ["deploy"], "replicasets": ["rs"], "daemonsets": ["ds"],
                "notebooks": ["nb"], "services": ["svc"], "serviceaccounts": ["sa"], "pods": ["po"],
                "persistentvolumeclaims": ["pvc"], "customresourcedefinitions": ["crd", "crds"],
                "virtualservices": ["vs"], "poddefaults": ["pd"], "resourcequotas": ["quota"],
                "networkpolicies": ["netpol"], "horizontalpodautoscalers": ["hpa"]}


class KubectlError(RuntimeError):
    pass


class Resource:
    def __init__(self, api_version: str, kind: str, plural: str, singular: str, namespaced: bool, short: list[str]):
        self.api_version, self.kind, self.plural = api_version, kind, plural
        self.singular, self.namespaced, self.short = singular, namespaced, short
        self.group = api_version.split("/")[0] if "/" in api_version else ""

    def names(self) -> set[str]:
        n = {self.plural, self.singular, self.kind.lower(), *self.short}
        if self.group:
            n |= {f"{self.plural}.{self.group}", f"{self.singular}.{self.group}", f"{self.kind.lower()}.{self.group}"}
        return {x for x in n if x}


def discover(client: KubeClient) -> list[Resource]:
    """Every served resource at its group's preferred version (kubectl's discovery walk)."""
    out = []
    versions = ["v1"] + [g["preferredVersion"]["groupVersion"] for g in client._req("GET", "/apis").get("groups", [])]
    for gv in versions:
        disc = client._req("GET", f"/api/{gv}" if gv == "v1" else f"/apis/{gv}")
        for r in disc.get("resources", []):
            if "/" in r["name"]:
                continue
            short = list(r.get("shortNames") or []) + _EXTRA_SHORT.get(r["name"], [])
            out.append(Resource(gv, r["kind"], r["name"], r.get("singularName") or r["kind"].lower(),
                                r.get("namespaced", True), short))
    return out


def resolve(client: KubeClient, name: str, _cache: dict = {}) -> Resource:  # noqa: B006 - per-client cache
    key = id(client)
    if key not in _cache:
        _cache[key] = discover(client)
    want = name.lower()
    hits = [r for r in _cache[key] if want in r.names()]
    if not hits:
        raise KubectlError(f'error: the server doesn\'t have a resource type "{name}"')
    # core / apps before extension groups for an ambiguous short name, as kubectl's priority does
    hits.sort(key=lambda r: (r.group not in ("", "apps"), r.group))
    return hits[0]


# ---- JSONPath (the kubectl subset: {.a.b}, [n], [*], multiple {} in one template) ------------------
def _jsonpath_eval(obj: Any, path: str) -> list[Any]:
    toks = re.findall(r"\.([A-Za-z0-9_\-]+|\*)|\[(\*|-?\d+|'[^']*'|\"[^\"]*\")\]", path)
    cur = [obj]
    for name, idx in toks:
        nxt = []
        for c in cur:
            if name:
                if name == "*":
                    nxt += list(c.values()) if isinstance(c, dict) else list(c) if isinstance(c, list) else []
                elif isinstance(c, dict) and name in c:
                    nxt.append(c[name])
            elif idx == "*":
                nxt += list(c.values()) if isinstance(c, dict) else list(c) if isinstance(c, list) else []
            elif idx[0] in "'\"":
                if isinstance(c, dict) and idx[1:-1] in c:
                    nxt.append(c[idx[1:-1]])
            elif isinstance(c, list):
                i = int(idx)
                if -len(c) <= i < len(c):
                    nxt.append(c[i])
        cur = nxt
    return cur


def _fmt_scalar(v: Any) -> str:
    if isinstance(v, (dict, list)):
        return json.dumps(v)
    if isinstance(v, bool):
        return "true" if v else "false"
    return "" if v is None else str(v)


def jsonpath(obj: Any, template: str) -> str:
    """Render a kubectl -o jsonpath template ('{.metadata.name}', 'x={.a[0].b} {.c}')."""
    out, pos = [], 0
    for m in re.finditer(r"\{([^}]*)\}", template):
        out.append(template[pos:m.start()])
        expr = m.group(1).strip()
        if expr.startswith("."):
            out.append(" ".join(_fmt_scalar(v) for v in _jsonpath_eval(obj, expr)))
        pos = m.end()
    out.append(template[pos:])
    return "".join(out)


# ---- table printing ----------------------------------------------------------------------------------
def _age(ts: str | None) -> str:
    if not ts:
        return "<unknown>"
    try:
        t = _dt.datetime.strptime(ts.split(".")[0].rstrip("Z"), "%Y-%m-%dT%H:%M:%S").replace(tzinfo=_dt.timezone.utc)
    except ValueError:
        return "<unknown>"
    s = max(0, int((_dt.datetime.now(_dt.timezone.utc) - t).total_seconds()))
    if s < 120:
        return f"{s}s"
    if s < 7200:
        return f"{s // 60}m"
    if s < 172800:
        return f"{s // 3600}h"
    return f"{s // 86400}d"


def _pod_status(p: dict) -> tuple[str, str, int]:
    st = p.get("status") or {}
    cs = st.get("containerStatuses") or []
    ready = sum(1 for c in cs if c.get("ready"))
    total = len((p.get("spec") or {}).get("containers") or []) or len(cs)
    restarts = sum(int(c.get("restartCount") or 0) for c in cs)
    reason = st.get("reason") or st.get("phase") or "Pending"
    for c in (st.get("initContainerStatuses") or []):
        w = (c.get("state") or {}).get("waiting") or {}
        t = (c.get("state") or {}).get("terminated") or {}
        if w.get("reason") and w["reason"] != "PodInitializing":
            reason = f"Init:{w['reason']}"
        elif t and t.get("exitCode", 0) != 0:
            reason = f"Init:Error"
    for c in cs:
        w = (c.get("state") or {}).get("waiting") or {}
        t = (c.get("state") or {}).get("terminated") or {}
        if w.get("reason"):
            reason = w["reason"]
        elif t.get("reason") and reason == "Running":
            reason = t["reason"]
    if (p.get("metadata") or {}).get("deletionTimestamp"):
        reason = "Terminating"
    return f"{ready}/{total}", reason, restarts


def _columns(kind: str, wide: bool) -> list[tuple[str, Callable[[dict], str]]]:
    md = lambda o: o.get("metadata") or {}  # noqa: E731
    st = lambda o: o.get("status") or {}  # noqa: E731
    sp = lambda o: o.get("spec") or {}  # noqa: E731
    age = ("AGE", lambda o: _age(md(o).get("creationTimestamp")))
    if kind == "Pod":
        cols = [("READY", lambda o: _pod_status(o)[0]), ("STATUS", lambda o: _pod_status(o)[1]),
                ("RESTARTS", lambda o: str(_pod_status(o)[2])), age]
        if wide:
            cols += [("IP", lambda o: st(o).get("podIP") or "<none>"), ("NODE", lambda o: sp(o).get("nodeName") or "<none>"),
                     ("GPUS", lambda o: (md(o).get("annotations") or {}).get("amd.com/gpu-ids") or "<none>")]
        return cols
    if kind == "StatefulSet":
        return [("READY", lambda o: f"{st(o).get('readyReplicas') or 0}/{sp(o).get('replicas', 1)}"), age]
    if kind == "Deployment":
        return [("READY", lambda o: f"{st(o).get('readyReplicas') or 0}/{sp(o).get('replicas', 1)}"),
                ("UP-TO-DATE", lambda o: str(st(o).get("updatedReplicas") or 0)),
                ("AVAILABLE", lambda o: str(st(o).get("availableReplicas") or 0)), age]
    if kind == "Service":
        return [("TYPE", lambda o: sp(o).get("type") or "ClusterIP"), ("CLUSTER-IP", lambda o: sp(o).get("clusterIP") or "<none>"),
                ("PORT(S)", lambda o: ",".join(f"{p.get('port')}/{p.get('protocol', 'TCP')}" for p in sp(o).get("ports") or []) or "<none>"),
                age]
    if kind == "Notebook":
        def nb_status(o):
            s = st(o)
            if s.get("readyReplicas") == 1:
                return "Ready"
            state = s.get("containerState") or {}
            if "waiting" in state:
                return (state["waiting"] or {}).get("reason") or "Waiting"
            return "Stopped" if "kubeflow-resource-stopped" in (md(o).get("annotations") or {}) else "Pending"
        cols = [("READY", lambda o: str(st(o).get("readyReplicas") or 0)), ("STATUS", nb_status), age]
        if wide:
            cols += [("GPUS", lambda o: st(o).get("gpus") or "<none>"),
                     ("IMAGE", lambda o: ((sp(o).get("template") or {}).get("spec", {}).get("containers") or [{}])[0].get("image", ""))]
        return cols
    if kind == "Namespace":
        return [("STATUS", lambda o: st(o).get("phase") or "Active"), age]
    if kind == "Event":
        return [("LAST SEEN", lambda o: _age(o.get("lastTimestamp") or o.get("eventTime") or md(o).get("creationTimestamp"))),
                ("TYPE", lambda o: o.get("type") or ""), ("REASON", lambda o: o.get("reason") or ""),
                ("OBJECT", lambda o: f"{(o.get('involvedObject') or {}).get('kind', '').lower()}/{(o.get('involvedObject') or {}).get('name', '')}"),
                ("MESSAGE", lambda o: o.get("message") or "")]
    if kind == "PersistentVolumeClaim":
        return [("STATUS", lambda o: st(o).get("phase") or "Pending"),
                ("CAPACITY", lambda o: ((st(o).get("capacity") or {}).get("storage")) or ""),
                ("ACCESS MODES", lambda o: ",".join({"ReadWriteOnce": "RWO", "ReadWriteMany": "RWX", "ReadOnlyMany": "ROX"}.get(m, m)
                                                     for m in sp(o).get("accessModes") or [])), age]
    if kind in ("Tensorboard", "PVCViewer"):
        return [("READY", lambda o: str(st(o).get("readyReplicas") if "readyReplicas" in st(o) else st(o).get("ready", ""))), age]
    return [age]


def render_table(items: list[dict], kind: str, wide: bool = False, all_ns: bool = False, headers: bool = True) -> str:
    cols = [("NAME", lambda o: (o.get("metadata") or {}).get("name", ""))] + _columns(kind, wide)
    if all_ns:
        cols = [("NAMESPACE", lambda o: (o.get("metadata") or {}).get("namespace", ""))] + cols
    rows = [[h for h, _ in cols]] if headers else []
    rows += [[f(o) for _, f in cols] for o in items]
    if not rows:
        return ""
    width = [max(len(r[i]) for r in rows) for i in range(len(cols))]
    return "\n".join("   ".join(c.ljust(width[i]) for i, c in enumerate(r)).rstrip() for r in rows) + "\n"


def _dump(obj: Any, fmt: str) -> str:
    if fmt == "json":
        return json.dumps(obj, indent=4) + "\n"
    import yaml
    return yaml.safe_dump(obj, sort_keys=False, default_flow_style=False)


# ---- verbs -------------------------------------------------------------------------------------------
def _parse_target(client: KubeClient, args: list[str]) -> tuple[Resource, list[str]]:
    """'pods x y' | 'pod/x' | 'pods/x pods/y' -> (resource, names)."""
    if not args:
        raise KubectlError("error: you must specify the type of resource to get")
    if "/" in args[0]:
        res = None
        names = []
        for a in args:
            t, n = a.split("/", 1)
            r = resolve(client, t)
            if res is not None and r.kind != res.kind:
                raise KubectlError("error: mixed resource types are not supported")
            res = r
            names.append(n)
        return res, names
    return resolve(client, args[0]), args[1:]


def _list(client: KubeClient, res: Resource, names: list[str], ns: str | None, all_ns: bool, selector: str) -> list[dict]:
    if names:
        out = []
        for n in names:
            try:
                out.append(client.get(res.api_version, res.kind, n, ns if res.namespaced else None))
            except ApiException as e:
                if e.status == 404:
                    raise KubectlError(f'Error from server (NotFound): {res.plural}{"." + res.group if res.group else ""} "{n}" not found')
                raise
        return out
    return client.list(res.api_version, res.kind, None if all_ns or not res.namespaced else ns,
                       label_selector=selector).get("items", [])


def cmd_get(client: KubeClient, a, out=sys.stdout) -> int:
    if "," in a.target[0] and "/" not in a.target[0]:  # get pods,svc: one table per type
        rc = 0
        for i, t in enumerate(x for x in a.target[0].split(",") if x):
            sub = type(a)(**{**vars(a), "target": [t, *a.target[1:]]})
            if i and not (a.output or "").startswith(("json", "yaml")):
                out.write("\n")
            rc |= cmd_get(client, sub, out)
        return rc
    res, names = _parse_target(client, a.target)
    items = _list(client, res, names, a.namespace, a.all_namespaces, a.selector or "")
    fmt = a.output or ""
    if fmt in ("yaml", "json"):
        if len(items) == 1 and names:
            out.write(_dump(items[0], fmt))
        else:
            out.write(_dump({"apiVersion": "v1", "kind": "List", "items": items, "metadata": {"resourceVersion": ""}}, fmt))
    elif fmt == "name":
        for o in items:
            out.write(f"{res.kind.lower()}{'.' + res.group if res.group else ''}/{o['metadata']['name']}\n")
    elif fmt.startswith("jsonpath="):
        tmpl = fmt[len("jsonpath="):].strip("'\"")
        obj = items[0] if len(items) == 1 and names else {"items": items}
        out.write(jsonpath(obj, tmpl))
    else:
        if not items:
            where = "" if a.all_namespaces or not res.namespaced else f" in {a.namespace or 'default'} namespace"
            sys.stderr.write(f"No resources found{where}.\n")
            return 0
        out.write(render_table(items, res.kind, wide=fmt == "wide", all_ns=a.all_namespaces and res.namespaced))
    return 0


def _describe_map(title: str, m: dict | None, indent: int = 14) -> str:
    if not m:
        return f"{title:<{indent}}<none>\n"
    lines = [f"{k}={v}" if title == "Labels:" else f"{k}: {v}" for k, v in sorted(m.items())]
    return f"{title:<{indent}}" + ("\n" + " " * indent).join(lines) + "\n"


def _yaml_block(obj: Any, indent: int) -> str:
    import yaml
    text = yaml.safe_dump(obj, sort_keys=False, default_flow_style=False).rstrip("\n")
    return "\n".join(" " * indent + ln for ln in text.splitlines()) + "\n"


def describe_one(client: KubeClient, res: Resource, o: dict) -> str:
    md = o.get("metadata") or {}
    s = f"{'Name:':<14}{md.get('name', '')}\n"
    if res.namespaced:
        s += f"{'Namespace:':<14}{md.get('namespace', '')}\n"
    s += _describe_map("Labels:", md.get("labels"))
    s += _describe_map("Annotations:", md.get("annotations"))
    s += f"{'API Version:':<14}{o.get('apiVersion', res.api_version)}\n{'Kind:':<14}{o.get('kind', res.kind)}\n"
    if md.get("creationTimestamp"):
        s += f"{'Created:':<14}{md['creationTimestamp']}\n"
    owners = md.get("ownerReferences") or []
    if owners:
        s += f"Controlled By:  {owners[0].get('kind')}/{owners[0].get('name')}\n"
    if res.kind == "Pod":
        ready, status, restarts = _pod_status(o)
        st = o.get("status") or {}
        s += f"{'Status:':<14}{status}\n{'IP:':<14}{st.get('podIP', '')}\n{'Node:':<14}{(o.get('spec') or {}).get('nodeName', '')}\n"
        ann = (o.get("metadata") or {}).get("annotations") or {}
        if ann.get("amd.com/gpu-ids"):  # the device plugin's allocation (kubelet annotations)
            s += f"{'GPUs:':<14}{ann['amd.com/gpu-ids']}"
            if ann.get("amd.com/xgmi-ring"):
                s += f"  (xGMI ring {ann['amd.com/xgmi-ring']})"
            if ann.get("amd.com/gpu-placement"):
                s += f"\n{'Placement:':<14}{ann['amd.com/gpu-placement']}"
            s += "\n"
        if ann.get("notebooks.kubeflow.org/gpu-readiness"):
            try:
                rep = json.loads(ann["notebooks.kubeflow.org/gpu-readiness"])
                verdict = "ok" if rep.get("ok") else f"FAILED ({rep.get('error') or rep.get('stage') or '?'})"
                s += f"{'GPU Check:':<14}{verdict}, {rep.get('total_ms', '?')} ms\n"
            except (ValueError, AttributeError):
                pass
        for title, key in (("Init Containers:", "initContainerStatuses"), ("Containers:", "containerStatuses")):
            cs = st.get(key) or []
            if cs:
                s += f"{title}\n"
                for c in cs:
                    state = c.get("state") or {}
                    sname = next(iter(state), "unknown")
                    detail = state.get(sname) or {}
                    s += f"  {c.get('name')}:\n    State:          {sname.capitalize()}"
                    if detail.get("reason"):
                        s += f"\n      Reason:       {detail['reason']}"
                    if sname == "terminated":
                        s += f"\n      Exit Code:    {detail.get('exitCode')}"
                    if detail.get("message"):
                        s += f"\n      Message:      {str(detail['message'])[:300]}"
                    s += f"\n    Ready:          {c.get('ready')}\n    Restart Count:  {c.get('restartCount', 0)}\n"
    else:
        if "spec" in o:
            s += "Spec:\n" + _yaml_block(o["spec"], 2)
    conds = (o.get("status") or {}).get("conditions") or []
    if res.kind != "Pod" and o.get("status"):
        rest = {k: v for k, v in o["status"].items() if k != "conditions"}
        if rest:
            s += "Status:\n" + _yaml_block(rest, 2)
    if conds:
        s += "Conditions:\n  Type" + " " * 18 + "Status  Reason\n  ----" + " " * 18 + "------  ------\n"
        for c in conds:
            s += f"  {c.get('type', ''):<22}{c.get('status', ''):<8}{c.get('reason', '')}\n"
    # events of this object (kubectl describe's field selector on involvedObject)
    sel = f"involvedObject.kind={res.kind},involvedObject.name={md.get('name', '')}"
    try:
        evs = client.list("v1", "Event", md.get("namespace") or None, field_selector=sel).get("items", [])
    except (ApiException, TypeError):
        evs = []
    evs = [e for e in evs if (e.get("involvedObject") or {}).get("name") == md.get("name")
           and (e.get("involvedObject") or {}).get("kind") == res.kind]
    if evs:
        s += "Events:\n  Type    Reason            Age    From                 Message\n  ----    ------            ----   ----                 -------\n"
        evs.sort(key=lambda e: e.get("lastTimestamp") or e.get("eventTime") or "")
        for e in evs:
            src = (e.get("source") or {}).get("component") or e.get("reportingComponent") or ""
            s += (f"  {e.get('type', ''):<8}{e.get('reason', ''):<18}{_age(e.get('lastTimestamp') or e.get('eventTime')):<7}"
                  f"{src:<21}{e.get('message', '')}\n")
    else:
        s += "Events:       <none>\n"
    return s


def cmd_describe(client: KubeClient, a, out=sys.stdout) -> int:
    res, names = _parse_target(client, a.target)
    items = _list(client, res, names, a.namespace, a.all_namespaces, a.selector or "")
    if not items:
        sys.stderr.write("No resources found.\n")
        return 0
    out.write("\n\n".join(describe_one(client, res, o) for o in items))
    return 0


def parse_duration(s: str) -> float:
    m = re.fullmatch(r"(\d+(?:\.\d+)?)(ms|s|m|h)?", s.strip())
    if not m:
        raise KubectlError(f"error: invalid duration {s!r}")
    return float(m.group(1)) * {"ms": 1e-3, "s": 1, "m": 60, "h": 3600, None: 1}[m.group(2)]


def _condition_checker(spec: str) -> Callable[[dict], bool]:
    if spec == "delete":
        raise AssertionError("handled by the caller")
    if spec.startswith("condition="):
        cond = spec[len("condition="):]
        want = "True"
        if "=" in cond:
            cond, want = cond.split("=", 1)
        cond_l = cond.lower()

        def check(o):
            for c in (o.get("status") or {}).get("conditions") or []:
                if str(c.get("type", "")).lower() == cond_l:
                    return str(c.get("status", "")).lower() == want.lower()
            return False
        return check
    if spec.startswith("jsonpath="):
        expr = spec[len("jsonpath="):]
        m = re.fullmatch(r"'?(\{[^}]*\})'?(?:=(.*))?", expr)
        if not m:
            raise KubectlError(f"error: unrecognized jsonpath condition {expr!r}")
        path, want = m.group(1)[1:-1].strip(), m.group(2)
        want = want.strip("'\"") if want is not None else None

        def check(o):
            vals = _jsonpath_eval(o, path)
            if not vals:
                return False
            return want is None or _fmt_scalar(vals[0]) == want
        return check
    raise KubectlError(f"error: unrecognized condition: {spec!r}")


def cmd_wait(client: KubeClient, a, out=sys.stdout) -> int:
    res, names = _parse_target(client, a.target)
    deadline = time.time() + parse_duration(a.timeout)
    ns = a.namespace if res.namespaced else None
    spec = a.for_
    if spec is None:
        raise KubectlError("error: --for must be specified")
    gone = spec == "delete"
    check = None if gone else _condition_checker(spec)
    label = f"{res.kind.lower()}{'.' + res.group if res.group else ''}"
    pending: list[str] = list(names)
    if not names:
        # -l / --all: the objects that exist now (kubectl waits for at least one to appear)
        while True:
            items = client.list(res.api_version, res.kind, ns, label_selector=a.selector or "").get("items", [])
            if items:
                pending = [o["metadata"]["name"] for o in items]
                break
            if time.time() > deadline:
                sys.stderr.write("error: no matching resources found\n")
                return 1
            time.sleep(0.2)
    for n in pending:
        while True:
            try:
                o = client.get(res.api_version, res.kind, n, ns)
                if not gone and check(o):
                    out.write(f"{label}/{n} condition met\n")
                    break
            except ApiException as e:
                if e.status != 404:
                    raise
                if gone:
                    out.write(f"{label}/{n} condition met\n")
                    break
            if time.time() > deadline:
                sys.stderr.write(f"error: timed out waiting for the condition on {res.plural}/{n}\n")
                return 1
            time.sleep(0.05)
    return 0


def _rollout_done(o: dict) -> tuple[bool, str]:
    sp, st = o.get("spec") or {}, o.get("status") or {}
    want = sp.get("replicas", 1)
    ready = st.get("readyReplicas") or 0
    updated = st.get("updatedReplicas", ready)
    gen_ok = (st.get("observedGeneration") or 0) >= ((o.get("metadata") or {}).get("generation") or 0)
    if not gen_ok:
        return False, "Waiting for rollout to finish: observed generation lags"
    if updated < want:
        return False, f"Waiting for {want - updated} pods to be updated..."
    if ready < want:
        return False, f"Waiting for {want - ready} pods to be ready..."
    return True, ""


def cmd_rollout(client: KubeClient, a, out=sys.stdout) -> int:
    if a.action != "status":
        raise KubectlError(f"error: rollout {a.action} is not supported (status only)")
    res, names = _parse_target(client, a.target)
    if res.kind not in ("StatefulSet", "Deployment", "DaemonSet") or len(names) != 1:
        raise KubectlError("error: rollout status needs one statefulset/deployment/daemonset")
    deadline = time.time() + (parse_duration(a.timeout) if a.timeout else 1e12)
    last = ""
    while True:
        o = client.get(res.api_version, res.kind, names[0], a.namespace)
        done, msg = _rollout_done(o)
        if done:
            want = (o.get("spec") or {}).get("replicas", 1)
            if res.kind == "StatefulSet":
                out.write(f"partitioned roll out complete: {want} new pods have been updated...\n")
            else:
                out.write(f'{res.kind.lower()} "{names[0]}" successfully rolled out\n')
            return 0
        if msg != last:
            out.write(msg + "\n")
            last = msg
        if not a.watch:
            return 0
        if time.time() > deadline:
            sys.stderr.write("error: timed out waiting for the condition\n")
            return 1
        time.sleep(0.1)


def cmd_logs(client: KubeClient, a, out=sys.stdout) -> int:
    name = a.pod.split("/", 1)[1] if a.pod.startswith(("pod/", "pods/")) else a.pod
    ns = a.namespace or "default"
    try:
        text = client.pod_logs(name, ns, container=a.container, tail_lines=a.tail if a.tail is not None and a.tail >= 0 else None)
    except ApiException as e:
        raise KubectlError(f"Error from server ({e.reason or e.status}): {e.message}")
    out.write(text)
    out.flush()
    if not a.follow:
        return 0
    # follow: poll the log endpoint and print what was appended (the API streams no chunked logs here)
    seen = len(text)
    while True:
        time.sleep(0.5)
        try:
            text = client.pod_logs(name, ns, container=a.container)
        except ApiException as e:
            if e.status == 404:
                return 0
            raise
        if len(text) > seen:
            out.write(text[seen:])
            out.flush()
            seen = len(text)


def cmd_exec(client: KubeClient, a, out=sys.stdout) -> int:
    """kubectl exec POD [-c C] -- CMD...: runs in the container's env / working directory / CPU mask
    (no TTY, no stdin); prints the combined output and exits with the command's status."""
    cmd = list(a.command)
    if not cmd:
        raise KubectlError("error: you must specify at least one command for the container")
    name = a.pod.split("/", 1)[1] if a.pod.startswith(("pod/", "pods/")) else a.pod
    try:
        r = client.pod_exec(name, a.namespace or "default", cmd, container=a.container,
                            timeout=parse_duration(a.timeout))
    except ApiException as e:
        raise KubectlError(f"Error from server ({e.reason or e.status}): {e.message}")
    out.write(r.get("output", ""))
    out.flush()
    code = int(r.get("exitCode", 1))
    if code:
        sys.stderr.write(f"command terminated with exit code {code}\n")
    return code


_SAMPLE_RE = None


def parse_samples(text: str) -> list[tuple[str, dict, float]]:
    """Prometheus text exposition -> [(metric, {label: value}, sample value)] (no histograms needed)."""
    import re
    global _SAMPLE_RE
    if _SAMPLE_RE is None:
        _SAMPLE_RE = (re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(?:\{(.*)\})?\s+(\S+)'), re.compile(r'(\w+)="((?:[^"\\]|\\.)*)"'))
    line_re, label_re = _SAMPLE_RE
    out = []
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        m = line_re.match(line)
        if not m:
            continue
        try:
            v = float(m.group(3))
        except ValueError:
            continue
        out.append((m.group(1), dict(label_re.findall(m.group(2) or "")), v))
    return out


def _gib(b: float | None) -> str:
    return "-" if b is None else f"{b / (1 << 30):.1f}Gi"


def gpu_table(samples: list[tuple[str, dict, float]]) -> dict[str, dict]:
    """Per-GPU view of the kubelet's device-plugin and AMD SMI series (node-level ``kfctl top``)."""
    gpus: dict[str, dict] = {}
    for name, lab, v in samples:
        if not name.startswith("kfamd_gpu_") or "gpu" not in lab:
            continue
        g = gpus.setdefault(lab["gpu"], {"gpu": lab["gpu"]})
        key = name[len("kfamd_gpu_"):]
        if key == "allocated" and v >= 1:
            g["pod"] = f"{lab.get('namespace', '')}/{lab.get('pod', '')}"
        elif key == "temperature_celsius":
            g[f"temp_{lab.get('sensor', '')}"] = v
        elif key in ("gfx_activity_percent", "hbm_activity_percent", "busy_percent", "vram_used_bytes",
                     "vram_total_bytes", "power_watts", "gfxclk_mhz"):
            g[key] = v
            if lab.get("pod"):
                g.setdefault("pod", f"{lab.get('namespace', '')}/{lab['pod']}")
    return gpus


def cmd_top(client: KubeClient, a, out=sys.stdout) -> int:
    """``top node``: one row per MI355X (holding pod, GFX / HBM activity, VRAM, power, clock, hotspot);
    ``top pod``: per pod, its GPUs and their summed use. From the kubelet's /metrics series."""
    if getattr(a, "metrics_url", None):  # split deployment: the node agent serves its own /metrics
        import requests
        r = requests.get(a.metrics_url, timeout=10)
        r.raise_for_status()
        text = r.text
    else:
        text = client._req("GET", "/metrics", raw=True)
    gpus = gpu_table(parse_samples(text))
    if not gpus:
        raise KubectlError("no GPU metrics from the node (kubelet metrics not registered)")
    num = lambda k: (lambda g: g.get(k))  # noqa: E731
    if a.what in ("node", "nodes", "no", "gpu", "gpus"):
        rows = [["GPU", "POD", "GFX%", "HBM%", "VRAM", "POWER", "SCLK", "HOTSPOT"]]
        for key in sorted(gpus, key=lambda x: int(x) if x.isdigit() else 0):
            g = gpus[key]
            act = g.get("gfx_activity_percent", g.get("busy_percent"))
            rows.append([key, g.get("pod", "<none>"), "-" if act is None else f"{act:.0f}%",
                         "-" if num("hbm_activity_percent")(g) is None else f"{g['hbm_activity_percent']:.0f}%",
                         f"{_gib(g.get('vram_used_bytes'))}/{_gib(g.get('vram_total_bytes'))}",
                         "-" if g.get("power_watts") is None else f"{g['power_watts']:.0f}W",
                         "-" if g.get("gfxclk_mhz") is None else f"{g['gfxclk_mhz']:.0f}MHz",
                         "-" if g.get("temp_hotspot") is None else f"{g['temp_hotspot']:.0f}C"])
    elif a.what in ("pod", "pods", "po"):
        pods: dict[str, dict] = {}
        for g in gpus.values():
            if "pod" not in g:
                continue
            ns, pod = g["pod"].split("/", 1)
            if a.namespace and ns != a.namespace:
                continue
            p = pods.setdefault(g["pod"], {"ns": ns, "pod": pod, "gpus": [], "act": [], "vram": 0.0, "power": 0.0})
            p["gpus"].append(g["gpu"])
            act = g.get("gfx_activity_percent", g.get("busy_percent"))
            if act is not None:
                p["act"].append(act)
            p["vram"] += g.get("vram_used_bytes") or 0.0
            p["power"] += g.get("power_watts") or 0.0
        rows = [["NAMESPACE", "POD", "GPUS", "GFX%", "VRAM", "POWER"]]
        for key in sorted(pods):
            p = pods[key]
            rows.append([p["ns"], p["pod"], ",".join(sorted(p["gpus"], key=lambda x: int(x) if x.isdigit() else 0)),
                         f"{sum(p['act']) / len(p['act']):.0f}%" if p["act"] else "-", _gib(p["vram"]),
                         f"{p['power']:.0f}W" if p["power"] else "-"])
        if len(rows) == 1:
            out.write("No GPU pods found" + (f" in {a.namespace} namespace.\n" if a.namespace else ".\n"))
            return 0
    else:
        raise KubectlError(f'error: unknown resource for top: "{a.what}" (node | pod)')
    widths = [max(len(r[i]) for r in rows) for i in range(len(rows[0]))]
    for r in rows:
        out.write("   ".join(c.ljust(w) for c, w in zip(r, widths)).rstrip() + "\n")
    return 0


def load_docs(path: str) -> list[dict]:
    import yaml
    text = sys.stdin.read() if path == "-" else open(path).read()
    return [d for d in yaml.safe_load_all(text) if d]


def add_parsers(sub) -> None:
    def common(p, selector=True):
        p.add_argument("-n", "--namespace", default=None)
        p.add_argument("-A", "--all-namespaces", action="store_true")
        if selector:
            p.add_argument("-l", "--selector", default=None)
        p.add_argument("--server", default=None)

    g = sub.add_parser("get", help="list or read resources")
    g.add_argument("target", nargs="+")
    g.add_argument("-o", "--output", default=None)
    common(g)
    d = sub.add_parser("describe", help="show a resource with its conditions and events")
    d.add_argument("target", nargs="+")
    common(d)
    w = sub.add_parser("wait", help="wait for a condition / jsonpath value / deletion")
    w.add_argument("target", nargs="+")
    w.add_argument("--for", dest="for_", default=None)
    w.add_argument("--timeout", default="30s")
    w.add_argument("--all", action="store_true")
    common(w)
    r = sub.add_parser("rollout", help="rollout status of a StatefulSet / Deployment")
    r.add_argument("action")
    r.add_argument("target", nargs="+")
    r.add_argument("-w", "--watch", action="store_true", default=True)
    r.add_argument("--timeout", default=None)
    common(r, selector=False)
    lg = sub.add_parser("logs", help="print a pod's container log")
    lg.add_argument("pod")
    lg.add_argument("-c", "--container", default=None)
    lg.add_argument("-f", "--follow", action="store_true")
    lg.add_argument("--tail", type=int, default=None)
    lg.add_argument("-n", "--namespace", default=None)
    lg.add_argument("--server", default=None)
    ex = sub.add_parser("exec", help="run a command in a pod's container (no TTY / stdin)")
    ex.add_argument("pod")
    ex.add_argument("-c", "--container", default=None)
    ex.add_argument("-n", "--namespace", default=None)
    ex.add_argument("--timeout", default="30s")
    ex.add_argument("--server", default=None)
    ex.add_argument("command", nargs=argparse.REMAINDER)
    t = sub.add_parser("top", help="GPU use per MI355X (top node) or per pod (top pod), from the kubelet metrics")
    t.add_argument("what", choices=["node", "nodes", "no", "gpu", "gpus", "pod", "pods", "po"])
    t.add_argument("--metrics-url", default=None,
                   help="the node agent's /metrics when it runs apart from the API server (kfamd-node)")
    common(t, selector=False)
    from . import kubectl_mutate
    kubectl_mutate.add_parsers(sub, common)


VERBS = {"get": cmd_get, "describe": cmd_describe, "wait": cmd_wait, "rollout": cmd_rollout, "logs": cmd_logs,
         "top": cmd_top, "exec": cmd_exec}


def _exec_split(a) -> None:
    """kubectl accepts exec's flags after the pod name; argparse's REMAINDER took them with the
    command: move everything before ``--`` back onto the namespace."""
    cmd = list(a.command)
    if "--" not in cmd:
        a.command = cmd
        return
    i = cmd.index("--")
    pre, a.command = cmd[:i], cmd[i + 1:]
    flags = {"-n": "namespace", "--namespace": "namespace", "-c": "container", "--container": "container",
             "--timeout": "timeout", "--server": "server"}
    it = iter(pre)
    for tok in it:
        key, _, val = tok.partition("=")
        if key not in flags:
            raise KubectlError(f"error: unknown flag: {tok}")
        setattr(a, flags[key], val if val else next(it, ""))


def run(verb: str, args, client: KubeClient | None = None) -> int:
    if verb == "exec":
        try:
            _exec_split(args)
        except KubectlError as e:
            sys.stderr.write(str(e) + "\n")
            return 1
    client = client or KubeClient(getattr(args, "server", None))
    if client.warning_handler is None:
        client.warning_handler = print_warning
    if getattr(args, "namespace", None) is None and verb not in ("logs", "exec"):
        args.namespace = None if getattr(args, "all_namespaces", False) else "default"
    try:
        return VERBS[verb](client, args)
    except KubectlError as e:
        sys.stderr.write(str(e) + "\n")
        return 1
    except ApiException as e:
        sys.stderr.write(f"Error from server ({e.reason or e.status}): {e.message}\n")
        return 1
    except OSError as e:  # -f / --cert / --from-file paths, as kubectl words it
        sys.stderr.write(f"error: open {e.filename}: {(e.strerror or str(e)).lower()}\n")
        return 1


from . import kubectl_mutate as _mutate  # noqa: E402 - the writing verbs build on the helpers above

VERBS.update(_mutate.VERBS)
# verbs whose flags may sit between positionals (exec keeps argparse's plain form: its command follows `--`)
INTERMIXED = frozenset(v for v in VERBS if v != "exec")
