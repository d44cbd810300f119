"""kfctl — render and apply the platform's manifests (kustomize-lite + the REST client).

    python -m kubeflow_rm_amd.kfctl build manifests/example            # multi-doc YAML on stdout
    python -m kubeflow_rm_amd.kfctl apply manifests/example [--server URL] [--dry-run]
    python -m kubeflow_rm_amd.kfctl delete manifests/example [--server URL]
    python -m kubeflow_rm_amd.kfctl crds [--out manifests/crds]         # regenerate CRD YAML from
                                                                        # the native registry
    python -m kubeflow_rm_amd.kfctl up [--data-dir DIR]                  # local kube-lite cluster
    python -m kubeflow_rm_amd.kfctl apply -f notebook.yaml | -           # kubectl-style file apply
    python -m kubeflow_rm_amd.kfctl get|describe|wait|rollout|logs|exec|top ...   # kubectl subset (kubectl.py)

Apply order follows kubectl's dependency order (Namespaces and CRDs first, webhooks last) so
that every object's kind and namespace exist when it arrives; ``--dry-run`` sends every object
with ``dryRun=All`` (server-side validation, admission and defaulting, nothing stored).
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

from . import kustomize
from .client import ApiException, KubeClient, print_warning

ORDER = ["Namespace", "CustomResourceDefinition", "ClusterRole", "ClusterRoleBinding", "ServiceAccount", "Role",
         "RoleBinding", "ConfigMap", "Secret", "PersistentVolumeClaim", "Service", "Deployment", "StatefulSet",
         "DaemonSet", "Gateway", "VirtualService", "AuthorizationPolicy"]
LAST = ["MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"]


def apply_order(objs: list[dict]) -> list[dict]:
    def key(o):
        k = o.get("kind", "")
        if k in LAST:
            return (len(ORDER) + 1 + LAST.index(k),)
        return (ORDER.index(k) if k in ORDER else len(ORDER),)
    return sorted(objs, key=key)


def apply(client: KubeClient, objs: list[dict], dry_run: bool = False, log=print) -> list[str]:
    """``kubectl apply`` every object in dependency order (kubeflow_rm_amd.apply: last-applied
    annotation + three-way strategic merge patch). ``dry_run``: the same requests with dryRun=All
    (server-side: validation, admission, defaulting, nothing stored), so a changed object reports
    "configured" from a real diff. Returns "kind/name verb" lines (created / configured / unchanged)."""
    from .apply import apply_object
    done = []
    for o in apply_order(objs):
        md = o["metadata"]
        verb, live = apply_object(client, o, dry_run=dry_run)
        ns = md.get("namespace") or ((live or {}).get("metadata") or {}).get("namespace")
        ref = f"{o['kind']}/{md['name']}" + (f" -n {ns}" if ns else "")
        if dry_run:
            verb += " (server dry run)"
        elif o["kind"] == "CustomResourceDefinition" and verb != "unchanged":
            _wait_crd(client, o)
        done.append(f"{ref} {verb}")
        if log:
            log(f"{ref} {verb}")
    return done


def _wait_crd(client: KubeClient, crd: dict, timeout: float = 10.0) -> None:
    group = crd["spec"]["group"]
    version = next(v["name"] for v in crd["spec"]["versions"] if v.get("served", True))
    kind = crd["spec"]["names"]["kind"]
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            client.resource(f"{group}/{version}", kind)
            return
        except Exception:  # noqa: BLE001 - discovery not refreshed yet
            time.sleep(0.1)


def delete(client: KubeClient, objs: list[dict], log=print) -> None:
    for o in reversed(apply_order(objs)):
        md = o["metadata"]
        try:
            client.delete(o["apiVersion"], o["kind"], md["name"], md.get("namespace"))
            if log:
                log(f"{o['kind']}/{md['name']} deleted")
        except ApiException as e:
            if e.status != 404:
                raise


def write_crds(out: Path) -> list[Path]:
    import yaml

    from . import native
    out.mkdir(parents=True, exist_ok=True)
    paths = []
    for c in native.call("builtin_crds"):
        plural, group = c["metadata"]["name"].split(".", 1)
        body = {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
                "metadata": {"name": c["metadata"]["name"]}, "spec": c["spec"]}
        sub = out if "kubeflow" in group else out / "external"
        sub.mkdir(parents=True, exist_ok=True)
        p = sub / f"{group}_{plural}.yaml"
        p.write_text("# generated from the kube-lite builtin CRD registry (native/apiserver/resources.cc): "
                     "python -m kubeflow_rm_amd.kfctl crds\n" + yaml.safe_dump(body, sort_keys=False))
        paths.append(p)
    return paths


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="kfctl")
    sub = ap.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("build")
    b.add_argument("path")
    for name in ("apply", "delete"):
        s = sub.add_parser(name)
        s.add_argument("path", nargs="*", help="kustomize dir (or, for delete, <resource> <name>)")
        s.add_argument("-f", "--filename", default=None, help="YAML/JSON manifest file, '-' for stdin")
        s.add_argument("-n", "--namespace", default=None)
        s.add_argument("--server", default=None)
        if name == "apply":
            s.add_argument("--dry-run", action="store_true")
    from . import kubectl
    kubectl.add_parsers(sub)
    c = sub.add_parser("crds")
    c.add_argument("--out", default=str(Path(__file__).resolve().parent.parent / "manifests" / "crds"))
    u = sub.add_parser("up")
    u.add_argument("--data-dir", default=None)
    argv = sys.argv[1:] if argv is None else list(argv)
    if argv and argv[0] in kubectl.INTERMIXED:
        # kubectl takes flags between positionals (`create secret tls -n NS NAME --cert=...`);
        # argparse only allows that per sub-parser, via parse_intermixed_args
        args = sub.choices[argv[0]].parse_intermixed_args(argv[1:])
        args.cmd = argv[0]
    else:
        args = ap.parse_args(argv)
    if args.cmd == "build":
        sys.stdout.write(kustomize.dump(kustomize.build(args.path)))
        return 0
    if args.cmd in kubectl.VERBS:
        return kubectl.run(args.cmd, args)
    if args.cmd in ("apply", "delete"):
        client = KubeClient(args.server)
        client.warning_handler = print_warning
        try:
            if args.filename:
                objs = kubectl.load_docs(args.filename)
                for o in objs:
                    if args.namespace and "namespace" not in o.setdefault("metadata", {}):
                        o["metadata"]["namespace"] = args.namespace
            elif args.cmd == "delete" and len(args.path) == 2:  # delete <resource> <name>
                res = kubectl.resolve(client, args.path[0])
                client.delete(res.api_version, res.kind, args.path[1], (args.namespace or "default") if res.namespaced else None)
                print(f'{res.kind.lower()}{"." + res.group if res.group else ""} "{args.path[1]}" deleted')
                return 0
            elif len(args.path) == 1:
                objs = kustomize.build(args.path[0])
            else:
                print("error: must specify one of -f or a kustomize directory", file=sys.stderr)
                return 1
            if args.cmd == "apply":
                apply(client, objs, dry_run=args.dry_run)
            else:
                delete(client, objs)
        except (ApiException, kubectl.KubectlError) as e:
            print(e if isinstance(e, kubectl.KubectlError) else f"Error from server ({e.reason or e.status}): {e.message}",
                  file=sys.stderr)
            return 1
        return 0
    if args.cmd == "crds":
        for p in write_crds(Path(args.out)):
            print(p)
        return 0
    if args.cmd == "up":
        from .cluster import LocalCluster
        cl = LocalCluster(data_dir=args.data_dir, zygote=None).start()
        print(f"kube-lite API {cl.url}  gateway {cl.gateway}  kfam {cl.kfam}  (Ctrl-C to stop)", flush=True)
        try:
            while True:
                time.sleep(3600)
        except KeyboardInterrupt:
            cl.stop()
        return 0
    return 2


if __name__ == "__main__":
    sys.exit(main())
