"""Client-side ``kubectl apply``: last-applied-configuration + three-way strategic merge patch.

The reference's CI drives every object through ``kubectl apply -f``
(/root/reference/.github/workflows/odh_notebook_controller_integration_test.yaml:101,139,152,172,205,228,
notebook_controller_integration_test.yaml:92,105). kubectl's client-side apply:

* stores the applied manifest in ``metadata.annotations["kubectl.kubernetes.io/last-applied-configuration"]``;
* on re-apply computes a patch from three documents — ``original`` (the last applied), ``modified``
  (the new manifest) and ``current`` (the live object):
    - a field in ``original`` but not in ``modified`` is deleted (``null`` in a map, ``$patch: delete``
      for an item of a list merged by key);
    - a field in ``modified`` whose value differs from ``current`` is set;
    - a field only in ``current`` (set by the server, a controller or a mutating webhook — e.g. the
      ODH webhook's ``oauth-proxy`` sidecar) is left alone;
* lists of objects are merged by their strategic merge key (``containers`` / ``initContainers`` /
  ``env`` / ``volumes`` / ``imagePullSecrets`` by ``name``, ``volumeMounts`` by ``mountPath``,
  container ``ports`` by ``containerPort``, Service ``ports`` by ``port``), other lists replaced whole;
* an empty patch is not sent: the object is ``unchanged`` (same resourceVersion, no admission).

The patch goes to the API server as ``application/strategic-merge-patch+json``
(native/core/json.cc strategic_merge_patch).
"""
from __future__ import annotations

import copy
import json

LAST_APPLIED = "kubectl.kubernetes.io/last-applied-configuration"

# field name -> merge key of its list items (the server's table, native/core/json.cc merge_key_for)
MERGE_KEYS = {
    "containers": "name", "initContainers": "name", "ephemeralContainers": "name", "volumes": "name",
    "env": "name", "imagePullSecrets": "name", "volumeMounts": "mountPath", "volumeDevices": "devicePath",
    "ports": "containerPort", "hostAliases": "ip",
}


def _merge_key(field: str, items: list) -> str | None:
    key = MERGE_KEYS.get(field)
    if key is None:
        return None
    if field == "ports" and items and all(isinstance(i, dict) and "containerPort" not in i and "port" in i
                                          for i in items):
        return "port"  # Service ports
    if not all(isinstance(i, dict) and key in i for i in items):
        return None  # not mergeable by key: replace the whole list
    return key


def _list_patch(field: str, original: list, modified: list, current: list):
    """Patch of a list field, or None for no change. Keyed lists get per-item patches."""
    key = _merge_key(field, modified + original + current)
    if key is None:
        return None if modified == current else copy.deepcopy(modified)
    cur = {i[key]: i for i in current}
    orig = {i[key]: i for i in original}
    mod_keys = {i[key] for i in modified}
    ops = []
    for k, item in orig.items():
        if k not in mod_keys and k in cur:
            ops.append({key: k, "$patch": "delete"})
    for item in modified:
        k = item[key]
        if k not in cur:
            ops.append(copy.deepcopy(item))
            continue
        sub = three_way_patch(orig.get(k, {}), item, cur[k])
        if sub:
            sub[key] = k
            ops.append(sub)
    return ops or None


def three_way_patch(original: dict | None, modified: dict, current: dict | None) -> dict:
    """kubectl's three-way strategic merge patch (client-side apply). Empty dict = nothing to do."""
    original = original if isinstance(original, dict) else {}
    current = current if isinstance(current, dict) else {}
    patch: dict = {}
    for k in original:
        if k not in modified and k in current:
            patch[k] = None
    for k, mv in modified.items():
        cv, ov = current.get(k), original.get(k)
        if isinstance(mv, dict) and isinstance(cv, dict):
            sub = three_way_patch(ov if isinstance(ov, dict) else {}, mv, cv)
            if sub:
                patch[k] = sub
        elif isinstance(mv, list) and isinstance(cv, list):
            sub = _list_patch(k, ov if isinstance(ov, list) else [], mv, cv)
            if sub is not None:
                patch[k] = sub
        elif mv != cv:
            patch[k] = copy.deepcopy(mv)
    return patch


def last_applied_of(obj: dict) -> dict | None:
    raw = ((obj.get("metadata") or {}).get("annotations") or {}).get(LAST_APPLIED)
    if not raw:
        return None
    try:
        return json.loads(raw)
    except ValueError:
        return None


def with_last_applied(manifest: dict) -> dict:
    """The manifest carrying its own last-applied annotation (what kubectl stores)."""
    m = copy.deepcopy(manifest)
    ann = (m.setdefault("metadata", {}).get("annotations") or {})
    ann.pop(LAST_APPLIED, None)
    bare = copy.deepcopy(m)
    if not ann:
        bare["metadata"].pop("annotations", None)
    m["metadata"]["annotations"] = {**ann, LAST_APPLIED: json.dumps(bare, sort_keys=True, separators=(",", ":"))}
    return m


def apply_object(client, manifest: dict, dry_run: bool = False) -> tuple[str, dict]:
    """Create or three-way-patch one object. Returns (verb, object) with verb "created",
    "configured" or "unchanged" (kubectl's words)."""
    from .client import ApiException
    manifest = copy.deepcopy(manifest)
    md = manifest.setdefault("metadata", {})
    if not md.get("namespace") and client.resource(manifest["apiVersion"], manifest["kind"])[1]:
        md["namespace"] = "default"  # kubectl's default namespace for a namespaced kind
    modified = with_last_applied(manifest)
    try:
        current = client.get(manifest["apiVersion"], manifest["kind"], md["name"], md.get("namespace"))
    except ApiException as e:
        if e.status != 404:
            raise
        current = None
    if current is None:
        try:
            return "created", client.create(modified, namespace=md.get("namespace"), dry_run=dry_run)
        except ApiException as e:
            if e.status != 409:  # created meanwhile: fall through to a patch
                raise
            current = client.get(manifest["apiVersion"], manifest["kind"], md["name"], md.get("namespace"))
    original = last_applied_of(current)
    if original is None:
        # no annotation (created by something else): kubectl warns and uses the live object's view
        # of the manifest's fields as the original, so nothing the manifest omits is deleted
        original = {}
    patch = three_way_patch(original, modified, current)
    if not patch:
        return "unchanged", current
    out = client.patch(manifest["apiVersion"], manifest["kind"], md["name"], patch, md.get("namespace"),
                       "strategic", dry_run=dry_run)
    return "configured", out
