"""API volumes of the spawner form -> PVCs, pod volumes and mounts.

An API volume is ``{mount, newPvc?: {metadata, spec}, existingSource?: {<V1VolumeSource>}}``.
"""
from __future__ import annotations

import copy

from werkzeug.exceptions import BadRequest

from . import utils

PVC_SOURCE = "persistentVolumeClaim"
EXISTING_SOURCE = "existingSource"
NEW_PVC = "newPvc"
MOUNT = "mount"
NAME = "name"


def check_volume_format(v: dict) -> None:
    if MOUNT not in v:
        raise BadRequest(f"Volume should have a mount: {v}")
    if EXISTING_SOURCE not in v and NEW_PVC not in v:
        raise BadRequest(f"Volume has neither {EXISTING_SOURCE} nor {NEW_PVC}: {v}")
    if EXISTING_SOURCE in v and NEW_PVC in v:
        raise BadRequest(f"Volume has both {EXISTING_SOURCE} and {NEW_PVC}: {v}")


def get_volume_name(v: dict) -> str:
    if EXISTING_SOURCE not in v:
        raise BadRequest(f"Failed to retrieve a volume name from '{v}'")
    src = v[EXISTING_SOURCE]
    if PVC_SOURCE in src:
        if "claimName" not in src[PVC_SOURCE]:
            raise BadRequest(f"Failed to retrieve the PVC name from '{v}'")
        return src[PVC_SOURCE]["claimName"]
    return "existing-source-volume-" + utils.random_string(8)


def get_pod_volume(v: dict, pvc: dict | None) -> dict:
    check_volume_format(v)
    if pvc is not None:
        name = pvc["metadata"]["name"]
        return {"name": name, "persistentVolumeClaim": {"claimName": name}}
    vol = {"name": get_volume_name(v)}
    vol.update(v[EXISTING_SOURCE])
    return vol


def get_container_mount(v: dict, volume_name: str) -> dict:
    check_volume_format(v)
    return {"name": volume_name, "mountPath": v[MOUNT]}


def get_new_pvc(v: dict, notebook_name: str | None = None) -> dict | None:
    check_volume_format(v)
    if NEW_PVC not in v:
        return None
    pvc = copy.deepcopy(v[NEW_PVC])
    md = pvc.setdefault("metadata", {})
    if md.get("namespace") is not None:
        raise BadRequest("PVC should not specify the namespace.")
    if notebook_name and "{notebook-name}" in md.get("name", ""):
        md["name"] = md["name"].replace("{notebook-name}", notebook_name)
    if not isinstance(pvc.get("spec"), dict):
        raise BadRequest(f"PVC spec missing in {v}")
    return pvc


def add_notebook_volume(nb: dict, volume: dict) -> dict:
    nb["spec"]["template"]["spec"].setdefault("volumes", []).append(volume)
    return nb


def add_notebook_container_mount(nb: dict, mount: dict) -> dict:
    nb["spec"]["template"]["spec"]["containers"][0].setdefault("volumeMounts", []).append(mount)
    return nb
