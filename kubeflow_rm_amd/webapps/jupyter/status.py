"""Notebook status derivation for the JWA table (reference jupyter/backend/apps/common/status.py).

Order: freshly created and still empty (<= 10 s) -> stopped/stopping -> terminating -> ready ->
container waiting state -> pod conditions with a reason -> Warning events -> "no information".
Two reference behaviours are kept because the reference's tests pin them: a waiting container
is always reported as a *warning* (the PodInitializing special case never matches upstream), and
the events result does not override the final fallback message.
"""
from __future__ import annotations

import datetime as dt

from kubeflow_rm_amd.webapps.crud_backend import api
from kubeflow_rm_amd.webapps.crud_backend.status import STATUS_PHASE, create_status

EVENT_TYPE_WARNING = "Warning"
STOP_ANNOTATION = "kubeflow-resource-stopped"
TS = "%Y-%m-%dT%H:%M:%SZ"


def process_status(nb: dict) -> dict:
    for fn in (get_empty_status, get_stopped_status, get_deleted_status, check_ready_nb,
               get_status_from_container_state, get_status_from_conditions):
        phase, msg = fn(nb)
        if phase is not None:
            return create_status(phase, msg)
    try:
        get_status_from_events(get_notebook_events(nb))
    except Exception:  # noqa: BLE001 - events are best effort
        pass
    return create_status(STATUS_PHASE.WARNING, "Couldn't find any information for the status of this notebook.")


def get_empty_status(nb: dict):
    created = dt.datetime.strptime(nb.get("metadata", {}).get("creationTimestamp"), TS)
    st = nb.get("status", {}) or {}
    now = dt.datetime.utcnow().replace(microsecond=0)
    if not st.get("containerState") and not st.get("conditions") and (now - created).total_seconds() <= 10:
        return STATUS_PHASE.WAITING, "Waiting for StatefulSet to create the underlying Pod."
    return None, None


def get_stopped_status(nb: dict):
    ready = (nb.get("status") or {}).get("readyReplicas", 0)
    if STOP_ANNOTATION in ((nb.get("metadata") or {}).get("annotations") or {}):
        if ready == 0:
            return STATUS_PHASE.STOPPED, "No Pods are currently running for this Notebook Server."
        return STATUS_PHASE.WAITING, "Notebook Server is stopping."
    return None, None


def get_deleted_status(nb: dict):
    if "deletionTimestamp" in (nb.get("metadata") or {}):
        return STATUS_PHASE.TERMINATING, "Deleting this Notebook Server."
    return None, None


def check_ready_nb(nb: dict):
    if (nb.get("status") or {}).get("readyReplicas", 0) == 1:
        return STATUS_PHASE.READY, "Running"
    return None, None


def get_status_from_container_state(nb: dict):
    cs = (nb.get("status") or {}).get("containerState", {}) or {}
    if "waiting" not in cs:
        return None, None
    waiting = cs["waiting"]
    reason = waiting.get("reason", "Undefined")
    message = waiting.get("message", "No available message for container state.")
    return STATUS_PHASE.WARNING, f"{reason}: {message}"


def get_status_from_conditions(nb: dict):
    for cond in (nb.get("status") or {}).get("conditions", []) or []:
        if "reason" in cond:
            return STATUS_PHASE.WARNING, cond["reason"] + ": " + cond.get("message", "")
    return None, None


def event_timestamp(ev: dict) -> dt.datetime:
    return dt.datetime.strptime(ev["metadata"]["creationTimestamp"][:19] + "Z", TS)


def get_notebook_events(nb: dict) -> list:
    created = dt.datetime.strptime(nb["metadata"]["creationTimestamp"], TS)
    events = api.list_notebook_events(nb["metadata"]["name"], nb["metadata"]["namespace"])["items"]
    return [e for e in events if event_timestamp(e) >= created]


def get_status_from_events(events: list):
    for e in sorted(events, key=event_timestamp, reverse=True):
        if e.get("type") == EVENT_TYPE_WARNING:
            return STATUS_PHASE.WARNING, e.get("message")
    return None, None
