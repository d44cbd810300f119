"""Kubernetes calls made on the user's behalf (each authorized with a SubjectAccessReview) and the
JSON response envelope of the CRUD apps ({success, status, user, <field>: data})."""
from __future__ import annotations

from flask import jsonify

from . import authn, authz, k8s

NB_GROUP, NB_VERSION = "kubeflow.org", "v1beta1"


def success_response(data_field=None, data=None):
    resp = {"status": 200, "success": True, "user": authn.get_username()}
    if data_field is not None or data is not None:
        resp[data_field] = data
    return jsonify(resp)


def failed_response(msg, code):
    return {"success": False, "log": msg, "status": code, "user": authn.get_username()}, code


def events_field_selector(kind: str, name: str) -> str:
    return f"involvedObject.kind={kind},involvedObject.name={name}"


def _c():
    return k8s.client()


# ---- core/v1 ----------------------------------------------------------------------------------
def list_namespaces():
    authz.ensure_authorized("list", "", "v1", "namespaces")
    return _c().list("v1", "Namespace")


def list_pvcs(namespace):
    authz.ensure_authorized("list", "", "v1", "persistentvolumeclaims", namespace)
    return _c().list("v1", "PersistentVolumeClaim", namespace)


def get_pvc(name, namespace):
    authz.ensure_authorized("get", "", "v1", "persistentvolumeclaims", namespace)
    return _c().get("v1", "PersistentVolumeClaim", name, namespace)


def create_pvc(pvc, namespace, dry_run=False):
    authz.ensure_authorized("create", "", "v1", "persistentvolumeclaims", namespace)
    pvc = dict(pvc, apiVersion="v1", kind="PersistentVolumeClaim")
    return _c().create(pvc, namespace=namespace, dry_run=dry_run)


def delete_pvc(name, namespace):
    authz.ensure_authorized("delete", "", "v1", "persistentvolumeclaims", namespace)
    return _c().delete("v1", "PersistentVolumeClaim", name, namespace)


def list_pods(namespace, label_selector=""):
    authz.ensure_authorized("list", "", "v1", "pods", namespace)
    return _c().list("v1", "Pod", namespace, label_selector=label_selector)


def get_pod_logs(namespace, pod, container):
    authz.ensure_authorized("get", "", "v1", "pods", namespace, "log")
    return _c().pod_logs(pod, namespace, container=container)


def list_events(namespace, field_selector):
    authz.ensure_authorized("list", "", "v1", "events", namespace)
    return _c().list("v1", "Event", namespace, field_selector=field_selector)


def list_nodes():
    # the app's own service account (no per-user SAR), as the reference does for GPU discovery
    return _c().list("v1", "Node")


def list_secrets(namespace):
    authz.ensure_authorized("list", "", "v1", "secrets", namespace)
    return _c().list("v1", "Secret", namespace)


def list_storageclasses():
    authz.ensure_authorized("list", "storage.k8s.io", "v1", "storageclasses")
    return _c().list("storage.k8s.io/v1", "StorageClass")


# ---- custom resources -------------------------------------------------------------------------
def list_poddefaults(namespace):
    authz.ensure_authorized("list", "kubeflow.org", "v1alpha1", "poddefaults", namespace)
    return _c().list("kubeflow.org/v1alpha1", "PodDefault", namespace)


def get_notebook(name, namespace):
    authz.ensure_authorized("get", NB_GROUP, NB_VERSION, "notebooks", namespace)
    return _c().get(f"{NB_GROUP}/{NB_VERSION}", "Notebook", name, namespace)


def list_notebooks(namespace):
    authz.ensure_authorized("list", NB_GROUP, NB_VERSION, "notebooks", namespace)
    return _c().list(f"{NB_GROUP}/{NB_VERSION}", "Notebook", namespace)


def create_notebook(notebook, namespace, dry_run=False):
    authz.ensure_authorized("create", NB_GROUP, NB_VERSION, "notebooks", namespace)
    return _c().create(notebook, namespace=namespace, dry_run=dry_run)


def patch_notebook(name, namespace, body):
    authz.ensure_authorized("patch", NB_GROUP, NB_VERSION, "notebooks", namespace)
    return _c().patch(f"{NB_GROUP}/{NB_VERSION}", "Notebook", name, body, namespace, "merge")


def delete_notebook(name, namespace):
    authz.ensure_authorized("delete", NB_GROUP, NB_VERSION, "notebooks", namespace)
    return _c().delete(f"{NB_GROUP}/{NB_VERSION}", "Notebook", name, namespace, propagation_policy="Foreground")


def list_notebook_events(name, namespace):
    return list_events(namespace, events_field_selector("Notebook", name))


def custom_api(verb, group, version, plural, kind, namespace, name=None, body=None, dry_run=False, propagation=None):
    authz.ensure_authorized(verb, group, version, plural, namespace)
    av = f"{group}/{version}"
    c = _c()
    if verb == "list":
        return c.list(av, kind, namespace)
    if verb == "get":
        return c.get(av, kind, name, namespace)
    if verb == "create":
        return c.create(body, namespace=namespace, dry_run=dry_run)
    if verb == "delete":
        return c.delete(av, kind, name, namespace, propagation_policy=propagation)
    if verb == "patch":
        return c.patch(av, kind, name, body, namespace, "merge")
    raise ValueError(verb)


def list_pvc_events(namespace, pvc_name):
    return list_events(namespace, events_field_selector("PersistentVolumeClaim", pvc_name))
