"""Profile controller pure functions (native).

Ported cases:
  reference components/profile-controller/controllers/profile_controller_test.go:23-122 (namespace labels)
  reference components/profile-controller/controllers/plugin_iam_test.go:23-313 (AWS trust policy)
  reference components/profile-controller/controllers/plugin_workload_identity_test.go:27-134 (GCP bindings)
"""
import json

import pytest

NAME = "test-namespace"
DEFAULTS = {
    "katib.kubeflow.org/metrics-collector-injection": "enabled",
    "serving.kubeflow.org/inferenceservice": "enabled",
    "pipelines.kubeflow.org/enabled": "true",
    "app.kubernetes.io/part-of": "kubeflow-profile",
}

LABEL_CASES = [
    ({"name": NAME}, DEFAULTS, {"name": NAME, "labels": DEFAULTS}),
    ({"name": NAME, "labels": {"user-name": "Jim", "serving.kubeflow.org/inferenceservice": "disabled"}}, DEFAULTS,
     {"name": NAME, "labels": {**DEFAULTS, "user-name": "Jim", "serving.kubeflow.org/inferenceservice": "disabled"}}),
    ({"name": NAME, "labels": {"user-name": "Jim", "removal-label": "enabled"}}, {**DEFAULTS, "removal-label": ""},
     {"name": NAME, "labels": {**DEFAULTS, "user-name": "Jim"}}),
]


@pytest.mark.parametrize("meta,labels,want", LABEL_CASES)
def test_enforce_namespace_labels_from_config(native, meta, labels, want):
    got = native.call("set_namespace_labels", namespace={"metadata": meta}, labels=labels)
    assert got["metadata"] == want


def test_namespace_labels_file_parsing(native):
    # the shipped config file format (profile-controller/config/base/namespace-labels.yaml)
    text = """# comment
katib.kubeflow.org/metrics-collector-injection: "enabled"
serving.kubeflow.org/inferenceservice: 'enabled'
pipelines.kubeflow.org/enabled: "true"
app.kubernetes.io/part-of: kubeflow-profile   # trailing comment
removal-label: ""
"""
    r = native.call("parse_flat_yaml_map", text=text)
    assert r["ok"]
    assert r["map"] == {**DEFAULTS, "removal-label": ""}
    assert native.call("parse_flat_yaml_map", text="not a map line")["ok"] is False


ISSUER = "oidc.beta.us-west-2.wesley.amazonaws.com/id/50D94CFC65139194EDC21891B611EF72"
PROVIDER = f"arn:aws:iam::34892524:oidc-provider/{ISSUER}"


def _policy(subs=None, action="sts:AssumeRoleWithWebIdentity"):
    se = {f"{ISSUER}:aud": ["sts.amazonaws.com"]}
    if subs is not None:
        se[f"{ISSUER}:sub"] = subs
    return {"Version": "2012-10-17", "Statement": [{"Effect": "Allow", "Principal": {"Federated": PROVIDER},
                                                    "Action": action, "Condition": {"StringEquals": se}}]}


def test_issuer_and_role_name(native):
    assert native.call("get_issuer_url_from_provider_arn", arn=PROVIDER) == ISSUER
    assert native.call("get_iam_role_name_from_iam_role_arn", arn="arn:aws:iam::34892524:role/test-iam-role") == "test-iam-role"


@pytest.mark.parametrize("before,after", [
    (None, ["system:serviceaccount:ns1:sa1"]),
    ([], ["system:serviceaccount:ns1:sa1"]),
    (["system:serviceaccount:ns1:sa2"], ["system:serviceaccount:ns1:sa2", "system:serviceaccount:ns1:sa1"]),
])
def test_add_service_account_in_assume_role_policy(native, before, after):
    r = native.call("add_service_account_in_assume_role_policy", doc=json.dumps(_policy(before)), namespace="ns1", sa="sa1")
    assert json.loads(r["doc"]) == _policy(after)


def test_add_service_account_already_present(native):
    doc = json.dumps(_policy(["system:serviceaccount:ns1:sa1"]))
    r = native.call("add_service_account_in_assume_role_policy", doc=doc, namespace="ns1", sa="sa1")
    assert r["exists"] is True and r["changed"] is False


@pytest.mark.parametrize("before,after", [
    (["system:serviceaccount:ns1:sa1", "system:serviceaccount:ns1:sa2"], ["system:serviceaccount:ns1:sa1"]),
    (["system:serviceaccount:ns1:sa2"], None),
])
def test_remove_service_account_in_assume_role_policy(native, before, after):
    doc = json.dumps(_policy(before, action=["sts:AssumeRoleWithWebIdentity"]))
    r = native.call("remove_service_account_in_assume_role_policy", doc=doc, namespace="ns1", sa="sa2")
    assert json.loads(r["doc"]) == _policy(after)


def test_gcp_project_id(native):
    assert native.call("gcp_project_id", sa="kubeflow@project-id.iam.gserviceaccount.com") == "project-id"


def test_gcp_add_and_revoke_binding(native):
    role = "roles/iam.workloadIdentityUser"
    base = ["serviceAccount:kfctl.svc.id.goog[istio-system/kf-user]", "serviceAccount:kfctl.svc.id.goog[kubeflow-user1/default-editor]"]
    pol = {"bindings": [{"role": role, "members": list(base)}], "etag": "ShouldKeep"}
    out = native.call("gcp_add_binding", policy=pol, member="serviceAccount:kfctl.svc.id.goog[should/add]")
    assert out == {"bindings": [{"role": role, "members": base},
                                {"role": role, "members": ["serviceAccount:kfctl.svc.id.goog[should/add]"]}], "etag": "ShouldKeep"}
    pol = {"bindings": [{"role": role, "members": base + ["serviceAccount:kfctl.svc.id.goog[should/remove]"]}], "etag": "ShouldKeep"}
    out = native.call("gcp_revoke_binding", policy=pol, member="serviceAccount:kfctl.svc.id.goog[should/remove]")
    assert out == {"bindings": [{"role": role, "members": base}], "etag": "ShouldKeep"}


def test_authorization_policy_spec(native):
    prof = {"metadata": {"name": "alice"}, "spec": {"owner": {"kind": "User", "name": "alice@example.com"}}}
    spec = native.call("authorization_policy_spec", profile=prof, userid_header="kubeflow-userid", userid_prefix="")
    assert spec["action"] == "ALLOW"
    rules = spec["rules"]
    assert len(rules) == 4
    assert rules[0]["when"][0] == {"key": "request.headers[kubeflow-userid]", "values": ["alice@example.com"]}
    assert rules[1]["when"][0] == {"key": "source.namespace", "values": ["alice"]}
    assert rules[2]["to"][0]["operation"]["paths"] == ["/healthz", "/metrics", "/wait-for-drain"]
    assert rules[3]["to"][0]["operation"] == {"methods": ["GET"], "paths": ["*/api/kernels"]}
