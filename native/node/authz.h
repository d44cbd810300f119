// authz.h — Istio AuthorizationPolicy (security.istio.io/v1beta1) evaluation for the gateway's
// policy enforcement points: the ingress listener (end-user traffic, principal = the ingress
// gateway's) and the mesh listener (in-cluster callers, principal = their ServiceAccount).
//
// What the reference relies on Istio for:
//  * profile-controller/controllers/profile_controller.go:419-556 — ns-owner-access-istio: the owner's
//    userid header via the ingress-gateway / KFP-UI principals; same-namespace traffic; /healthz
//    /metrics /wait-for-drain; the notebook-controller principal's GET */api/kernels;
//  * access-management/kfam/bindings.go:112-155 — one ALLOW policy per contributor binding on
//    request.headers[<userid-header>].
//
// Semantics implemented (Istio's documented model, evaluated per destination workload):
//  * applicable policies: those in the workload's namespace whose selector matches the workload's
//    labels (no selector = every workload), plus those in the root namespace (mesh-wide);
//  * CUSTOM is not supported (ignored); any matching DENY rule denies; if any ALLOW policy applies
//    the request must match one of its rules, otherwise it is allowed;
//  * a policy without rules matches nothing (ALLOW {} = allow-nothing); a rule with no from / to /
//    when matches everything; from/to entries are OR-ed, the fields inside one entry AND-ed, and
//    every `when` condition must hold;
//  * string matches are exact, "prefix*", "*suffix" or "*" (any non-empty value); hosts compare
//    case-insensitively; ip blocks are IPv4 CIDRs.
#pragma once

#include <map>
#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

struct AuthzRequest {
  std::string principal;         // source.principal, e.g. cluster.local/ns/kubeflow/sa/notebook-controller-service-account
  std::string source_namespace;  // source.namespace
  std::string source_ip, remote_ip;
  std::string request_principal;  // request.auth.principal (JWT); empty here
  std::string method, path, host;
  int port = 0;
  std::map<std::string, std::string> headers;  // lower-case names
};

struct AuthzDecision {
  bool allowed = true;
  std::string policy;  // "<ns>/<name>" of the deciding policy ("" = no ALLOW policy applied)
  std::string reason;
};

bool istio_string_match(const std::string& pattern, const std::string& value);

// Istio's default pathNormalization (BASE) of an already percent-decoded request path: backslashes
// become slashes and RFC 3986 §5.2.4 remove_dot_segments collapses "." / ".." segments (never above
// the root). A decoded '?' or '#' stays part of the path: policies are matched on, and the request
// is forwarded with, exactly this string (/x/../admin, /./, %3F no longer slip past a
// DENY paths rule).
std::string normalize_authz_path(const std::string& decoded_path);
// The path as an upstream request-line token: every byte outside RFC 3986 pchar ('/' included)
// percent-encoded, so a decoded '?', '#', '%' or space reaches the backend as data, not syntax.
std::string encode_request_path(const std::string& path);
bool ipv4_in_cidr(const std::string& ip, const std::string& cidr);

// policies: AuthorizationPolicy objects (any namespaces; filtered here); workload_ns / labels: the
// destination workload
AuthzDecision evaluate_authz(const std::vector<Json>& policies, const AuthzRequest& r, const std::string& workload_ns,
                             const std::map<std::string, std::string>& workload_labels,
                             const std::string& root_namespace = "istio-system");

}  // namespace kf
