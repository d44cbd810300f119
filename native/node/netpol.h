// netpol.h — networking.k8s.io/v1 NetworkPolicy ingress evaluation, as a CNI enforces it: the
// pod's inbound listener (node/gateway.cc handle_inbound) asks whether a connection from `src` to
// `port` of a pod may proceed.
//
// Semantics (k8s NetworkPolicy API): policies in the pod's namespace whose spec.podSelector matches
// the pod and whose policyTypes include Ingress (the default when policyTypes is absent) isolate it;
// an isolated pod accepts a connection only if some ingress rule of some such policy allows it —
// the rule's ports (empty = all; number or named port; endPort ranges; protocol, default TCP) and
// its from peers (empty = everyone; podSelector = pods of the policy's namespace; namespaceSelector
// = every pod of the matching namespaces; both = those pods in those namespaces; ipBlock = CIDR
// minus except). A pod no policy selects is not isolated.
// Reference: ODH's <nb>-ctrl-np / <nb>-oauth-np (odh-notebook-controller/controllers/notebook_network.go:131-210).
#pragma once

#include <map>
#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

struct NetpolSource {
  bool pod = false;                                // a pod (or a workload standing for one)
  std::string ns;                                  // its namespace
  std::map<std::string, std::string> pod_labels;   // its labels ({} when unknown)
  std::map<std::string, std::string> ns_labels;    // its namespace's labels
  std::string ip;                                  // source address (ipBlock peers)
};

struct NetpolDecision {
  bool allowed = true;
  bool isolated = false;   // some policy selects the pod for ingress
  std::string policy;      // the allowing policy, or the (first) isolating one when denied
  std::string reason;
};

// `policies`: NetworkPolicies (any namespace: only pod_ns's apply); `port_name`: the
// containerPort's name ("" when it has none)
NetpolDecision evaluate_netpol(const std::vector<Json>& policies, const std::string& pod_ns,
                               const std::map<std::string, std::string>& pod_labels, int port,
                               const std::string& port_name, const std::string& protocol, const NetpolSource& src);

// "10.0.0.0/8" contains "10.1.2.3" (IPv4)
bool cidr_contains(const std::string& cidr, const std::string& ip);  // false for a malformed CIDR
bool cidr_valid(const std::string& cidr);

}  // namespace kf
