// netpol.cc — see netpol.h.
#include "node/netpol.h"

#include <arpa/inet.h>

#include "apiserver/selector.h"
#include "core/util.h"

namespace kf {

namespace {
Json labels_json(const std::map<std::string, std::string>& m) {
  Json j = Json::object();
  for (const auto& kv : m) j[kv.first] = kv.second;
  return j;
}

bool policy_is_ingress(const Json& np) {
  const Json& types = np.at_path({"spec", "policyTypes"});
  if (!types.is_array() || types.empty()) return true;  // default: Ingress (plus Egress when egress rules exist)
  for (const auto& t : types.as_array())
    if (t.as_string() == "Ingress") return true;
  return false;
}

bool port_matches(const Json& ports, int port, const std::string& port_name, const std::string& protocol) {
  if (!ports.is_array() || ports.empty()) return true;
  for (const auto& p : ports.as_array()) {
    if (p["protocol"].as_string_or("TCP") != protocol) continue;
    const Json& want = p["port"];
    if (want.is_null()) return true;  // all ports of the protocol
    if (want.is_string()) {
      if (!port_name.empty() && want.as_string() == port_name) return true;
      continue;
    }
    const int64_t lo = want.as_int(), hi = p["endPort"].is_number() ? p["endPort"].as_int() : lo;
    if (port >= lo && port <= hi) return true;
  }
  return false;
}

bool peer_matches(const Json& peer, const std::string& policy_ns, const NetpolSource& src) {
  if (peer["ipBlock"].is_object()) {
    if (src.ip.empty() || !cidr_contains(peer.at_path({"ipBlock", "cidr"}).as_string(), src.ip)) return false;
    for (const auto& ex : peer.at_path({"ipBlock", "except"}).as_array())  // a malformed exception excludes (closed)
      if (!cidr_valid(ex.as_string()) || cidr_contains(ex.as_string(), src.ip)) return false;
    return true;
  }
  const bool has_pod = peer["podSelector"].is_object(), has_ns = peer["namespaceSelector"].is_object();
  if (!has_pod && !has_ns) return false;
  if (!src.pod) return false;  // selectors match pods only
  if (has_ns) {
    if (!LabelSelector::from_json(peer["namespaceSelector"]).matches(labels_json(src.ns_labels))) return false;
  } else if (src.ns != policy_ns) {
    return false;  // a bare podSelector means pods of the policy's own namespace
  }
  return !has_pod || LabelSelector::from_json(peer["podSelector"]).matches(labels_json(src.pod_labels));
}
}  // namespace

namespace {
// "a.b.c.d/n" (n = 0..32, digits only) or a bare address (/32); anything else is malformed
bool parse_cidr(const std::string& cidr, uint32_t& net, int& bits) {
  const size_t slash = cidr.find('/');
  bits = 32;
  if (slash != std::string::npos) {
    const std::string n = cidr.substr(slash + 1);
    if (n.empty() || n.size() > 2 || n.find_first_not_of("0123456789") != std::string::npos) return false;
    bits = std::stoi(n);
    if (bits > 32) return false;
  }
  in_addr a{};
  if (::inet_pton(AF_INET, cidr.substr(0, slash).c_str(), &a) != 1) return false;
  net = ntohl(a.s_addr);
  return true;
}
}  // namespace

bool cidr_valid(const std::string& cidr) {
  uint32_t net = 0;
  int bits = 0;
  return parse_cidr(cidr, net, bits);
}

bool cidr_contains(const std::string& cidr, const std::string& ip) {
  uint32_t net = 0;
  int bits = 0;
  in_addr b{};
  if (!parse_cidr(cidr, net, bits) || ::inet_pton(AF_INET, ip.c_str(), &b) != 1) return false;  // malformed: no match
  if (bits == 0) return true;
  const uint32_t mask = bits >= 32 ? 0xFFFFFFFFu : ~((1u << (32 - bits)) - 1);
  return (net & mask) == (ntohl(b.s_addr) & mask);
}

NetpolDecision evaluate_netpol(const std::vector<Json>& policies, const std::string& pod_ns,
                               const std::map<std::string, std::string>& pod_labels, int port,
                               const std::string& port_name, const std::string& protocol, const NetpolSource& src) {
  NetpolDecision d;
  const Json labels = labels_json(pod_labels);
  for (const auto& np : policies) {
    if (np.str_at({"metadata", "namespace"}) != pod_ns || !policy_is_ingress(np)) continue;
    if (!LabelSelector::from_json(np.at_path({"spec", "podSelector"})).matches(labels)) continue;
    if (!d.isolated) d.policy = np.str_at({"metadata", "name"});
    d.isolated = true;
    for (const auto& rule : np.at_path({"spec", "ingress"}).as_array()) {
      if (!port_matches(rule["ports"], port, port_name, protocol)) continue;
      const Json& from = rule["from"];
      bool ok = !from.is_array() || from.empty();
      for (const auto& peer : from.as_array()) ok = ok || peer_matches(peer, pod_ns, src);
      if (ok) {
        d.allowed = true;
        d.policy = np.str_at({"metadata", "name"});
        d.reason = "allowed by NetworkPolicy " + pod_ns + "/" + d.policy;
        return d;
      }
    }
  }
  if (d.isolated) {
    d.allowed = false;
    d.reason = "denied by NetworkPolicy: no ingress rule of the policies selecting the pod allows " +
               (src.pod ? "namespace " + src.ns : std::string("source ") + (src.ip.empty() ? "?" : src.ip)) + " on port " +
               std::to_string(port);
  }
  return d;
}

}  // namespace kf
