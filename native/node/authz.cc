// authz.cc — see authz.h.
#include "node/authz.h"

#include <arpa/inet.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>

#include "core/util.h"
#include "node/netpol.h"

namespace kf {

bool istio_string_match(const std::string& pattern, const std::string& value) {
  if (pattern == "*") return !value.empty();
  if (pattern.size() > 1 && pattern.back() == '*') return starts_with(value, pattern.substr(0, pattern.size() - 1));
  if (pattern.size() > 1 && pattern.front() == '*') return ends_with(value, pattern.substr(1));
  return pattern == value;
}

// one parser with the NetworkPolicy ipBlocks (netpol.cc): a malformed prefix matches nothing
bool ipv4_in_cidr(const std::string& ip, const std::string& cidr) { return cidr_contains(cidr, ip); }

std::string normalize_authz_path(const std::string& decoded_path) {
  std::string p = decoded_path;
  std::replace(p.begin(), p.end(), '\\', '/');
  if (p.empty() || p[0] != '/') p.insert(p.begin(), '/');
  std::vector<std::string> out;
  size_t i = 1;
  bool trailing = false;  // the path ends in '/' (or in a dot segment, which names a directory)
  while (i <= p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    const std::string seg = p.substr(i, j - i);
    const bool last = j == p.size();
    if (seg == "..") {
      if (!out.empty()) out.pop_back();
      trailing = last;
    } else if (seg == ".") {
      trailing = last;
    } else {
      out.push_back(seg);
      trailing = false;
    }
    i = j + 1;
  }
  std::string r;
  for (const auto& seg : out) r += "/" + seg;
  if (r.empty() || trailing) r += "/";
  return r;
}

std::string encode_request_path(const std::string& path) {
  static const char* hex = "0123456789ABCDEF";
  std::string r;
  r.reserve(path.size());
  for (unsigned char ch : path) {
    const bool keep = std::isalnum(ch) || std::strchr("-._~!$&'()*+,;=:@/", ch) != nullptr;
    if (keep && ch != 0) {
      r.push_back(static_cast<char>(ch));
    } else {
      r.push_back('%');
      r.push_back(hex[ch >> 4]);
      r.push_back(hex[ch & 15]);
    }
  }
  return r;
}

namespace {

bool any_match(const Json& patterns, const std::string& v, bool ci = false) {
  const std::string val = ci ? to_lower(v) : v;
  for (const auto& p : patterns.as_array())
    if (istio_string_match(ci ? to_lower(p.as_string()) : p.as_string(), val)) return true;
  return false;
}

bool any_cidr(const Json& blocks, const std::string& ip) {
  for (const auto& b : blocks.as_array())
    if (ipv4_in_cidr(ip, b.as_string())) return true;
  return false;
}

// one field pair (positive list must match if present, negative list must not match)
bool field_ok(const Json& obj, const char* pos, const char* neg, const std::string& v, bool ci = false) {
  if (obj[pos].is_array() && !obj[pos].empty() && !any_match(obj[pos], v, ci)) return false;
  if (obj[neg].is_array() && !obj[neg].empty() && any_match(obj[neg], v, ci)) return false;
  return true;
}

bool source_matches(const Json& src, const AuthzRequest& r) {
  if (!field_ok(src, "principals", "notPrincipals", r.principal)) return false;
  if (!field_ok(src, "requestPrincipals", "notRequestPrincipals", r.request_principal)) return false;
  if (!field_ok(src, "namespaces", "notNamespaces", r.source_namespace)) return false;
  if (src["ipBlocks"].is_array() && !src["ipBlocks"].empty() && !any_cidr(src["ipBlocks"], r.source_ip)) return false;
  if (src["notIpBlocks"].is_array() && any_cidr(src["notIpBlocks"], r.source_ip)) return false;
  if (src["remoteIpBlocks"].is_array() && !src["remoteIpBlocks"].empty() && !any_cidr(src["remoteIpBlocks"], r.remote_ip))
    return false;
  if (src["notRemoteIpBlocks"].is_array() && any_cidr(src["notRemoteIpBlocks"], r.remote_ip)) return false;
  return true;
}

bool operation_matches(const Json& op, const AuthzRequest& r) {
  const std::string host = r.host.substr(0, r.host.find(':'));
  if (!field_ok(op, "hosts", "notHosts", host, true)) return false;
  if (!field_ok(op, "ports", "notPorts", std::to_string(r.port))) return false;
  if (!field_ok(op, "methods", "notMethods", r.method)) return false;
  // r.path is the normalized path alone (the query was split off before decoding)
  if (!field_ok(op, "paths", "notPaths", r.path)) return false;
  return true;
}

// the value a condition key names; false when the key is unknown (the condition never holds)
bool condition_value(const std::string& key, const AuthzRequest& r, std::string& out) {
  if (starts_with(key, "request.headers[") && ends_with(key, "]")) {
    auto it = r.headers.find(to_lower(key.substr(16, key.size() - 17)));
    out = it == r.headers.end() ? "" : it->second;
    return true;
  }
  if (key == "source.namespace") out = r.source_namespace;
  else if (key == "source.principal") out = r.principal;
  else if (key == "source.ip") out = r.source_ip;
  else if (key == "remote.ip") out = r.remote_ip;
  else if (key == "request.auth.principal") out = r.request_principal;
  else if (key == "destination.port") out = std::to_string(r.port);
  else return false;
  return true;
}

bool condition_holds(const Json& c, const AuthzRequest& r) {
  const std::string key = c["key"].as_string();
  std::string v;
  if (!condition_value(key, r, v)) return false;
  const bool ip = key == "source.ip" || key == "remote.ip";
  auto matches = [&](const Json& list) {
    for (const auto& p : list.as_array())
      if (ip ? ipv4_in_cidr(v, p.as_string()) : istio_string_match(p.as_string(), v)) return true;
    return false;
  };
  if (c["values"].is_array() && !c["values"].empty() && !matches(c["values"])) return false;
  if (c["notValues"].is_array() && !c["notValues"].empty() && matches(c["notValues"])) return false;
  return true;
}

bool rule_matches(const Json& rule, const AuthzRequest& r) {
  if (rule["from"].is_array() && !rule["from"].empty()) {
    bool any = false;
    for (const auto& f : rule["from"].as_array()) any = any || source_matches(f["source"], r);
    if (!any) return false;
  }
  if (rule["to"].is_array() && !rule["to"].empty()) {
    bool any = false;
    for (const auto& t : rule["to"].as_array()) any = any || operation_matches(t["operation"], r);
    if (!any) return false;
  }
  for (const auto& c : rule["when"].as_array())
    if (!condition_holds(c, r)) return false;
  return true;
}

bool selector_matches(const Json& spec, const std::map<std::string, std::string>& labels) {
  const Json& ml = spec.at_path({"selector", "matchLabels"});
  for (const auto& kv : ml.as_object()) {
    auto it = labels.find(kv.first);
    if (it == labels.end() || it->second != kv.second.as_string()) return false;
  }
  return true;
}

}  // namespace

AuthzDecision evaluate_authz(const std::vector<Json>& policies, const AuthzRequest& r, const std::string& workload_ns,
                             const std::map<std::string, std::string>& workload_labels, const std::string& root_namespace) {
  std::vector<const Json*> allow, deny;
  for (const auto& p : policies) {
    const std::string ns = p.str_at({"metadata", "namespace"});
    if (ns != workload_ns && ns != root_namespace) continue;
    const Json& spec = p["spec"];
    if (!selector_matches(spec, workload_labels)) continue;
    const std::string action = spec["action"].as_string_or("ALLOW");
    if (action == "DENY") deny.push_back(&p);
    else if (action == "ALLOW") allow.push_back(&p);  // CUSTOM / AUDIT: not enforced here
  }
  auto id = [](const Json& p) { return p.str_at({"metadata", "namespace"}) + "/" + p.str_at({"metadata", "name"}); };
  for (const Json* p : deny)
    for (const auto& rule : (*p)["spec"]["rules"].as_array())
      if (rule_matches(rule, r)) return {false, id(*p), "matched a DENY rule"};
  if (allow.empty()) return {true, "", "no ALLOW policy applies"};
  for (const Json* p : allow)
    for (const auto& rule : (*p)["spec"]["rules"].as_array())
      if (rule_matches(rule, r)) return {true, id(*p), "matched an ALLOW rule"};
  return {false, "", "no ALLOW rule matched"};
}

}  // namespace kf
