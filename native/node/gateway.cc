// gateway.cc — Istio-ingress-equivalent HTTP gateway and policy enforcement point (see node.h).
#include <unistd.h>

#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>

#include <algorithm>
#include <cstdlib>

#include "core/util.h"
#include "node/authz.h"
#include "node/netpol.h"
#include "node/node.h"

namespace kf {

namespace {
constexpr const char* kPeerTokenHeader = "X-Kfamd-Peer-Token";
constexpr const char* kProxySecretHeader = "X-Kfamd-Auth-Proxy-Secret";
// the ingress / mesh listener's proof that it authorized a request, for the pods' inbound listeners
// (what the peer's mTLS identity of the ingress gateway is to an Istio sidecar): claims (method, path,
// destination namespace, expiry, the caller's principal / namespace / pod labels) + an HMAC-SHA256
// under a node secret. Bound to one request shape for 30 s, never taken from a client.
constexpr const char* kHopHeader = "X-Kfamd-Hop";
constexpr int64_t kHopTtlMs = 30000;
constexpr const char* kMeshPolicyName = "istio-mesh";

std::string hmac_hex(const std::string& key, const std::string& msg) {
  unsigned char md[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  HMAC(EVP_sha256(), key.data(), static_cast<int>(key.size()), reinterpret_cast<const unsigned char*>(msg.data()),
       msg.size(), md, &len);
  static const char* hex = "0123456789abcdef";
  std::string out;
  for (unsigned i = 0; i < len; ++i) {
    out += hex[md[i] >> 4];
    out += hex[md[i] & 15];
  }
  return out;
}

// "<svc>.<ns>.svc[.<domain>]" (or "<svc>.<ns>") -> (svc, ns); false for anything else
bool split_service_host(const std::string& host_port, std::string& svc, std::string& ns) {
  const std::string host = host_port.substr(0, host_port.find(':'));
  auto parts = split(host, '.', true);
  if (parts.size() < 2) return false;
  if (parts.size() > 2 && parts[2] != "svc") return false;
  svc = parts[0];
  ns = parts[1];
  return true;
}

std::string cookie_value(const std::string& cookies, const std::string& name) {
  for (const auto& c : split(cookies, ';', true)) {
    const std::string kv = trim(c);
    if (starts_with(kv, name + "=")) return kv.substr(name.size() + 1);
  }
  return "";
}
}  // namespace

Gateway::Gateway(std::shared_ptr<Client> c, GatewayOptions o)
    : c_(std::move(c)),
      o_(std::move(o)),
      upgrades_(Registry::global().counter("gateway_upgraded_connections_total", "connections tunnelled after an HTTP Upgrade (WebSocket)")),
      streams_(Registry::global().counter("gateway_streamed_responses_total", "responses relayed incrementally (chunked / unframed / large)")),
      decisions_(Registry::global().counter("gateway_authz_decisions_total",
                                            "AuthorizationPolicy decisions by listener and result", {"listener", "result"})) {
  const char* d = std::getenv("KFAMD_ROUTE_DOMAIN");
  route_domain_ = d && *d ? d : "apps.kube-lite";
  hop_secret_ = secure_random_hex(16);  // a credential: never guessable from the PRNG
}
Gateway::~Gateway() { stop(); }

void Gateway::setup(Manager& mgr) {
  vs_ = &mgr.informer("networking.istio.io/v1alpha3", "VirtualService");
  routes_ = &mgr.informer("route.openshift.io/v1", "Route");
  policies_ = &mgr.informer("security.istio.io/v1beta1", "AuthorizationPolicy");
  services_ = &mgr.informer("v1", "Service");
  netpols_ = &mgr.informer("networking.k8s.io/v1", "NetworkPolicy");
  namespaces_ = &mgr.informer("v1", "Namespace");
  mesh_np_ = std::make_shared<Controller>("istio-mesh-networkpolicy",
                                          [this](const Request& r, std::string* e) { return reconcile_mesh_policy(r, e); });
  mesh_np_->For(*namespaces_);
  mesh_np_->Watches(*netpols_, [](const std::string&, const Json& np) {
    std::vector<Request> out;
    if (np.str_at({"metadata", "name"}) == kMeshPolicyName) out.push_back({"", np.str_at({"metadata", "namespace"})});
    return out;
  });
  mgr.add(mesh_np_);
}

// OpenShift Service Mesh's member-namespace NetworkPolicy (Maistra's "istio-mesh"): every pod of a
// mesh-injected namespace accepts the mesh — other member namespaces, the ingress gateway's
// namespace and the control plane — so that a workload's own NetworkPolicies (ODH's <nb>-ctrl-np
// admits only the controller namespace on :8888) add to, and never cut off, mesh traffic. Policies
// are additive: a pod of an injected namespace is reachable from anything any policy allows.
Result Gateway::reconcile_mesh_policy(const Request& r, std::string* err) {
  Json n, live;
  const bool member = namespaces_->get("", r.name, n) && !n.at_path({"metadata", "deletionTimestamp"}).is_string() &&
                      n.at_path({"metadata", "labels", "istio-injection"}).as_string() == "enabled";
  const ApiError ge = c_->get("networking.k8s.io/v1", "NetworkPolicy", r.name, kMeshPolicyName, live);
  if (!member) {
    if (!ge && live.at_path({"metadata", "labels", "app.kubernetes.io/managed-by"}).as_string() == "kfamd-mesh")
      c_->remove("networking.k8s.io/v1", "NetworkPolicy", r.name, kMeshPolicyName);
    return {};
  }
  Json mesh_ns = Json::array({o_.ingress_namespace, o_.root_namespace, o_.control_plane_namespace, "kubeflow"});
  Json members = Json::object();
  members["namespaceSelector"] = Json{{"matchLabels", Json{{"istio-injection", "enabled"}}}};
  Json expr{{"key", "kubernetes.io/metadata.name"}, {"operator", "In"}, {"values", mesh_ns}};
  Json infra = Json::object();
  infra["namespaceSelector"] = Json{{"matchExpressions", Json::array({expr})}};
  Json rule = Json::object();
  rule["from"] = Json::array({members, infra});
  Json spec = Json::object();
  spec["podSelector"] = Json::object();
  spec["policyTypes"] = Json::array({"Ingress"});
  spec["ingress"] = Json::array({rule});
  if (!ge && live["spec"] == spec) return {};
  ApiError e;
  if (ge.code == 404) {
    Json np{{"apiVersion", "networking.k8s.io/v1"},
            {"kind", "NetworkPolicy"},
            {"metadata", Json{{"name", kMeshPolicyName}, {"namespace", r.name},
                              {"labels", Json{{"app.kubernetes.io/managed-by", "kfamd-mesh"}}}}},
            {"spec", spec}};
    e = c_->create(np);
  } else if (!ge) {
    live["spec"] = spec;
    e = c_->update(live);
  } else {
    e = ge;
  }
  if (e && e.code != 409) *err = e.message;
  return {};
}

// pods of `ns` have inbound listeners: every pod when pods get network namespaces, else the
// mesh-injected namespaces' (and NetworkPolicy-selected pods, which do not need the hop proof)
bool Gateway::dest_has_listener(const std::string& ns) {
  if (pods_have_listeners_) return true;
  Json n;
  return namespaces_ && namespaces_->get("", ns, n) && n.at_path({"metadata", "labels", "istio-injection"}).as_string() == "enabled";
}

bool Gateway::start(const std::string& addr, int port, std::string* err) {
  srv_ = std::make_unique<HttpServer>();
  if (!srv_->listen(addr, port, err)) return false;
  srv_->set_handler([this](HttpRequest& req, HttpResponse& resp) { handle(req, resp); });
  srv_->start();
  if (o_.mesh_port >= 0) {
    mesh_ = std::make_unique<HttpServer>();
    if (!mesh_->listen(addr, o_.mesh_port, err)) return false;
    mesh_->set_handler([this](HttpRequest& req, HttpResponse& resp) { handle_mesh(req, resp); });
    mesh_->start();
  }
  return true;
}

void Gateway::stop() {
  if (srv_) srv_->stop();
  if (mesh_) mesh_->stop();
}

Gateway::Identity Gateway::review_token(const std::string& token) {
  Identity id;
  if (token.empty()) return id;
  const double now = now_seconds();
  {
    std::lock_guard<std::mutex> g(tok_mu_);
    auto it = tok_cache_.find(token);
    if (it != tok_cache_.end() && it->second.second > now) return it->second.first;
  }
  Json tr{{"apiVersion", "authentication.k8s.io/v1"}, {"kind", "TokenReview"}, {"spec", Json{{"token", token}}}};
  const bool ok = !c_->create(tr);
  if (ok && tr.at_path({"status", "authenticated"}).as_bool()) {
    id.authenticated = true;
    id.username = tr.at_path({"status", "user", "username"}).as_string();
    for (const auto& g : tr.at_path({"status", "user", "groups"}).as_array()) id.groups.push_back(g.as_string());
  }
  std::lock_guard<std::mutex> g(tok_mu_);
  if (tok_cache_.size() > 4096) tok_cache_.clear();
  // an API server error is not cached: the next request asks again
  if (ok) tok_cache_[token] = {id, now + (id.authenticated ? 10.0 : 2.0)};
  return id;
}

bool Gateway::authorize(const std::string& dest_host, int dest_port, const HttpRequest& req, const std::string& path,
                        const Headers& fwd, const std::string& principal, const std::string& source_ns, std::string* why) {
  if (!o_.enforce || !policies_) return true;
  std::string svc, ns;
  if (!split_service_host(dest_host, svc, ns)) {
    if (why) *why = "destination " + dest_host + " is not a Service";
    return false;
  }
  std::map<std::string, std::string> labels;  // the workload's labels: the Service's selector
  Json s;
  if (services_ && services_->get(ns, svc, s))
    for (const auto& kv : s.at_path({"spec", "selector"}).as_object()) labels[kv.first] = kv.second.as_string();
  return authorize_workload(ns, labels, dest_port, req, path, fwd, principal, source_ns, why);
}

bool Gateway::authorize_workload(const std::string& ns, const std::map<std::string, std::string>& labels, int dest_port,
                                 const HttpRequest& req, const std::string& path, const Headers& fwd,
                                 const std::string& principal, const std::string& source_ns, std::string* why) {
  if (!o_.enforce || !policies_) return true;
  // fail closed: until both informers have listed, "no ALLOW policy applies" would
  // admit everything
  if (!policies_->synced() || (services_ && !services_->synced())) {
    if (why) *why = "authorization policies not synced yet";
    return false;
  }
  AuthzRequest ar;
  ar.principal = principal;
  ar.source_namespace = source_ns;
  ar.remote_ip = req.remote_addr.substr(0, req.remote_addr.rfind(':'));
  ar.source_ip = ar.remote_ip;
  ar.method = req.method;
  ar.path = path;
  ar.host = req.header("Host");
  ar.port = dest_port;
  for (const auto& kv : fwd) ar.headers[to_lower(kv.first)] = kv.second;
  AuthzDecision d = evaluate_authz(policies_->list(), ar, ns, labels, o_.root_namespace);
  if (!d.allowed && why) *why = d.reason + (d.policy.empty() ? "" : " (" + d.policy + ")");
  return d.allowed;
}

// the caller's workload identity (Istio: the peer's mTLS certificate; here its ServiceAccount
// token); a caller without one is plaintext: no principal, no source namespace
void Gateway::peer_identity(const HttpRequest& req, std::string& principal, std::string& source_ns) {
  Identity peer = review_token(req.header(kPeerTokenHeader));
  if (peer.authenticated && peer.service_account()) {
    auto parts = split(peer.username, ':', false);  // system:serviceaccount:<ns>:<name>
    if (parts.size() == 4) {
      source_ns = parts[2];
      principal = o_.cluster_domain + "/ns/" + parts[2] + "/sa/" + parts[3];
    }
  }
}

std::string Gateway::stamp_hop(const std::string& method, const std::string& path, const std::string& dest_ns,
                               const HopClaims& who) const {
  Json labels = Json::object();
  for (const auto& kv : who.source_labels) labels[kv.first] = kv.second;
  const Json claims{{"m", method}, {"p", path}, {"ns", dest_ns}, {"exp", now_unix_ms() + kHopTtlMs},
                    {"pr", who.principal}, {"sns", who.source_ns}, {"spod", who.source_pod}, {"sl", labels}};
  const std::string payload = base64_encode(claims.dump());
  return payload + "." + hmac_hex(hop_secret_, payload);
}

bool Gateway::verify_hop(const std::string& value, const std::string& method, const std::string& path,
                         const std::string& dest_ns, HopClaims& out) const {
  const size_t dot = value.rfind('.');
  if (value.empty() || dot == std::string::npos) return false;
  const std::string payload = value.substr(0, dot), mac = value.substr(dot + 1), want = hmac_hex(hop_secret_, payload);
  if (mac.size() != want.size() || CRYPTO_memcmp(mac.data(), want.data(), want.size()) != 0) return false;
  Json c;
  if (!Json::try_parse(base64_decode(payload), c)) return false;
  const int64_t now = now_unix_ms(), exp = c["exp"].as_int();
  if (c["m"].as_string() != method || c["p"].as_string() != path || c["ns"].as_string() != dest_ns || exp < now ||
      exp > now + kHopTtlMs)
    return false;
  out.principal = c["pr"].as_string();
  out.source_ns = c["sns"].as_string();
  out.source_pod = c["spod"].as_bool();
  for (const auto& kv : c["sl"].as_object()) out.source_labels[kv.first] = kv.second.as_string();
  return true;
}

// the source of a request the mesh listener received: the pod behind an egress relay (netns mode:
// its namespace + labels), else the ServiceAccount token's namespace
Gateway::HopClaims Gateway::mesh_caller(const HttpRequest& req) {
  HopClaims who;
  peer_identity(req, who.principal, who.source_ns);
  PodSource ps;
  if (lookup_pod_source(req.remote_addr, ps)) {
    who.source_pod = true;
    who.source_labels = ps.labels;
    if (who.source_ns.empty() || who.source_ns != ps.ns) who.principal.clear();  // a token of another namespace proves nothing
    who.source_ns = ps.ns;
  } else {
    who.source_pod = !who.source_ns.empty();
  }
  return who;
}

std::map<std::string, std::string> Gateway::namespace_labels(const std::string& ns) {
  std::map<std::string, std::string> out;
  Json n;
  if (namespaces_ && namespaces_->get("", ns, n))
    for (const auto& kv : n.at_path({"metadata", "labels"}).as_object()) out[kv.first] = kv.second.as_string();
  if (out.empty()) out["kubernetes.io/metadata.name"] = ns;
  return out;
}

// A pod's inbound listener: NetworkPolicy for every pod that has one, Istio AuthorizationPolicy on
// the pod's own labels for mesh-injected pods (the gateway decided on the Service
// selector; re-evaluated here with the principal it carried), then the app.
void Gateway::handle_inbound(const InboundTarget& t, HttpRequest& req, HttpResponse& resp) {
  if (path_has_escaped_slash(req.target.substr(0, req.target.find('?')))) {
    resp.text(400, "Bad Request: escaped slashes are not allowed in the path\n");
    return;
  }
  const std::string path = normalize_authz_path(req.path);
  HopClaims who;
  const bool hopped = verify_hop(req.header(kHopHeader), req.method, path, t.ns, who);
  Headers h;
  for (const auto& kv : req.headers) {
    const std::string k = to_lower(kv.first);
    if (k == "content-length" || k == "transfer-encoding" || k == "connection") continue;
    if (k == to_lower(kPeerTokenHeader) || k == to_lower(kHopHeader)) continue;
    h[kv.first] = kv.second;
  }
  if (!hopped) {
    // dialed directly: the pod network (netns mode) lets only node processes reach this address, so
    // an unattributed caller is the control plane; a ServiceAccount token names its namespace
    peer_identity(req, who.principal, who.source_ns);
    who.source_pod = true;
    if (who.source_ns.empty()) who.source_ns = o_.control_plane_namespace;
  }
  if (netpols_) {
    NetpolSource src;
    src.pod = who.source_pod;
    src.ns = who.source_ns;
    src.pod_labels = who.source_labels;
    src.ns_labels = namespace_labels(who.source_ns);
    src.ip = req.remote_addr.substr(0, req.remote_addr.rfind(':'));
    const NetpolDecision d = evaluate_netpol(netpols_->list(t.ns), t.ns, t.labels, t.port, t.port_name, "TCP", src);
    if (d.isolated) decisions_->inc({"netpol", d.allowed ? "allow" : "deny"});
    if (!d.allowed) {
      resp.headers["X-Kfamd-Netpol"] = d.reason + " (" + d.policy + ")";
      resp.text(403, "NetworkPolicy: connection refused");
      return;
    }
  }
  if (t.mesh && o_.enforce) {
    std::string why;
    const std::string principal = hopped || !who.principal.empty() ? who.principal : "";
    if (!authorize_workload(t.ns, t.labels, t.port, req, path, h, principal, hopped || !principal.empty() ? who.source_ns : "", &why)) {
      decisions_->inc({"sidecar", "deny"});
      resp.headers["X-Kfamd-Authz"] = why;
      resp.text(403, "RBAC: access denied");
      return;
    }
    decisions_->inc({"sidecar", "allow"});
  }
  const std::string url = "http://" + t.app_ip + ":" + std::to_string(t.port) + encode_request_path(path) +
                          (req.raw_query.empty() ? "" : "?" + req.raw_query);
  NetnsScope in(t.netns.get());  // the connection to the app is made inside the pod's namespace
  if (!in.ok()) {
    resp.text(503, "upstream connect error: cannot enter the pod's network namespace\n");
    return;
  }
  forward(req, resp, url, std::move(h), 300000);
}

bool Gateway::match(const std::vector<Json>& vss, const std::string& gateway, const std::string& host,
                    const std::string& path, Route& out) {
  size_t best_len = 0;
  bool found = false;
  for (const auto& vs : vss) {
    const Json& spec = vs["spec"];
    bool gw_ok = spec["gateways"].empty();
    for (const auto& g : spec["gateways"].as_array()) {
      const std::string& gs = g.as_string();
      // "ns/name" or bare "name" (same namespace as the VS)
      gw_ok = gw_ok || gs == gateway || gs == "mesh" ||
              (gs.find('/') == std::string::npos && vs.str_at({"metadata", "namespace"}) + "/" + gs == gateway);
    }
    if (!gw_ok) continue;
    bool host_ok = spec["hosts"].empty();
    for (const auto& h : spec["hosts"].as_array()) {
      const std::string& hs = h.as_string();
      std::string hostname = host.substr(0, host.find(':'));
      host_ok = host_ok || hs == "*" || hs == hostname || (starts_with(hs, "*.") && ends_with(hostname, hs.substr(1)));
    }
    if (!host_ok) continue;
    for (const auto& http : spec["http"].as_array()) {
      const Json& matches = http["match"];
      std::vector<std::pair<std::string, bool>> prefixes;  // (value, exact)
      if (!matches.is_array() || matches.empty()) prefixes.push_back({"/", false});
      for (const auto& m : matches.as_array()) {
        if (m.at_path({"uri", "prefix"}).is_string()) prefixes.push_back({m.at_path({"uri", "prefix"}).as_string(), false});
        else if (m.at_path({"uri", "exact"}).is_string()) prefixes.push_back({m.at_path({"uri", "exact"}).as_string(), true});
      }
      for (const auto& p : prefixes) {
        bool hit = p.second ? path == p.first : starts_with(path, p.first);
        // "/notebook/ns/nb/" also serves "/notebook/ns/nb" (Istio redirects; we match leniently)
        if (!hit && !p.second && ends_with(p.first, "/") && path == p.first.substr(0, p.first.size() - 1)) hit = true;
        if (!hit || p.first.size() < best_len) continue;
        const Json& route = http["route"][0];
        if (!route.is_object()) continue;
        best_len = p.first.size();
        found = true;
        out = Route();
        out.prefix = p.first;
        out.exact = p.second;
        out.rewrite = http.at_path({"rewrite", "uri"}).as_string_or(p.first);
        out.dest_host = route.at_path({"destination", "host"}).as_string();
        out.dest_port = static_cast<int>(route.at_path({"destination", "port", "number"}).as_int(80));
        out.headers = http.at_path({"headers", "request", "set"});
        std::string to = http["timeout"].as_string();
        if (!to.empty()) out.timeout_s = std::atof(to.c_str());
        if (out.dest_host.find('.') == std::string::npos)  // short name -> same namespace
          out.dest_host += "." + vs.str_at({"metadata", "namespace"}) + ".svc";
      }
    }
  }
  return found;
}

void Gateway::handle(HttpRequest& req, HttpResponse& resp) {
  const std::string host = req.header("Host");
  if (path_has_escaped_slash(req.target.substr(0, req.target.find('?')))) {
    resp.text(400, "Bad Request: escaped slashes are not allowed in the path\n");
    return;
  }
  // routing, authorization and the upstream request all see one normalized path (Istio BASE)
  const std::string path = normalize_authz_path(req.path);
  Route rt;
  bool ok = vs_ && match(vs_->list(), o_.gateway_name, host, path, rt);
  bool routed_by_route = false;  // OpenShift Routes bypass the mesh (the ODH OAuth proxy guards them)
  std::string target_path;
  if (ok) {
    std::string rest = path.size() >= rt.prefix.size() ? path.substr(rt.prefix.size()) : "";
    target_path = rt.rewrite + rest;
    if (target_path.empty()) target_path = "/";
  } else if (routes_) {
    // OpenShift Route (host based)
    for (const auto& r : routes_->list()) {
      std::string rhost = r.at_path({"spec", "host"}).as_string();
      if (rhost.empty()) rhost = r.str_at({"metadata", "name"}) + "-" + r.str_at({"metadata", "namespace"}) + "." + route_domain_;
      if (rhost != host.substr(0, host.find(':'))) continue;
      const std::string svc = r.at_path({"spec", "to", "name"}).as_string();
      rt.dest_host = svc + "." + r.str_at({"metadata", "namespace"}) + ".svc";
      const Json& tp = r.at_path({"spec", "port", "targetPort"});
      rt.dest_port = tp.is_number() ? static_cast<int>(tp.as_int()) : 80;
      if (tp.is_string()) {
        Json s;
        if (!c_->get("v1", "Service", r.str_at({"metadata", "namespace"}), svc, s))
          for (const auto& p : s.at_path({"spec", "ports"}).as_array())
            if (p["name"].as_string() == tp.as_string() || p["targetPort"] == tp) rt.dest_port = static_cast<int>(p["port"].as_int());
      }
      target_path = path;
      ok = routed_by_route = true;
      break;
    }
  }
  if (!ok) {
    resp.text(404, "no route for " + host + path + "\n");
    return;
  }
  std::string url = "http://" + rt.dest_host + ":" + std::to_string(rt.dest_port) + encode_request_path(target_path) +
                    (req.raw_query.empty() ? "" : "?" + req.raw_query);
  // authentication: a trusted authn proxy's assertion, else a bearer token / session cookie
  // (TokenReview); client-supplied identity headers never pass otherwise
  const std::string uid_lc = to_lower(o_.userid_header);
  const bool trusted_proxy = !o_.trusted_proxy_secret.empty() && req.header(kProxySecretHeader) == o_.trusted_proxy_secret;
  Identity who;
  if (!trusted_proxy) {
    const std::string auth = req.header("Authorization");
    std::string token = starts_with(auth, "Bearer ") ? trim(auth.substr(7)) : "";
    if (token.empty()) token = cookie_value(req.header("Cookie"), o_.auth_cookie);
    who = review_token(token);
  }
  Headers h;
  for (const auto& kv : req.headers) {
    std::string k = to_lower(kv.first);
    if (k == "content-length" || k == "transfer-encoding" || k == "connection") continue;
    if (k == to_lower(kPeerTokenHeader) || k == to_lower(kProxySecretHeader) || k == to_lower(kHopHeader)) continue;
    if (!trusted_proxy && (k == uid_lc || k == "kubeflow-groups")) continue;  // spoofed identity
    h[kv.first] = kv.second;
  }
  if (who.authenticated && !who.service_account()) h[o_.userid_header] = o_.userid_prefix + who.username;
  for (const auto& m : rt.headers.as_object()) h[m.first] = m.second.as_string();
  h["X-Forwarded-Prefix"] = rt.prefix;
  h["X-Envoy-Original-Path"] = path;
  // authorization at the destination workload (what its Istio sidecar does in the reference): the
  // request arrives from the ingress gateway's principal, with the path after the rewrite
  std::string why;
  if (!routed_by_route && !authorize(rt.dest_host, rt.dest_port, req, target_path, h, o_.ingress_principal,
                                     o_.ingress_namespace, &why)) {
    decisions_->inc({"ingress", "deny"});
    resp.headers["X-Kfamd-Authz"] = why;
    resp.text(403, "RBAC: access denied");
    return;
  }
  if (!routed_by_route && o_.enforce) {
    decisions_->inc({"ingress", "allow"});
    // the destination pod's inbound listener takes this decision (when it has one: a pod without one
    // must not even see the proof)
    std::string svc, dns;
    if (split_service_host(rt.dest_host, svc, dns) && dest_has_listener(dns)) {
      HopClaims who;
      who.principal = o_.ingress_principal;
      who.source_ns = o_.ingress_namespace;
      who.source_pod = true;
      who.source_labels = {{"istio", "ingressgateway"}};
      h[kHopHeader] = stamp_hop(req.method, normalize_authz_path(target_path), dns, who);
    }
  }
  forward(req, resp, url, std::move(h), static_cast<int>(rt.timeout_s * 1000));
}

void Gateway::handle_mesh(HttpRequest& req, HttpResponse& resp) {
  std::string svc, ns;
  const std::string host = req.header("Host");
  if (!split_service_host(host, svc, ns)) {
    resp.text(404, "mesh: Host must name a Service (<svc>.<ns>.svc[.<domain>]), got " + host + "\n");
    return;
  }
  if (path_has_escaped_slash(req.target.substr(0, req.target.find('?')))) {
    resp.text(400, "Bad Request: escaped slashes are not allowed in the path\n");
    return;
  }
  const HopClaims who = mesh_caller(req);
  const std::string principal = who.principal, source_ns = who.source_ns;
  Headers h;
  for (const auto& kv : req.headers) {
    std::string k = to_lower(kv.first);
    if (k == "content-length" || k == "transfer-encoding" || k == "connection") continue;
    if (k == to_lower(kPeerTokenHeader) || k == to_lower(kHopHeader)) continue;
    h[kv.first] = kv.second;
  }
  const size_t colon = host.find(':');
  const int port = colon == std::string::npos ? 80 : std::atoi(host.c_str() + colon + 1);
  std::string why;
  const std::string path = normalize_authz_path(req.path);
  if (!authorize(host.substr(0, colon), port, req, path, h, principal, source_ns, &why)) {
    decisions_->inc({"mesh", "deny"});
    resp.headers["X-Kfamd-Authz"] = why;
    resp.text(403, "RBAC: access denied");
    return;
  }
  if (o_.enforce) {
    decisions_->inc({"mesh", "allow"});
    if (dest_has_listener(ns)) h[kHopHeader] = stamp_hop(req.method, path, ns, who);
  }
  const std::string url = "http://" + svc + "." + ns + ".svc." + o_.cluster_domain + ":" + std::to_string(port) +
                          encode_request_path(path) +
                          (req.raw_query.empty() ? "" : "?" + req.raw_query);
  forward(req, resp, url, std::move(h), 300000);
}

void Gateway::forward(HttpRequest& req, HttpResponse& resp, const std::string& url, Headers h, int timeout_ms) {
  const bool upgrade = contains(to_lower(req.header("Connection")), "upgrade") && !req.header("Upgrade").empty();
  if (upgrade) h["Connection"] = req.header("Connection");
  // Istio's default retry policy: 2 retries on connect-failure / refused-stream (a pod that is
  // Ready without a readiness probe may not be listening yet)
  auto with_retries = [](auto attempt) {
    auto r = attempt();
    for (int i = 0; i < 2 && !r; ++i) {
      ::usleep(25000);
      r = attempt();
    }
    return r;
  };
  std::string err;
  if (upgrade) {
    // WebSocket (JupyterLab kernel channels, terminals): forward the handshake, then the
    // connection is a byte tunnel until either side closes
    auto up = with_retries([&] { return http_dial(url, timeout_ms, &err); });
    if (!up) {
      resp.text(503, "upstream connect error or disconnect/reset before headers. reset reason: " + err + "\n");
      return;
    }
    Url u;
    Url::parse(url, u);
    std::string head = req.method + " " + u.target() + " HTTP/1.1\r\n";
    if (!h.count("Host")) head += "Host: " + u.host + ":" + std::to_string(u.port) + "\r\n";
    for (const auto& kv : h) head += kv.first + ": " + kv.second + "\r\n";
    if (!req.body.empty()) head += "Content-Length: " + std::to_string(req.body.size()) + "\r\n";
    head += "\r\n" + req.body;
    if (!up->write(head)) {
      resp.text(503, "upstream reset before the upgrade\n");
      return;
    }
    std::shared_ptr<RawConn> upstream(std::move(up));
    upgrades_->inc();
    resp.upgrade = [upstream](RawConn& client, const std::string& pending) {
      pump_bidirectional(client, *upstream, pending, "");
    };
    return;
  }
  auto r = with_retries([&] { return http_open(req.method, url, req.body, h, timeout_ms, &err); });
  if (!r) {
    resp.text(503, "upstream connect error or disconnect/reset before headers. reset reason: " + err + "\n");
    return;
  }
  resp.status = r->status;
  for (const auto& kv : r->headers) {
    std::string k = to_lower(kv.first);
    if (k == "content-length" || k == "transfer-encoding" || k == "connection") continue;
    resp.headers[kv.first] = kv.second;
  }
  if (!r->chunked && r->length >= 0 && r->length <= (4 << 20)) {
    resp.body = r->read_all();  // small, framed body: buffered (keeps the client connection alive)
    return;
  }
  // chunked / EOF-delimited / large bodies (log follow, watch, server-sent events, downloads)
  // are relayed piece by piece as they arrive
  std::shared_ptr<HttpClientResponse> body(std::move(r));
  streams_->inc();
  resp.stream = [body](StreamWriter& w) {
    std::string piece;
    for (;;) {
      const auto n = body->next(piece);
      if (n == HttpClientResponse::kTimeout) {
        if (!w.alive()) return;
        continue;
      }
      if (n != HttpClientResponse::kData || !w.write(piece)) return;
    }
  };
}

}  // namespace kf
