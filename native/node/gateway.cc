// gateway.cc — Istio-ingress-equivalent HTTP gateway (see node.h).
#include <unistd.h>

#include <algorithm>
#include <cstdlib>

#include "core/util.h"
#include "node/node.h"

namespace kf {

Gateway::Gateway(std::shared_ptr<Client> c, std::string gateway_name)
    : c_(std::move(c)),
      gw_(std::move(gateway_name)),
      upgrades_(Registry::global().counter("gateway_upgraded_connections_total", "connections tunnelled after an HTTP Upgrade (WebSocket)")),
      streams_(Registry::global().counter("gateway_streamed_responses_total", "responses relayed incrementally (chunked / unframed / large)")) {
  const char* d = std::getenv("KFAMD_ROUTE_DOMAIN");
  route_domain_ = d && *d ? d : "apps.kube-lite";
}
Gateway::~Gateway() { stop(); }

void Gateway::setup(Manager& mgr) {
  vs_ = &mgr.informer("networking.istio.io/v1alpha3", "VirtualService");
  routes_ = &mgr.informer("route.openshift.io/v1", "Route");
}

bool Gateway::start(const std::string& addr, int port, std::string* err) {
  srv_ = std::make_unique<HttpServer>();
  if (!srv_->listen(addr, port, err)) return false;
  srv_->set_handler([this](HttpRequest& req, HttpResponse& resp) { handle(req, resp); });
  srv_->start();
  return true;
}

void Gateway::stop() {
  if (srv_) srv_->stop();
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
  Route rt;
  bool ok = vs_ && match(vs_->list(), gw_, host, req.path, rt);
  std::string target_path;
  if (ok) {
    std::string rest = req.path.size() >= rt.prefix.size() ? req.path.substr(rt.prefix.size()) : "";
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
      target_path = req.path;
      ok = true;
      break;
    }
  }
  if (!ok) {
    resp.text(404, "no route for " + host + req.path + "\n");
    return;
  }
  std::string url = "http://" + rt.dest_host + ":" + std::to_string(rt.dest_port) + target_path +
                    (req.raw_query.empty() ? "" : "?" + req.raw_query);
  const bool upgrade = contains(to_lower(req.header("Connection")), "upgrade") && !req.header("Upgrade").empty();
  Headers h;
  for (const auto& kv : req.headers) {
    std::string k = to_lower(kv.first);
    if (k == "content-length" || k == "transfer-encoding") continue;
    if (k == "connection" && !upgrade) continue;
    h[kv.first] = kv.second;
  }
  for (const auto& m : rt.headers.as_object()) h[m.first] = m.second.as_string();
  h["X-Forwarded-Prefix"] = rt.prefix;
  h["X-Envoy-Original-Path"] = req.path;
  const int timeout_ms = static_cast<int>(rt.timeout_s * 1000);
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
