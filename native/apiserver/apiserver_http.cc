// apiserver_http.cc — Kubernetes REST conventions over kube-lite:
//   /api/v1/[namespaces/{ns}/]{plural}[/{name}[/{subresource}]]
//   /apis/{group}/{version}/[namespaces/{ns}/]{plural}[/{name}[/{subresource}]]
// GET (get / list / ?watch=1), POST, PUT, PATCH (merge, json-patch, strategic-merge, apply),
// DELETE (single + collection), discovery (/api, /apis, /apis/{g}/{v}), /version, /healthz,
// /readyz, /livez, /metrics, pod logs, the services/{name}:{port}/proxy subresource (used by the
// culler in DEV mode like `kubectl proxy`), and /debug/faults for fault injection.
#include <atomic>
#include <algorithm>
#include <chrono>

#include "apiserver/apiserver.h"
#include "core/metrics.h"
#include "core/util.h"

namespace kf {

namespace {
void send_error(HttpResponse& resp, const ApiError& e, const std::string& kind = "", const std::string& name = "") {
  resp.json(e.code ? e.code : 500, e.status_json(kind, name).dump());
}
std::string verb_for(const std::string& method, bool has_name, bool watch) {
  if (method == "GET") return watch ? "watch" : (has_name ? "get" : "list");
  if (method == "POST") return "create";
  if (method == "PUT") return "update";
  if (method == "PATCH") return "patch";
  if (method == "DELETE") return has_name ? "delete" : "deletecollection";
  return to_lower(method);
}
}  // namespace

void ApiServer::http_discovery(HttpRequest& req, HttpResponse& resp, const std::vector<std::string>& segs) {
  auto all = reg_.all();
  if (segs.size() == 1 && segs[0] == "api") {
    resp.json(200, Json{{"kind", "APIVersions"}, {"versions", Json::array({"v1"})},
                        {"serverAddressByClientCIDRs", Json::array()}}.dump());
    return;
  }
  if (segs.size() == 1 && segs[0] == "apis") {
    std::map<std::string, std::pair<std::vector<std::string>, std::string>> groups;
    for (const auto& r : all) {
      if (r->group.empty()) continue;
      auto& g = groups[r->group];
      for (const auto& v : r->versions)
        if (std::find(g.first.begin(), g.first.end(), v) == g.first.end()) g.first.push_back(v);
      g.second = r->storage_version;
    }
    Json list = Json::array();
    for (const auto& kv : groups) {
      Json vs = Json::array();
      for (const auto& v : kv.second.first) vs.push_back(Json{{"groupVersion", kv.first + "/" + v}, {"version", v}});
      list.push_back(Json{{"name", kv.first}, {"versions", vs},
                          {"preferredVersion", Json{{"groupVersion", kv.first + "/" + kv.second.second}, {"version", kv.second.second}}}});
    }
    resp.json(200, Json{{"kind", "APIGroupList"}, {"apiVersion", "v1"}, {"groups", list}}.dump());
    return;
  }
  std::string group = segs[0] == "api" ? "" : segs[1];
  std::string version = segs[0] == "api" ? segs[1] : segs[2];
  Json rs = Json::array();
  for (const auto& r : all) {
    if (r->group != group || !r->serves(version)) continue;
    Json verbs = r->virtual_only ? Json::array({"create"})
                                 : Json::array({"create", "delete", "deletecollection", "get", "list", "patch", "update", "watch"});
    Json e{{"name", r->plural}, {"singularName", r->singular}, {"namespaced", r->namespaced}, {"kind", r->kind}, {"verbs", verbs}};
    if (!r->short_names.empty()) {
      Json sn = Json::array();
      for (auto& s : r->short_names) sn.push_back(s);
      e["shortNames"] = sn;
    }
    rs.push_back(e);
    if (r->has_status)
      rs.push_back(Json{{"name", r->plural + "/status"}, {"singularName", ""}, {"namespaced", r->namespaced},
                        {"kind", r->kind}, {"verbs", Json::array({"get", "patch", "update"})}});
  }
  (void)req;
  resp.json(200, Json{{"kind", "APIResourceList"}, {"apiVersion", "v1"},
                      {"groupVersion", group.empty() ? version : group + "/" + version}, {"resources", rs}}.dump());
}

void ApiServer::http_watch(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                           const ListOptions& lo, HttpResponse& resp) {
  ApiError err;
  WatchPtr w = r_watch(res, version, ns, lo, &err);
  if (!w) {
    if (err.code == 410) {
      // watch error event, like kube-apiserver does for expired resourceVersions
      resp.status = 200;
      resp.headers["Content-Type"] = "application/json";
      Json ev{{"type", "ERROR"}, {"object", err.status_json()}};
      std::string line = ev.dump() + "\n";
      resp.stream = [line](StreamWriter& sw) { sw.write(line); };
      return;
    }
    send_error(resp, err);
    return;
  }
  resp.status = 200;
  resp.headers["Content-Type"] = "application/json";
  int timeout = lo.timeout_seconds > 0 ? lo.timeout_seconds : 1800;
  bool bookmarks = lo.allow_bookmarks;
  auto self = this;
  resp.stream = [w, timeout, bookmarks, self, res, version](StreamWriter& sw) {
    double deadline = now_seconds() + timeout;
    double last_bookmark = now_seconds();
    while (self->running_ || true) {
      if (now_seconds() > deadline) break;
      WatchEvent ev;
      if (w->next(ev, 500)) {
        Json line{{"type", ev.type}, {"object", ev.object}};
        if (!sw.write(line.dump() + "\n")) break;
        continue;
      }
      if (w->closed()) break;
      if (!sw.alive()) break;
      if (bookmarks && now_seconds() - last_bookmark > 10) {
        last_bookmark = now_seconds();
        Json bm{{"type", "BOOKMARK"},
                {"object", Json{{"apiVersion", res->api_version(version.empty() ? res->storage_version : version)},
                                {"kind", res->kind},
                                {"metadata", Json{{"resourceVersion", std::to_string(self->current_rv())}}}}}};
        if (!sw.write(bm.dump() + "\n")) break;
      }
    }
    w->stop();
  };
}

void ApiServer::http_proxy(HttpRequest& req, HttpResponse& resp, const std::string& ns, const std::string& svc_port,
                           const std::string& rest) {
  std::string svc = svc_port, port_name;
  size_t c = svc_port.find(':');
  if (c != std::string::npos) {
    svc = svc_port.substr(0, c);
    port_name = svc_port.substr(c + 1);
  }
  Json s;
  if (ApiError e = r_get(reg_.by_plural("", "services"), "", ns, svc, s)) {
    send_error(resp, e);
    return;
  }
  int port = 0;
  for (const auto& p : s.at_path({"spec", "ports"}).as_array())
    if (port_name.empty() || p["name"].as_string() == port_name || std::to_string(p["port"].as_int()) == port_name)
      port = static_cast<int>(p["port"].as_int());
  std::string ip;
  int tport = 0;
  if (!port || !resolve_service(svc + "." + ns + ".svc", port, ip, tport)) {
    resp.json(503, ApiError{503, "ServiceUnavailable", "no endpoints available for service \"" + svc + "\""}.status_json().dump());
    return;
  }
  std::string url = "http://" + ip + ":" + std::to_string(tport) + "/" + rest + (req.raw_query.empty() ? "" : "?" + req.raw_query);
  Headers h;
  for (const auto& kv : req.headers)
    if (to_lower(kv.first) != "host" && to_lower(kv.first) != "content-length" && to_lower(kv.first) != "connection")
      h[kv.first] = kv.second;
  HttpResult r = http_request(req.method, url, req.body, h, 30000);
  if (r.status == 0) {
    resp.json(502, ApiError{502, "BadGateway", r.error}.status_json().dump());
    return;
  }
  resp.status = r.status;
  resp.body = r.body;
  for (const auto& kv : r.headers) {
    std::string k = to_lower(kv.first);
    if (k == "content-length" || k == "transfer-encoding" || k == "connection") continue;
    resp.headers[kv.first] = kv.second;
  }
}

void ApiServer::handle_http(HttpRequest& req, HttpResponse& resp) {
  const std::string& path = req.path;
  if (path == "/healthz" || path == "/readyz" || path == "/livez") {
    resp.text(200, "ok");
    return;
  }
  if (path == "/version") {
    resp.json(200, Json{{"major", "1"}, {"minor", "29"}, {"gitVersion", "v1.29.0-kflite"}, {"platform", "linux/amd64"},
                        {"goVersion", "n/a (C++17)"}}.dump());
    return;
  }
  if (path == "/metrics") {
    resp.text(200, Registry::global().expose(), "text/plain; version=0.0.4");
    return;
  }
  if (path == "/debug/faults") {
    if (req.method == "DELETE") {
      clear_faults();
      resp.json(200, "{}");
      return;
    }
    Json b;
    if (!Json::try_parse(req.body, b)) {
      resp.json(400, R"({"error":"body must be JSON {\"spec\": \"kind:plural:count[:arg]\"}"})");
      return;
    }
    std::string err = inject_fault(b["spec"].as_string());
    resp.json(err.empty() ? 200 : 400, Json{{"error", err}}.dump());
    return;
  }
  auto segs = split(path, '/', true);
  if (segs.empty()) {
    resp.json(200, Json{{"paths", Json::array({"/api", "/api/v1", "/apis", "/healthz", "/metrics", "/version"})}}.dump());
    return;
  }
  if (segs[0] != "api" && segs[0] != "apis") {
    send_error(resp, ApiError::NotFound("path", path));
    return;
  }
  if (segs.size() == 1 || (segs[0] == "api" && segs.size() == 2) || (segs[0] == "apis" && segs.size() <= 3)) {
    if (segs[0] == "apis" && segs.size() == 2) {
      // group discovery
      Json vs = Json::array();
      std::string pref;
      for (const auto& r : reg_.all())
        if (r->group == segs[1]) {
          for (const auto& v : r->versions) {
            Json e{{"groupVersion", segs[1] + "/" + v}, {"version", v}};
            bool dup = false;
            for (const auto& x : vs.as_array()) dup = dup || x == e;
            if (!dup) vs.push_back(e);
          }
          pref = r->storage_version;
        }
      if (vs.empty()) {
        send_error(resp, ApiError::NotFound("group", segs[1]));
        return;
      }
      resp.json(200, Json{{"kind", "APIGroup"}, {"apiVersion", "v1"}, {"name", segs[1]}, {"versions", vs},
                          {"preferredVersion", Json{{"groupVersion", segs[1] + "/" + pref}, {"version", pref}}}}.dump());
      return;
    }
    http_discovery(req, resp, segs);
    return;
  }
  std::string group, version;
  size_t i;
  if (segs[0] == "api") {
    version = segs[1];
    i = 2;
  } else {
    group = segs[1];
    version = segs[2];
    i = 3;
  }
  std::string ns, plural, name, sub;
  std::vector<std::string> rest(segs.begin() + static_cast<long>(i), segs.end());
  if (rest.size() >= 2 && rest[0] == "namespaces" && group.empty() && rest.size() >= 3) {
    ns = rest[1];
    rest.erase(rest.begin(), rest.begin() + 2);
  } else if (rest.size() >= 3 && rest[0] == "namespaces" && !group.empty()) {
    ns = rest[1];
    rest.erase(rest.begin(), rest.begin() + 2);
  }
  if (rest.empty()) {
    send_error(resp, ApiError::NotFound("resource", path));
    return;
  }
  plural = rest[0];
  if (rest.size() > 1) name = rest[1];
  if (rest.size() > 2) sub = rest[2];
  auto res = reg_.by_plural(group, plural);
  if (!res || !res->serves(version)) {
    send_error(resp, ApiError::NotFound("the server could not find the requested resource", plural));
    return;
  }
  UserInfo user;
  if (!authenticate(req, user)) {
    resp.json(401, ApiError{401, "Unauthorized", "Unauthorized"}.status_json().dump());
    return;
  }
  bool watch = req.q("watch") == "true" || req.q("watch") == "1";
  std::string verb = verb_for(req.method, !name.empty(), watch);
  // pods/exec runs a command in the container whatever the HTTP method (kubectl upgrades a GET to a
  // stream): authorize it as "create", as Kubernetes does since CVE-2018-1002105's follow-ups, so a role
  // with only get on pods/* cannot run commands
  if (group.empty() && plural == "pods" && (sub == "exec" || sub == "attach")) verb = "create";
  std::string authz_sub = sub;
  if (cfg_.authz_rbac) {
    std::string reason;
    if (!authorize(user, verb, group, plural, authz_sub, ns, name, &reason)) {
      send_error(resp, ApiError::Forbidden(plural + (group.empty() ? "" : "." + group) + " \"" + name + "\" is forbidden: User \"" +
                                           user.username + "\" cannot " + verb + " resource \"" + plural + "\" in API group \"" +
                                           group + "\"" + (ns.empty() ? "" : " in the namespace \"" + ns + "\"")),
                 res->kind, name);
      return;
    }
  }
  double t0 = now_seconds();
  WriteOptions wo;
  wo.user = user;
  wo.dry_run = req.q("dryRun") == "All";
  wo.field_manager = req.q("fieldManager");
  ListOptions lo;
  lo.label_selector = req.q("labelSelector");
  lo.field_selector = req.q("fieldSelector");
  lo.resource_version = req.q("resourceVersion");
  lo.limit = std::atoll(req.q("limit", "0").c_str());
  lo.continue_token = req.q("continue");
  lo.timeout_seconds = std::atoi(req.q("timeoutSeconds", "0").c_str());
  lo.allow_bookmarks = req.q("allowWatchBookmarks") == "true";

  // subresources handled specially
  if (res->group.empty() && plural == "pods" && sub == "log") {
    std::string out;
    if (!log_provider_ || !log_provider_(ns, name, req.q("container"), std::atoll(req.q("tailLines", "-1").c_str()), out)) {
      Json p;
      if (ApiError e = r_get(res, version, ns, name, p)) {
        send_error(resp, e, "Pod", name);
        return;
      }
      resp.json(400, ApiError::BadRequest("container logs are not available for pod " + name).status_json().dump());
      return;
    }
    resp.text(200, out);
    return;
  }
  if (res->group.empty() && plural == "serviceaccounts" && sub == "token") {
    // TokenRequest (authentication.k8s.io/v1): a bound token for the ServiceAccount; authorized
    // above as "create serviceaccounts/token"
    if (req.method != "POST") {
      resp.json(405, ApiError{405, "MethodNotAllowed", "TokenRequest takes POST"}.status_json().dump());
      return;
    }
    Json body;
    if (!req.body.empty() && !Json::try_parse(req.body, body)) {
      resp.json(400, ApiError::BadRequest("invalid TokenRequest body").status_json().dump());
      return;
    }
    std::string token;
    double exp = 0;
    if (ApiError e = issue_sa_token(ns, name, body.at_path({"spec", "expirationSeconds"}).as_int(3600), token, exp)) {
      send_error(resp, e, "ServiceAccount", name);
      return;
    }
    Json spec = body["spec"].is_object() ? body["spec"] : Json::object();
    resp.json(201, Json{{"apiVersion", "authentication.k8s.io/v1"}, {"kind", "TokenRequest"},
                        {"metadata", Json{{"name", name}, {"namespace", ns}}}, {"spec", spec},
                        {"status", Json{{"token", token},
                                        {"expirationTimestamp", rfc3339_from_ms(static_cast<int64_t>(exp * 1000))}}}}
                       .dump());
    return;
  }
  if (res->group.empty() && plural == "pods" && sub == "exec") {
    // kubectl exec without a TTY or stdin: ?command=a&command=b[&container=c][&timeoutSeconds=n];
    // reply {"exitCode": n, "output": "<stdout+stderr>"} (authorized above as create pods/exec)
    if (req.method != "POST" && req.method != "GET") {
      resp.json(405, ApiError{405, "MethodNotAllowed", "exec takes POST"}.status_json().dump());
      return;
    }
    auto it = req.query.find("command");
    if (it == req.query.end() || it->second.empty()) {
      resp.json(400, ApiError::BadRequest("you must specify at least one command for the container").status_json().dump());
      return;
    }
    Json p;
    if (ApiError e = r_get(res, version, ns, name, p)) {
      send_error(resp, e, "Pod", name);
      return;
    }
    // each exec holds an API server worker for its duration: at most kMaxConcurrentExec at once, so
    // long execs can never starve controllers and watches of workers
    static std::atomic<int> active_exec{0};
    constexpr int kMaxConcurrentExec = 4;
    if (active_exec.fetch_add(1) >= kMaxConcurrentExec) {
      active_exec.fetch_sub(1);
      resp.json(429, ApiError{429, "TooManyRequests", "too many concurrent exec sessions, retry later"}.status_json().dump());
      return;
    }
    struct ExecSlot {
      std::atomic<int>& n;
      ~ExecSlot() { n.fetch_sub(1); }
    } exec_slot{active_exec};
    int code = 0;
    std::string out, err;
    // bounded: the request holds one API server worker for its duration
    const double timeout = std::min(3600.0, std::max(1.0, std::atof(req.q("timeoutSeconds", "30").c_str())));
    if (!exec_provider_ || !exec_provider_(ns, name, req.q("container"), it->second, timeout, code, out, err)) {
      resp.json(400, ApiError::BadRequest(err.empty() ? "exec is not available for pod " + name : err).status_json().dump());
      return;
    }
    resp.json(200, Json{{"exitCode", static_cast<int64_t>(code)}, {"output", out}}.dump());
    return;
  }
  if (res->group.empty() && plural == "services" && sub == "proxy") {
    std::string r;
    for (size_t k = 3; k < rest.size(); ++k) r += (k > 3 ? "/" : "") + rest[k];
    if (ends_with(path, "/") && !r.empty()) r += "/";
    http_proxy(req, resp, ns, name, r);
    return;
  }
  if (!sub.empty() && sub != "status" && sub != "scale" && !(res->group.empty() && plural == "pods" && sub == "binding")) {
    send_error(resp, ApiError::NotFound("subresource", sub));
    return;
  }
  ApiError err;
  Json out;
  int code = 200;
  if (req.method == "GET") {
    if (watch) {
      http_watch(res, version, ns, lo, resp);
      return;
    }
    if (!name.empty()) {
      err = r_get(res, version, ns, name, out);
      if (!err && sub == "scale")
        out = Json{{"apiVersion", "autoscaling/v1"}, {"kind", "Scale"},
                   {"metadata", Json{{"name", name}, {"namespace", ns}}},
                   {"spec", Json{{"replicas", out.at_path({"spec", "replicas"})}}},
                   {"status", Json{{"replicas", out.at_path({"status", "replicas"})}}}};
    } else {
      err = r_list(res, version, ns, lo, out);
    }
  } else if (req.method == "POST") {
    if (!Json::try_parse(req.body, out)) {
      send_error(resp, ApiError::BadRequest("invalid JSON body"));
      return;
    }
    if (sub == "binding") {
      // pods/{name}/binding: set spec.nodeName
      Json pod;
      err = r_get(res, version, ns, name, pod);
      if (!err) {
        pod["spec"]["nodeName"] = out.at_path({"target", "name"});
        WriteOptions sys = wo;
        err = r_update(res, version, ns, name, pod, sys, "");
        out = ApiError{}.status_json();
        code = 201;
      }
    } else {
      err = r_create(res, version, ns, out, wo);
      code = res->virtual_only ? 201 : 201;
    }
  } else if (req.method == "PUT") {
    if (!Json::try_parse(req.body, out)) {
      send_error(resp, ApiError::BadRequest("invalid JSON body"));
      return;
    }
    err = r_update(res, version, ns, name, out, wo, sub);
  } else if (req.method == "PATCH") {
    Json p;
    if (!Json::try_parse(req.body, p)) {
      send_error(resp, ApiError::BadRequest("invalid JSON patch body (YAML apply bodies must be sent as JSON)"));
      return;
    }
    std::string ct = to_lower(req.header("Content-Type", "application/merge-patch+json"));
    if (contains(ct, "apply-patch")) {
      // server-side apply (simplified): create if missing, else merge
      Json cur;
      if (r_get(res, version, ns, name, cur).code == 404) {
        p["metadata"]["name"] = name;
        err = r_create(res, version, ns, p, wo);
        out = p;
        code = 201;
      } else {
        err = r_patch(res, version, ns, name, "merge", p, out, wo, sub);
      }
    } else {
      err = r_patch(res, version, ns, name, ct, p, out, wo, sub);
    }
  } else if (req.method == "DELETE") {
    DeleteOptions d;
    d.user = user;
    d.dry_run = wo.dry_run;
    d.propagation = req.q("propagationPolicy");
    d.grace_seconds = req.has_q("gracePeriodSeconds") ? std::atoll(req.q("gracePeriodSeconds").c_str()) : -1;
    Json body;
    if (!req.body.empty() && Json::try_parse(req.body, body)) {
      if (body["propagationPolicy"].is_string()) d.propagation = body["propagationPolicy"].as_string();
      if (body["gracePeriodSeconds"].is_number()) d.grace_seconds = body["gracePeriodSeconds"].as_int();
      if (body["dryRun"].is_array() && !body["dryRun"].empty()) d.dry_run = true;
      d.precondition_uid = body.at_path({"preconditions", "uid"}).as_string();
      d.precondition_rv = body.at_path({"preconditions", "resourceVersion"}).as_string();
    }
    if (!name.empty()) {
      Json deleted;
      err = r_delete(res, ns, name, d, &deleted);
      if (!err) {
        out = deleted;
        if (!out.is_null()) convert_out(res, version, out);
      }
    } else {
      Json lst;
      err = r_list(res, version, ns, lo, lst);
      if (!err) {
        for (const auto& item : lst["items"].as_array())
          r_delete(res, item.str_at({"metadata", "namespace"}), item.str_at({"metadata", "name"}), d);
        out = ApiError{}.status_json();
      }
    }
  } else {
    send_error(resp, ApiError{405, "MethodNotAllowed", "method not allowed"});
    return;
  }

  Registry::global()
      .histogram("apiserver_http_request_duration_seconds", "kube-lite HTTP request latency", {"verb", "resource"},
                 HistogramVec::exponential(0.0001, 2, 18))
      ->observe({verb, plural}, now_seconds() - t0);
  if (err) {
    send_error(resp, err, res->kind, name);
    return;
  }
  resp.json(code, out.dump());
}

}  // namespace kf
