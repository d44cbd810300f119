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
    http_faults(req, resp);
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
    if (segs[0] == "apis" && segs.size() == 2) http_group_discovery(resp, segs[1]);
    else http_discovery(req, resp, segs);
    return;
  }
  HttpTarget t;
  size_t i;
  if (segs[0] == "api") {
    t.version = segs[1];
    i = 2;
  } else {
    t.group = segs[1];
    t.version = segs[2];
    i = 3;
  }
  t.rest.assign(segs.begin() + static_cast<long>(i), segs.end());
  if (t.rest.size() >= 3 && t.rest[0] == "namespaces") {
    t.ns = t.rest[1];
    t.rest.erase(t.rest.begin(), t.rest.begin() + 2);
  }
  if (t.rest.empty()) {
    send_error(resp, ApiError::NotFound("resource", path));
    return;
  }
  t.plural = t.rest[0];
  if (t.rest.size() > 1) t.name = t.rest[1];
  if (t.rest.size() > 2) t.sub = t.rest[2];
  t.res = reg_.by_plural(t.group, t.plural);
  if (!t.res || !t.res->serves(t.version)) {
    send_error(resp, ApiError::NotFound("the server could not find the requested resource", t.plural));
    return;
  }
  if (!authenticate(req, t.user)) {
    resp.json(401, ApiError{401, "Unauthorized", "Unauthorized"}.status_json().dump());
    return;
  }
  t.watch = req.q("watch") == "true" || req.q("watch") == "1";
  t.verb = verb_for(req.method, !t.name.empty(), t.watch);
  // pods/exec runs a command in the container whatever the HTTP method (kubectl upgrades a GET to a
  // stream): authorize it as "create", as Kubernetes does since CVE-2018-1002105's follow-ups, so a role
  // with only get on pods/* cannot run commands
  if (t.group.empty() && t.plural == "pods" && (t.sub == "exec" || t.sub == "attach")) t.verb = "create";
  if (cfg_.authz_rbac) {
    std::string reason;
    if (!authorize(t.user, t.verb, t.group, t.plural, t.sub, t.ns, t.name, &reason)) {
      send_error(resp, ApiError::Forbidden(t.plural + (t.group.empty() ? "" : "." + t.group) + " \"" + t.name +
                                           "\" is forbidden: User \"" + t.user.username + "\" cannot " + t.verb +
                                           " resource \"" + t.plural + "\" in API group \"" + t.group + "\"" +
                                           (t.ns.empty() ? "" : " in the namespace \"" + t.ns + "\"")),
                 t.res->kind, t.name);
      return;
    }
  }
  if (http_connect_subresource(req, resp, t)) return;
  if (!t.sub.empty() && t.sub != "status" && t.sub != "scale" && !(t.group.empty() && t.plural == "pods" && t.sub == "binding")) {
    send_error(resp, ApiError::NotFound("subresource", t.sub));
    return;
  }
  http_crud(req, resp, t);
}

void ApiServer::http_faults(HttpRequest& req, HttpResponse& resp) {
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
}

void ApiServer::http_group_discovery(HttpResponse& resp, const std::string& group) {
  Json vs = Json::array();
  std::string pref;
  for (const auto& r : reg_.all())
    if (r->group == group) {
      for (const auto& v : r->versions) {
        Json e{{"groupVersion", group + "/" + v}, {"version", v}};
        bool dup = false;
        for (const auto& x : vs.as_array()) dup = dup || x == e;
        if (!dup) vs.push_back(e);
      }
      pref = r->storage_version;
    }
  if (vs.empty()) {
    send_error(resp, ApiError::NotFound("group", group));
    return;
  }
  resp.json(200, Json{{"kind", "APIGroup"}, {"apiVersion", "v1"}, {"name", group}, {"versions", vs},
                      {"preferredVersion", Json{{"groupVersion", group + "/" + pref}, {"version", pref}}}}.dump());
}

// the connect-style subresources (pods/log, pods/exec, serviceaccounts/token, services/proxy):
// true when one of them handled the request
bool ApiServer::http_connect_subresource(HttpRequest& req, HttpResponse& resp, const HttpTarget& t) {
  const bool core = t.res->group.empty();
  if (core && t.plural == "pods" && t.sub == "log") {
    std::string out;
    if (!log_provider_ || !log_provider_(t.ns, t.name, req.q("container"), std::atoll(req.q("tailLines", "-1").c_str()), out)) {
      Json p;
      if (ApiError e = r_get(t.res, t.version, t.ns, t.name, p)) {
        send_error(resp, e, "Pod", t.name);
        return true;
      }
      resp.json(400, ApiError::BadRequest("container logs are not available for pod " + t.name).status_json().dump());
      return true;
    }
    resp.text(200, out);
    return true;
  }
  if (core && t.plural == "serviceaccounts" && t.sub == "token") {
    http_token_request(req, resp, t);
    return true;
  }
  if (core && t.plural == "pods" && t.sub == "exec") {
    http_exec(req, resp, t);
    return true;
  }
  if (core && t.plural == "services" && t.sub == "proxy") {
    std::string r;
    for (size_t k = 3; k < t.rest.size(); ++k) r += (k > 3 ? "/" : "") + t.rest[k];
    if (ends_with(req.path, "/") && !r.empty()) r += "/";
    http_proxy(req, resp, t.ns, t.name, r);
    return true;
  }
  return false;
}

// TokenRequest (authentication.k8s.io/v1): a bound token for the ServiceAccount; authorized as
// "create serviceaccounts/token"
void ApiServer::http_token_request(HttpRequest& req, HttpResponse& resp, const HttpTarget& t) {
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
  if (ApiError e = issue_sa_token(t.ns, t.name, body.at_path({"spec", "expirationSeconds"}).as_int(3600), token, exp)) {
    send_error(resp, e, "ServiceAccount", t.name);
    return;
  }
  Json spec = body["spec"].is_object() ? body["spec"] : Json::object();
  resp.json(201, Json{{"apiVersion", "authentication.k8s.io/v1"}, {"kind", "TokenRequest"},
                      {"metadata", Json{{"name", t.name}, {"namespace", t.ns}}}, {"spec", spec},
                      {"status", Json{{"token", token},
                                      {"expirationTimestamp", rfc3339_from_ms(static_cast<int64_t>(exp * 1000))}}}}
                     .dump());
}

// kubectl exec without a TTY or stdin: ?command=a&command=b[&container=c][&timeoutSeconds=n];
// reply {"exitCode": n, "output": "<stdout+stderr>"} (authorized as create pods/exec)
void ApiServer::http_exec(HttpRequest& req, HttpResponse& resp, const HttpTarget& t) {
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
  if (ApiError e = r_get(t.res, t.version, t.ns, t.name, p)) {
    send_error(resp, e, "Pod", t.name);
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
  const double timeout = std::min(3600.0, std::max(1.0, std::atof(req.q("timeoutSeconds", "30").c_str())));
  if (!exec_provider_ || !exec_provider_(t.ns, t.name, req.q("container"), it->second, timeout, code, out, err)) {
    resp.json(400, ApiError::BadRequest(err.empty() ? "exec is not available for pod " + t.name : err).status_json().dump());
    return;
  }
  resp.json(200, Json{{"exitCode", static_cast<int64_t>(code)}, {"output", out}}.dump());
}

// the REST verbs on a resource / collection / status / scale / binding
void ApiServer::http_crud(HttpRequest& req, HttpResponse& resp, const HttpTarget& t) {
  const double t0 = now_seconds();
  std::vector<std::string> warnings;
  WriteOptions wo;
  wo.user = t.user;
  wo.dry_run = req.q("dryRun") == "All";
  wo.field_manager = req.q("fieldManager");
  wo.field_validation = req.q("fieldValidation", "Warn");
  wo.warnings = &warnings;
  if (wo.field_validation != "Ignore" && wo.field_validation != "Warn" && wo.field_validation != "Strict") {
    send_error(resp, ApiError::BadRequest("fieldValidation must be one of Ignore, Warn or Strict"));
    return;
  }
  ApiError err;
  Json out;
  int code = 200;
  if (req.method == "GET") {
    if (t.watch) {
      http_watch(t.res, t.version, t.ns, list_options(req), resp);
      return;
    }
    if (!t.name.empty()) {
      err = r_get(t.res, t.version, t.ns, t.name, out);
      if (!err && t.sub == "scale") out = scale_view(t, out);
    } else {
      err = r_list(t.res, t.version, t.ns, list_options(req), out);
    }
  } else if (req.method == "POST" || req.method == "PUT" || req.method == "PATCH") {
    Json body;
    if (!Json::try_parse(req.body, body)) {
      send_error(resp, ApiError::BadRequest(req.method == "PATCH" ? "invalid JSON patch body (YAML apply bodies must be sent as JSON)"
                                                                  : "invalid JSON body"));
      return;
    }
    err = http_write(req, t, body, wo, out, code);
  } else if (req.method == "DELETE") {
    err = http_delete(req, t, wo, out);
  } else {
    send_error(resp, ApiError{405, "MethodNotAllowed", "method not allowed"});
    return;
  }
  Registry::global()
      .histogram("apiserver_http_request_duration_seconds", "kube-lite HTTP request latency", {"verb", "resource"},
                 HistogramVec::exponential(0.0001, 2, 18))
      ->observe({t.verb, t.plural}, now_seconds() - t0);
  if (!warnings.empty()) {
    // RFC 7234 warn-code 299, one warn-value per unknown field (kubectl prints each as "Warning: ...")
    std::vector<std::string> vals;
    for (const auto& w : warnings) vals.push_back("299 - " + Json(w).dump());
    resp.headers["Warning"] = join(vals, ", ");
  }
  if (err) {
    send_error(resp, err, t.res->kind, t.name);
    return;
  }
  resp.json(code, out.dump());
}

ListOptions ApiServer::list_options(HttpRequest& req) {
  ListOptions lo;
  lo.label_selector = req.q("labelSelector");
  lo.field_selector = req.q("fieldSelector");
  lo.resource_version = req.q("resourceVersion");
  lo.limit = std::atoll(req.q("limit", "0").c_str());
  lo.continue_token = req.q("continue");
  lo.timeout_seconds = std::atoi(req.q("timeoutSeconds", "0").c_str());
  lo.allow_bookmarks = req.q("allowWatchBookmarks") == "true";
  return lo;
}

Json ApiServer::scale_view(const HttpTarget& t, const Json& obj) {
  return Json{{"apiVersion", "autoscaling/v1"}, {"kind", "Scale"},
              {"metadata", Json{{"name", t.name}, {"namespace", t.ns}}},
              {"spec", Json{{"replicas", obj.at_path({"spec", "replicas"})}}},
              {"status", Json{{"replicas", obj.at_path({"status", "replicas"})}}}};
}

ApiError ApiServer::http_write(HttpRequest& req, const HttpTarget& t, Json& body, const WriteOptions& wo, Json& out,
                               int& code) {
  if (req.method == "POST") {
    code = 201;
    if (t.sub == "binding") {  // pods/{name}/binding: set spec.nodeName
      Json pod;
      ApiError err = r_get(t.res, t.version, t.ns, t.name, pod);
      if (err) return err;
      pod["spec"]["nodeName"] = body.at_path({"target", "name"});
      err = r_update(t.res, t.version, t.ns, t.name, pod, wo, "");
      out = ApiError{}.status_json();
      return err;
    }
    ApiError err = r_create(t.res, t.version, t.ns, body, wo);
    out = body;
    return err;
  }
  if (req.method == "PUT") {
    ApiError err = r_update(t.res, t.version, t.ns, t.name, body, wo, t.sub);
    out = body;
    return err;
  }
  const std::string ct = to_lower(req.header("Content-Type", "application/merge-patch+json"));
  if (contains(ct, "apply-patch")) {
    // server-side apply (simplified): create if missing, else merge
    Json cur;
    if (r_get(t.res, t.version, t.ns, t.name, cur).code == 404) {
      body["metadata"]["name"] = t.name;
      code = 201;
      ApiError err = r_create(t.res, t.version, t.ns, body, wo);
      out = body;
      return err;
    }
    return r_patch(t.res, t.version, t.ns, t.name, "merge", body, out, wo, t.sub);
  }
  return r_patch(t.res, t.version, t.ns, t.name, ct, body, out, wo, t.sub);
}

ApiError ApiServer::http_delete(HttpRequest& req, const HttpTarget& t, const WriteOptions& wo, Json& out) {
  DeleteOptions d;
  d.user = t.user;
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
  if (!t.name.empty()) {
    Json deleted;
    ApiError err = r_delete(t.res, t.ns, t.name, d, &deleted);
    if (!err) {
      out = deleted;
      if (!out.is_null()) convert_out(t.res, t.version, out);
    }
    return err;
  }
  Json lst;
  ApiError err = r_list(t.res, t.version, t.ns, list_options(req), lst);
  if (err) return err;
  for (const auto& item : lst["items"].as_array())
    r_delete(t.res, item.str_at({"metadata", "namespace"}), item.str_at({"metadata", "name"}), d);
  out = ApiError{}.status_json();
  return {};
}

}  // namespace kf
