// kfam.cc — N19 KFAM REST service (see kfam.h).
#include "kfam/kfam.h"

#include <cctype>

#include "controllers/profile.h"
#include "core/metrics.h"
#include "core/util.h"

namespace kf {

namespace {
constexpr const char* kComponent = "kfam";

std::string sanitize(const std::string& s) {
  // regexp [^a-zA-Z0-9]+ -> "-"
  std::string out;
  bool in_run = false;
  for (char ch : s) {
    if (std::isalnum(static_cast<unsigned char>(ch))) {
      out += ch;
      in_run = false;
    } else if (!in_run) {
      out += '-';
      in_run = true;
    }
  }
  return out;
}
}  // namespace

std::string kfam_binding_name(const Json& b) {
  const std::string raw = to_lower(b.at_path({"user", "kind"}).as_string() + "-" + sanitize(b.at_path({"user", "name"}).as_string()) +
                                   "-" + b.at_path({"RoleRef", "kind"}).as_string() + "-" + b.at_path({"RoleRef", "name"}).as_string());
  return sanitize(raw);
}

std::string kfam_role_map(const std::string& role) {
  static const std::map<std::string, std::string> m = {{"kubeflow-admin", "admin"}, {"kubeflow-edit", "edit"},
                                                       {"kubeflow-view", "view"},  {"admin", "kubeflow-admin"},
                                                       {"edit", "kubeflow-edit"},  {"view", "kubeflow-view"}};
  auto it = m.find(role);
  return it == m.end() ? "" : it->second;
}

Json kfam_authorization_policy_spec(const Json& b, const std::string& header, const std::string& prefix) {
  const std::string igw = getenv_or("ISTIO_INGRESS_GATEWAY_PRINCIPAL", "cluster.local/ns/istio-system/sa/istio-ingressgateway-service-account");
  const std::string kfp = getenv_or("KFP_UI_PRINCIPAL", "cluster.local/ns/kubeflow/sa/ml-pipeline-ui");
  return Json{{"rules", Json::array({Json{{"when", Json::array({Json{{"key", "request.headers[" + header + "]"},
                                                                      {"values", Json::array({prefix + b.at_path({"user", "name"}).as_string()})}}})},
                                          {"from", Json::array({Json{{"source", Json{{"principals", Json::array({igw, kfp})}}}}})}}})}};
}

struct KfamService::HeartbeatHolder {
  Heartbeat hb{kComponent, 10.0, "critical"};
};

KfamService::KfamService(std::shared_ptr<Client> c, KfamOptions o, Informer* rbs)
    : c_(std::move(c)), o_(std::move(o)), rbs_(rbs), hb_(std::make_unique<HeartbeatHolder>()) {}

KfamService::~KfamService() { stop(); }

bool KfamService::is_cluster_admin(const std::string& user) const {
  for (const auto& a : o_.cluster_admins)
    if (a == user) return true;
  return false;
}

bool KfamService::is_owner_or_admin(const std::string& user, const std::string& profile) {
  const bool admin = is_cluster_admin(user);
  Json p;
  if (c_->get("kubeflow.org/v1beta1", "Profile", "", profile, p)) return false;  // missing profile: nobody
  return admin || p.at_path({"spec", "owner", "name"}).as_string() == user;
}

std::string KfamService::user_of(const HttpRequest& req) const {
  const std::string v = req.header(o_.userid_header);
  return v.size() >= o_.userid_prefix.size() ? v.substr(o_.userid_prefix.size()) : "";
}

ApiError KfamService::create_binding(const Json& b) {
  const std::string name = kfam_binding_name(b);
  const std::string ns = b["referredNamespace"].as_string();
  const std::string role = b.at_path({"RoleRef", "name"}).as_string();
  Json subj = b["user"];
  Json rb{{"apiVersion", "rbac.authorization.k8s.io/v1"},
          {"kind", "RoleBinding"},
          {"metadata", Json{{"name", name}, {"namespace", ns}, {"annotations", Json{{"user", b.at_path({"user", "name"})}, {"role", role}}}}},
          {"roleRef", Json{{"apiGroup", b.at_path({"RoleRef", "apiGroup"}).as_string_or("rbac.authorization.k8s.io")},
                           {"kind", b.at_path({"RoleRef", "kind"})},
                           {"name", kfam_role_map(role)}}},
          {"subjects", Json::array({subj})}};
  ApiError e = c_->create(rb);
  if (e) return e;
  Json ap{{"apiVersion", "security.istio.io/v1beta1"},
          {"kind", "AuthorizationPolicy"},
          {"metadata", Json{{"name", name}, {"namespace", ns}, {"annotations", Json{{"user", b.at_path({"user", "name"})}, {"role", role}}}}},
          {"spec", kfam_authorization_policy_spec(b, o_.userid_header, o_.userid_prefix)}};
  return c_->create(ap);
}

ApiError KfamService::delete_binding(const Json& b) {
  const std::string name = kfam_binding_name(b);
  const std::string ns = b["referredNamespace"].as_string();
  Json tmp;
  ApiError e = c_->get("rbac.authorization.k8s.io/v1", "RoleBinding", ns, name, tmp);
  if (e) return e;
  e = c_->get("security.istio.io/v1beta1", "AuthorizationPolicy", ns, name, tmp);
  if (e) return e;
  e = c_->remove("rbac.authorization.k8s.io/v1", "RoleBinding", ns, name);
  if (e) return e;
  return c_->remove("security.istio.io/v1beta1", "AuthorizationPolicy", ns, name);
}

ApiError KfamService::list_bindings(const std::string& user, const std::vector<std::string>& namespaces, const std::string& role,
                                    Json& out) {
  Json bindings = Json::array();
  for (const auto& ns : namespaces) {
    std::vector<Json> rbs;
    if (rbs_ && rbs_->synced()) {
      rbs = rbs_->list(ns);
    } else {
      Json l;
      ApiError e = c_->list("rbac.authorization.k8s.io/v1", "RoleBinding", ns, ListOptions(), l);
      if (e) return e;
      rbs.assign(l["items"].as_array().begin(), l["items"].as_array().end());
    }
    for (const auto& rb : rbs) {
      if (!has_annotation(rb, "user")) continue;
      const std::string u = annotation(rb, "user");
      if (!user.empty() && user != u) continue;
      if (!has_annotation(rb, "role")) continue;
      if (!role.empty() && role != annotation(rb, "role")) continue;
      const Json& subs = rb["subjects"];
      if (subs.size() != 1)
        return ApiError::Internal("binding subject length not equal to 1, actual length: " + std::to_string(subs.size()));
      bindings.push_back(Json{{"user", Json{{"kind", subs[0]["kind"]}, {"name", subs[0]["name"]}}},
                              {"referredNamespace", ns},
                              {"RoleRef", Json{{"kind", rb.at_path({"roleRef", "kind"})},
                                               {"name", kfam_role_map(rb.at_path({"roleRef", "name"}).as_string())}}}});
    }
  }
  out = Json::object();
  if (!bindings.empty()) out["bindings"] = bindings;  // omitempty
  return {};
}

void KfamService::handle(HttpRequest& req, HttpResponse& resp) {
  resp.headers["Content-Type"] = "application/json; charset=UTF-8";
  const std::string& p = req.path;
  const std::string user = user_of(req);
  auto fail = [&](int code, const std::string& msg, const std::string& action, const std::string& u) {
    inc_request_error_counter_full(kComponent, msg, u, action, p, "major");
    resp.status = code;
    resp.body = msg;
  };
  if (p == "/kfam/" || p == "/kfam") {
    resp.text(200, "Hello World!");
    return;
  }
  if (p == "/metrics") {
    resp.text(200, Registry::global().expose(), "text/plain; version=0.0.4");
    return;
  }
  if (p == "/kfam/v1/bindings" && (req.method == "POST" || req.method == "DELETE")) {
    const std::string action = req.method == "POST" ? "create" : "delete";
    Json b;
    std::string perr;
    if (!Json::try_parse(req.body, b, &perr)) return fail(403, perr, action, "");
    if (!is_owner_or_admin(user, b["referredNamespace"].as_string())) {
      inc_request_counter_full(kComponent, "forbidden", user, action, p);
      resp.status = 403;
      return;
    }
    ApiError e = action == "create" ? create_binding(b) : delete_binding(b);
    if (e) return fail(403, e.message, action, user);
    inc_request_counter_full(kComponent, "", user, action, p);
    resp.status = 200;
    return;
  }
  if (p == "/kfam/v1/bindings" && req.method == "GET") {
    std::vector<std::string> nss;
    if (req.q("namespace").empty()) {
      Json l;
      ApiError e = c_->list("kubeflow.org/v1beta1", "Profile", "", ListOptions(), l);
      if (e) return fail(403, e.message, "read", "");
      for (const auto& pr : l["items"].as_array()) nss.push_back(pr.str_at({"metadata", "name"}));
    } else {
      nss.push_back(req.q("namespace"));
    }
    Json out;
    ApiError e = list_bindings(req.q("user"), nss, req.q("role"), out);
    if (e) return fail(401, e.message, "read", "");
    inc_request_counter_full(kComponent, "", "", "read", p);
    resp.status = 200;
    resp.body = out.dump();
    return;
  }
  if (p == "/kfam/v1/profiles" && req.method == "POST") {
    Json prof;
    std::string perr;
    if (!Json::try_parse(req.body, prof, &perr)) return fail(403, perr, "create", "");
    prof["apiVersion"] = "kubeflow.org/v1beta1";
    prof["kind"] = "Profile";
    ApiError e = c_->create(prof);
    if (e) return fail(403, e.message, "create", "");
    inc_request_counter_full(kComponent, "", "", "create", p);
    resp.status = 200;
    return;
  }
  if (starts_with(p, "/kfam/v1/profiles/") && req.method == "DELETE") {
    const std::string name = p.substr(std::string("/kfam/v1/profiles/").size());
    if (!is_owner_or_admin(user, name)) {
      inc_request_counter_full(kComponent, "forbidden", user, "delete", p);
      resp.status = 401;
      return;
    }
    ApiError e = c_->remove("kubeflow.org/v1beta1", "Profile", "", name);
    if (e) return fail(401, e.message, "delete", user);
    inc_request_counter_full(kComponent, "", user, "delete", p);
    resp.status = 200;
    return;
  }
  if (p == "/kfam/v1/role/clusteradmin" && req.method == "GET") {
    inc_request_counter_full(kComponent, "", "", "read", p);
    resp.status = 200;
    resp.body = is_cluster_admin(req.q("user")) ? "true" : "false";
    return;
  }
  resp.status = 404;
  resp.body = "404 page not found\n";
}

bool KfamService::start(const std::string& addr, int port, std::string* err) {
  srv_ = std::make_unique<HttpServer>();
  if (!srv_->listen(addr, port, err)) return false;
  srv_->set_handler([this](HttpRequest& q, HttpResponse& r) {
    const double t0 = now_seconds();
    handle(q, r);
    KF_DEBUG("kfam", q.method + " " + q.target, Json{{"status", r.status}, {"ms", (now_seconds() - t0) * 1e3}});
  });
  srv_->start();
  return true;
}

void KfamService::stop() {
  if (srv_) srv_->stop();
}

}  // namespace kf
