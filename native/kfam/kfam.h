// kfam.h — N19 KFAM (access management) REST service.
//
// Reference components/access-management/kfam/{routers.go,api_default.go,bindings.go,profiles.go}:
//   GET    /kfam/                         "Hello World!"
//   POST   /kfam/v1/bindings              create binding (profile owner or cluster admin only)
//   DELETE /kfam/v1/bindings              delete binding (owner / admin)
//   GET    /kfam/v1/bindings?user=&namespace=&role=   list (default: every Profile namespace)
//   POST   /kfam/v1/profiles              create Profile (v1beta1)
//   DELETE /kfam/v1/profiles/{profile}    delete Profile (owner / admin; 401 otherwise)
//   GET    /kfam/v1/role/clusteradmin?user=   "true" | "false"
//   GET    /metrics
// A binding is a RoleBinding named <kind>-<sanitized user>-<rolekind>-<role> annotated
// user/role, plus an Istio AuthorizationPolicy of the same name admitting the user's header.
// Role names map admin|edit|view <-> kubeflow-admin|kubeflow-edit|kubeflow-view.
// The requesting user is header(userid-header) minus userid-prefix.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "core/http.h"
#include "core/json.h"
#include "runtime/runtime.h"

namespace kf {

std::string kfam_binding_name(const Json& binding);  // getBindingName (bindings.go:61-77)
std::string kfam_role_map(const std::string& role);   // roleBindingNameMap, "" if unknown
Json kfam_authorization_policy_spec(const Json& binding, const std::string& userid_header, const std::string& userid_prefix);

struct KfamOptions {
  std::string userid_header = "x-goog-authenticated-user-email";
  std::string userid_prefix = "accounts.google.com:";
  std::vector<std::string> cluster_admins;
};

class KfamService {
 public:
  // role_bindings: optional informer cache (the reference reads bindings from a lister)
  KfamService(std::shared_ptr<Client> c, KfamOptions o, Informer* role_bindings = nullptr);
  ~KfamService();
  bool start(const std::string& addr, int port, std::string* err);
  void stop();
  int port() const { return srv_ ? srv_->port() : 0; }
  // exposed for tests / in-process use
  void handle(HttpRequest& req, HttpResponse& resp);

  // operations (HTTP-independent)
  ApiError create_binding(const Json& binding);
  ApiError delete_binding(const Json& binding);
  ApiError list_bindings(const std::string& user, const std::vector<std::string>& namespaces, const std::string& role,
                         Json& out);
  bool is_cluster_admin(const std::string& user) const;
  bool is_owner_or_admin(const std::string& user, const std::string& profile);

 private:
  std::string user_of(const HttpRequest& req) const;
  std::shared_ptr<Client> c_;
  KfamOptions o_;
  Informer* rbs_;
  std::unique_ptr<HttpServer> srv_;
  struct HeartbeatHolder;
  std::unique_ptr<HeartbeatHolder> hb_;
};

}  // namespace kf
