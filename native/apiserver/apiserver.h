// apiserver.h — kube-lite: an embedded, single-binary Kubernetes-convention API server.
//
// It replaces kube-apiserver + etcd for this framework and doubles as the
// envtest equivalent for the test suites (§4.4): resourceVersion + optimistic concurrency,
// generation, status/scale subresources, merge / JSON / strategic-merge patches, dry-run,
// finalizers + deletionTimestamp, graceful pod deletion, ownerReference garbage collection
// (background / foreground / orphan), namespace lifecycle, CRD registration with structural
// schema validation and "None" multi-version conversion, list/watch with label + field
// selectors and resumable watch (410 Gone on a compacted resourceVersion), an admission chain
// (in-process mutating/validating plugins + HTTP admission webhooks with failurePolicy),
// RBAC authorization + SubjectAccessReview with ClusterRole aggregation, a WAL for restart
// persistence (§5.4), and a fault-injection switchboard (§5.3).
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <fstream>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "apiserver/resources.h"
#include "apiserver/selector.h"
#include "core/http.h"
#include "core/json.h"
#include "core/metrics.h"

namespace kf {

// admission latency histograms (in-process plugins / webhooks), apiserver.cc
std::shared_ptr<HistogramVec> admission_latency(bool webhook);


struct UserInfo {
  std::string username = "system:admin";
  std::vector<std::string> groups = {"system:masters", "system:authenticated"};
};

struct ApiError {
  int code = 0;  // HTTP status; 0 = success
  std::string reason, message;
  bool ok() const { return code == 0; }
  explicit operator bool() const { return code != 0; }
  Json status_json(const std::string& kind = "", const std::string& name = "") const;
  static ApiError NotFound(const std::string& what, const std::string& name);
  static ApiError AlreadyExists(const std::string& what, const std::string& name);
  static ApiError Conflict(const std::string& msg);
  static ApiError Invalid(const std::string& msg);
  static ApiError BadRequest(const std::string& msg);
  static ApiError Forbidden(const std::string& msg);
  static ApiError Internal(const std::string& msg);
};

struct ListOptions {
  std::string label_selector, field_selector, resource_version;
  int64_t limit = 0;
  std::string continue_token;
  int timeout_seconds = 0;
  bool allow_bookmarks = false;
};

struct WriteOptions {
  bool dry_run = false;
  UserInfo user;
  std::string field_manager;
  // ?fieldValidation= for fields a structural CRD schema does not know: "Ignore" (prune silently),
  // "Warn" (the default: prune and return a Warning header per field) or "Strict" (400)
  std::string field_validation;
  std::vector<std::string>* warnings = nullptr;  // where "Warn" appends (HTTP: Warning headers)
};

struct DeleteOptions {
  bool dry_run = false;
  UserInfo user;
  std::string propagation;  // "", Foreground, Background, Orphan
  int64_t grace_seconds = -1;
  std::string precondition_uid, precondition_rv;
};

struct WatchEvent {
  std::string type;  // ADDED MODIFIED DELETED BOOKMARK ERROR
  Json object;
  int64_t rv = 0;
};

class Watch {
 public:
  // Blocks up to timeout_ms; false on timeout or when closed (check closed()).
  bool next(WatchEvent& ev, int timeout_ms);
  void stop();
  bool closed() const;

 private:
  friend class ApiServer;
  // Events are queued as shared immutable snapshots: one object per (write, served version) is
  // shared by every watcher and by the resume log; each consumer copies it in next(), on its own
  // thread and outside the API server's lock (fan-out cost no longer scales the write latency).
  struct Item {
    std::string type;
    std::shared_ptr<const Json> obj;
    int64_t rv = 0;
  };
  void push(Item ev);
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> q_;
  bool closed_ = false;
  // filter
  std::string res_key_, ns_, version_;
  std::shared_ptr<const ResourceInfo> res_;
  LabelSelector labels_;
  FieldSelector fields_;
  size_t max_queue_ = 1 << 20;
};
using WatchPtr = std::shared_ptr<Watch>;

struct AdmissionAttrs {
  std::string operation;  // CREATE UPDATE DELETE
  std::shared_ptr<const ResourceInfo> res;
  std::string subresource, ns, name, version;
  std::string uid;                   // AdmissionReview request uid (webhook mode); "" in-process
  Json* object = nullptr;            // mutable during the mutating phase
  const Json* old_object = nullptr;  // UPDATE/DELETE
  const UserInfo* user = nullptr;
  bool dry_run = false;
  // Called once when the request ends (true = object committed, false = rejected / failed / dry
  // run). Lets an admission plugin hold a reservation across the check -> commit window (quota).
  std::vector<std::function<void(bool committed)>> on_done;
};
using AdmissionFn = std::function<ApiError(AdmissionAttrs&)>;
using LogProvider = std::function<bool(const std::string& ns, const std::string& pod, const std::string& container,
                                       int64_t tail_lines, std::string& out)>;
// pods/exec (non-interactive): run argv in the container's environment, wait up to timeout_s;
// returns false when the pod / container is not running here (err says why)
using ExecProvider = std::function<bool(const std::string& ns, const std::string& pod, const std::string& container,
                                        const std::vector<std::string>& argv, double timeout_s, int& exit_code,
                                        std::string& output, std::string& err)>;

class ApiServer {
 public:
  struct Config {
    std::string data_dir;                        // "" = in-memory only
    bool authz_rbac = false;                     // false = AlwaysAllow
    std::map<std::string, UserInfo> tokens;      // bearer token -> user
    int64_t event_ttl_seconds = 3600;
    size_t watch_log_size = 200000;
    bool openshift_sa_pull_secrets = true;       // emulate OpenShift dockercfg secrets on SAs
    std::string cluster_domain = "cluster.local";
  };

  explicit ApiServer(Config cfg);
  ~ApiServer();
  void bootstrap();
  void start_background();  // GC / namespace / event-TTL / aggregation loops
  void stop();
  ResourceRegistry& registry() { return reg_; }
  const Config& config() const { return cfg_; }

  // ---- typed helpers for in-process clients (apiVersion + kind) -------------------------------
  ApiError create(Json& obj, const WriteOptions& o = {});
  ApiError get(const std::string& api_version, const std::string& kind, const std::string& ns,
               const std::string& name, Json& out);
  ApiError list(const std::string& api_version, const std::string& kind, const std::string& ns,
                const ListOptions& lo, Json& out);
  ApiError update(Json& obj, const WriteOptions& o = {});
  ApiError update_status(Json& obj, const WriteOptions& o = {});
  ApiError patch(const std::string& api_version, const std::string& kind, const std::string& ns,
                 const std::string& name, const std::string& patch_type, const Json& patch, Json& out,
                 const WriteOptions& o = {}, const std::string& subresource = "");
  ApiError remove(const std::string& api_version, const std::string& kind, const std::string& ns,
                  const std::string& name, const DeleteOptions& o = {});
  WatchPtr watch(const std::string& api_version, const std::string& kind, const std::string& ns,
                 const ListOptions& lo, ApiError* err);

  // ---- resource-level operations (HTTP layer) -------------------------------------------------
  ApiError r_create(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                    Json& obj, const WriteOptions& o);
  ApiError r_get(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                 const std::string& name, Json& out);
  ApiError r_list(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                  const ListOptions& lo, Json& out);
  ApiError r_update(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                    const std::string& name, Json& obj, const WriteOptions& o, const std::string& subresource);
  ApiError r_patch(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                   const std::string& name, const std::string& patch_type, const Json& patch, Json& out,
                   const WriteOptions& o, const std::string& subresource);
  ApiError r_delete(std::shared_ptr<const ResourceInfo> res, const std::string& ns, const std::string& name,
                    const DeleteOptions& o, Json* out = nullptr);
  WatchPtr r_watch(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                   const ListOptions& lo, ApiError* err);

  // ---- admission / authz / misc ---------------------------------------------------------------
  void add_mutating_plugin(const std::string& name, AdmissionFn fn);
  void add_validating_plugin(const std::string& name, AdmissionFn fn);
  void set_log_provider(LogProvider p) { log_provider_ = std::move(p); }
  void set_exec_provider(ExecProvider p) { exec_provider_ = std::move(p); }
  bool authorize(const UserInfo& u, const std::string& verb, const std::string& group, const std::string& resource,
                 const std::string& subresource, const std::string& ns, const std::string& name,
                 std::string* reason = nullptr);
  bool authenticate(const HttpRequest& req, UserInfo& out) const;
  // A bearer token: the static token file's, or one issued by TokenRequest for a ServiceAccount
  // that still exists (same uid) and has not expired.
  bool authenticate_token(const std::string& token, UserInfo& out) const;
  // TokenRequest (POST serviceaccounts/<name>/token): a random bound token for the ServiceAccount,
  // valid for expiration_s (clamped to [600 s, 48 h]); false when the ServiceAccount does not exist.
  ApiError issue_sa_token(const std::string& ns, const std::string& sa, int64_t expiration_s, std::string& token,
                          double& expires_unix);
  int64_t current_rv() const;
  // Fault injection: "<kind>:<plural|*>:<count>[:<arg>]", kinds: conflict, error, delay, dropwatch.
  std::string inject_fault(const std::string& spec);
  void clear_faults();

  // ---- HTTP -------------------------------------------------------------------------------------
  void handle_http(HttpRequest& req, HttpResponse& resp);

  // Resolve "<svc>.<ns>.svc[.<domain>]" / "<svc>.<ns>" to a ready pod endpoint (ip, port).
  bool resolve_service(const std::string& host, int port, std::string& ip, int& out_port);

 private:
  struct Fault {
    std::string kind, plural;
    int count = 0;
    int64_t arg = 0;
  };
  using ObjMap = std::map<std::string, Json>;  // "ns/name" -> object (storage version)

  ApiError run_admission(AdmissionAttrs& a, bool mutating);
  ApiError call_webhooks(AdmissionAttrs& a, bool mutating);
  ApiError validate(std::shared_ptr<const ResourceInfo> res, const Json& obj, const Json* old,
                    const std::string& subresource);
  static ApiError validate_workload_resources(std::shared_ptr<const ResourceInfo> res, const Json& obj);
  // structural CRD semantics on a write: prune unknown fields (reported per o.field_validation
  // when `report`), then apply schema defaults
  static ApiError structural(std::shared_ptr<const ResourceInfo> res, Json& obj, const WriteOptions& o, bool report);
  void apply_defaults(std::shared_ptr<const ResourceInfo> res, Json& obj, bool create);
  void convert_out(std::shared_ptr<const ResourceInfo> res, const std::string& version, Json& obj) const;
  void to_storage(std::shared_ptr<const ResourceInfo> res, Json& obj) const;
  std::string object_key(const std::string& ns, const std::string& name) const { return ns + "/" + name; }
  void commit_put(std::shared_ptr<const ResourceInfo> res, const std::string& key, Json& obj, const std::string& type);  // stamps obj.metadata.resourceVersion
  void commit_delete(std::shared_ptr<const ResourceInfo> res, const std::string& key);
  void broadcast(std::shared_ptr<const ResourceInfo> res, const std::string& type, const Json& obj,
                 const Json* old_obj, int64_t rv);
  void wal_append(const Json& rec);
  void load_wal();
  void post_commit(std::shared_ptr<const ResourceInfo> res, const std::string& type, const Json& obj);
  bool take_fault(const std::string& kind, const std::string& plural, int64_t* arg = nullptr);
  ApiError finalize_delete_locked(std::shared_ptr<const ResourceInfo> res, const std::string& key);
  void background_loop();
  void gc_pass();
  void namespace_pass();
  void event_ttl_pass();
  void aggregate_clusterroles();
  void bootstrap_rbac();
  bool check_namespace(std::shared_ptr<const ResourceInfo> res, const std::string& ns, bool creating, ApiError& err);
  std::string alloc_cluster_ip();
  // one parsed /api|/apis request (apiserver_http.cc: handle_http -> connect subresources | http_crud)
  struct HttpTarget {
    std::string group, version, ns, plural, name, sub, verb;
    std::vector<std::string> rest;  // path segments from the resource on
    std::shared_ptr<const ResourceInfo> res;
    UserInfo user;
    bool watch = false;
  };
  void http_faults(HttpRequest& req, HttpResponse& resp);
  void http_group_discovery(HttpResponse& resp, const std::string& group);
  bool http_connect_subresource(HttpRequest& req, HttpResponse& resp, const HttpTarget& t);
  void http_token_request(HttpRequest& req, HttpResponse& resp, const HttpTarget& t);
  void http_exec(HttpRequest& req, HttpResponse& resp, const HttpTarget& t);
  void http_crud(HttpRequest& req, HttpResponse& resp, const HttpTarget& t);
  ApiError http_write(HttpRequest& req, const HttpTarget& t, Json& body, const WriteOptions& wo, Json& out, int& code);
  ApiError http_delete(HttpRequest& req, const HttpTarget& t, const WriteOptions& wo, Json& out);
  static ListOptions list_options(HttpRequest& req);
  static Json scale_view(const HttpTarget& t, const Json& obj);
  void http_discovery(HttpRequest& req, HttpResponse& resp, const std::vector<std::string>& segs);
  void http_watch(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                  const ListOptions& lo, HttpResponse& resp);
  void http_proxy(HttpRequest& req, HttpResponse& resp, const std::string& ns, const std::string& svc_port,
                  const std::string& rest);

  Config cfg_;
  ResourceRegistry reg_;
  mutable std::mutex mu_;
  std::map<std::string, ObjMap> data_;  // res key -> objects
  std::map<std::string, std::string> uid_index_;  // uid -> "reskey|ns/name"
  int64_t rv_ = 1;
  struct LogEntry {
    std::string res_key, type;
    std::shared_ptr<const Json> obj;  // storage version
    int64_t rv = 0;
  };
  std::deque<LogEntry> log_;  // for resumable watches
  std::list<std::weak_ptr<Watch>> watchers_;
  std::vector<std::pair<std::string, AdmissionFn>> mutating_, validating_;
  LogProvider log_provider_;
  ExecProvider exec_provider_;
  std::ofstream wal_;
  std::mutex wal_mu_;
  size_t wal_records_ = 0;
  std::vector<Fault> faults_;
  std::mutex fault_mu_;
  std::atomic<bool> running_{false};
  std::thread bg_;
  std::mutex bg_mu_;
  std::condition_variable bg_cv_;
  bool bg_kick_ = false;
  uint32_t next_ip_ = 1;
  struct SaToken {
    std::string ns, name, uid;
    double expires = 0;  // unix seconds
  };
  mutable std::mutex tok_mu_;
  std::map<std::string, SaToken> sa_tokens_;  // issued token -> service account
};

}  // namespace kf
