// runtime.h — the controller runtime (the C++ counterpart of controller-runtime / client-go):
//
//   Client        abstract API client; LocalClient (in-process, straight into kube-lite) and
//                 RestClient (HTTP, Kubernetes REST conventions, discovery-cached kind->plural)
//   Informer      list + watch -> local cache with indexers and event handlers; re-lists on
//                 watch failure / 410 Gone with backoff
//   WorkQueue     rate-limited, delaying, de-duplicating queue (client-go semantics: an item is
//                 never processed concurrently; per-item exponential backoff 5 ms .. 1000 s
//                 combined with a 10 qps / 100 burst token bucket)
//   Controller    N workers over a WorkQueue; For / Owns / Watches wiring; reconcile metrics
//   EventRecorder core/v1 Events with count aggregation
//   Manager       shared informers, leader election on a coordination.k8s.io Lease, /metrics,
//                 /healthz and /readyz servers, graceful start/stop
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <queue>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "apiserver/apiserver.h"
#include "core/http.h"
#include "core/json.h"
#include "core/metrics.h"

namespace kf {

// ---- client ---------------------------------------------------------------------------------
class WatchSource {
 public:
  virtual ~WatchSource() = default;
  virtual bool next(WatchEvent& ev, int timeout_ms) = 0;
  virtual void stop() = 0;
  virtual bool closed() = 0;
};

class Client {
 public:
  virtual ~Client() = default;
  virtual ApiError get(const std::string& api_version, const std::string& kind, const std::string& ns,
                       const std::string& name, Json& out) = 0;
  virtual ApiError list(const std::string& api_version, const std::string& kind, const std::string& ns,
                        const ListOptions& lo, Json& out) = 0;
  virtual ApiError create(Json& obj, bool dry_run = false) = 0;
  virtual ApiError update(Json& obj) = 0;
  virtual ApiError update_status(Json& obj) = 0;
  virtual ApiError patch(const std::string& api_version, const std::string& kind, const std::string& ns,
                         const std::string& name, const std::string& patch_type, const Json& patch, Json& out,
                         const std::string& subresource = "") = 0;
  virtual ApiError remove(const std::string& api_version, const std::string& kind, const std::string& ns,
                          const std::string& name, const std::string& propagation = "", int64_t grace = -1) = 0;
  virtual std::shared_ptr<WatchSource> watch(const std::string& api_version, const std::string& kind,
                                             const std::string& ns, const ListOptions& lo, ApiError* err) = 0;
  // Convenience: merge-patch helper; create-or-ignore-exists.
  ApiError merge_patch(const Json& obj, const Json& patch, Json* out = nullptr);
  // RetryOnConflict(DefaultRetry) helper: re-get + mutate + update until no 409 (5 attempts).
  ApiError update_with_retry(const std::string& api_version, const std::string& kind, const std::string& ns,
                             const std::string& name, const std::function<bool(Json&)>& mutate, bool status = false);
  // Same, but the first attempt mutates `cur` (an object the caller already read) instead of a
  // fresh GET: an unchanged status costs no API call at all (kubelet per-pod sync loop).
  ApiError update_with_retry_from(Json cur, const std::function<bool(Json&)>& mutate, bool status = false);
};

bool resolve_service_via(Client& c, const std::string& host, int port, std::string& ip, int& out_port);

class LocalClient : public Client {
 public:
  explicit LocalClient(ApiServer* s, UserInfo user = UserInfo()) : s_(s), user_(std::move(user)) {}
  ApiError get(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name, Json& out) override;
  ApiError list(const std::string& av, const std::string& kind, const std::string& ns, const ListOptions& lo, Json& out) override;
  ApiError create(Json& obj, bool dry_run = false) override;
  ApiError update(Json& obj) override;
  ApiError update_status(Json& obj) override;
  ApiError patch(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name,
                 const std::string& patch_type, const Json& patch, Json& out, const std::string& subresource = "") override;
  ApiError remove(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name,
                  const std::string& propagation = "", int64_t grace = -1) override;
  std::shared_ptr<WatchSource> watch(const std::string& av, const std::string& kind, const std::string& ns,
                                     const ListOptions& lo, ApiError* err) override;
  ApiServer* server() { return s_; }

 private:
  ApiServer* s_;
  UserInfo user_;
};

class RestClient : public Client {
 public:
  explicit RestClient(std::string base_url, std::string token = "", int qps = 0);
  ApiError get(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name, Json& out) override;
  ApiError list(const std::string& av, const std::string& kind, const std::string& ns, const ListOptions& lo, Json& out) override;
  ApiError create(Json& obj, bool dry_run = false) override;
  ApiError update(Json& obj) override;
  ApiError update_status(Json& obj) override;
  ApiError patch(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name,
                 const std::string& patch_type, const Json& patch, Json& out, const std::string& subresource = "") override;
  ApiError remove(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name,
                  const std::string& propagation = "", int64_t grace = -1) override;
  std::shared_ptr<WatchSource> watch(const std::string& av, const std::string& kind, const std::string& ns,
                                     const ListOptions& lo, ApiError* err) override;
  const std::string& base_url() const { return base_; }

 private:
  struct Res {
    std::string plural;
    bool namespaced = true;
  };
  bool resolve(const std::string& av, const std::string& kind, Res& out, ApiError* err);
  std::string path_for(const std::string& av, const Res& r, const std::string& ns, const std::string& name,
                       const std::string& sub = "") const;
  ApiError do_req(const std::string& method, const std::string& path, const std::string& body, Json& out,
                  const std::string& ctype = "application/json");
  std::string base_, token_;
  std::mutex mu_;
  std::map<std::string, Res> cache_;  // "av|kind" -> res
};

std::shared_ptr<Client> make_client(const std::string& url_or_empty, ApiServer* local, const std::string& token = "");

// ---- object helpers -------------------------------------------------------------------------
Json owner_ref(const Json& owner, bool controller = true, bool block_owner_deletion = true);
void set_controller_reference(const Json& owner, Json& obj);
const Json* controller_of(const Json& obj);
bool is_controlled_by(const Json& obj, const Json& owner);
std::string ns_name(const Json& obj);
bool has_annotation(const Json& obj, const std::string& key);
std::string annotation(const Json& obj, const std::string& key, const std::string& def = "");
void set_annotation(Json& obj, const std::string& key, const std::string& value);
std::string label(const Json& obj, const std::string& key, const std::string& def = "");

// ---- informer -------------------------------------------------------------------------------
class Informer {
 public:
  using Handler = std::function<void(const std::string& type, const Json& obj, const Json* old)>;
  using IndexFn = std::function<std::vector<std::string>(const Json& obj)>;
  Informer(std::shared_ptr<Client> c, std::string api_version, std::string kind, std::string ns = "",
           std::string label_selector = "");
  ~Informer();
  void add_handler(Handler h);
  void add_index(const std::string& name, IndexFn fn);
  void start();
  void stop();
  bool wait_synced(double timeout_s);
  bool synced() const { return synced_.load(); }
  bool get(const std::string& ns, const std::string& name, Json& out) const;
  std::vector<Json> list(const std::string& ns = "", const LabelSelector& sel = LabelSelector()) const;
  // Zero-copy scan of the cache (ns = "" for all) under the cache lock: the hot paths (owned-pod
  // lookup, scheduler fit, quota usage) read a few fields of every pod, and copying each cached
  // object for that was O(pods) deep copies per reconcile. fn must not call back into this informer.
  void visit(const std::string& ns, const std::function<void(const Json&)>& fn) const;
  std::vector<Json> by_index(const std::string& index, const std::string& value) const;
  const std::string& api_version() const { return av_; }
  const std::string& kind() const { return kind_; }
  size_t size() const;

 private:
  void run();
  bool relist(int64_t& rv);
  void apply(const std::string& type, const Json& obj);
  std::shared_ptr<Client> c_;
  std::string av_, kind_, ns_, labels_;
  mutable std::mutex mu_;
  std::map<std::string, Json> items_;  // ns/name
  std::map<std::string, std::pair<IndexFn, std::map<std::string, std::set<std::string>>>> indexes_;
  std::vector<Handler> handlers_;
  std::mutex handlers_mu_;
  std::atomic<bool> running_{false}, synced_{false};
  std::thread th_;
  std::shared_ptr<WatchSource> cur_watch_;
  std::mutex watch_mu_;
};

// ---- work queue ------------------------------------------------------------------------------
struct Request {
  std::string ns, name;
  bool operator<(const Request& o) const { return ns != o.ns ? ns < o.ns : name < o.name; }
  bool operator==(const Request& o) const { return ns == o.ns && name == o.name; }
  std::string str() const { return ns.empty() ? name : ns + "/" + name; }
};

class WorkQueue {
 public:
  explicit WorkQueue(std::string name, double base_delay = 0.005, double max_delay = 1000.0, double qps = 10,
                     int burst = 100);
  ~WorkQueue();
  void add(const Request& r);
  void add_after(const Request& r, double seconds);
  void add_rate_limited(const Request& r);
  void forget(const Request& r);
  int num_requeues(const Request& r);
  bool get(Request& out, int timeout_ms);  // false on timeout or shutdown
  void done(const Request& r);
  void shutdown();
  bool shutting_down() const {
    std::lock_guard<std::mutex> g(mu_);
    return shutdown_;
  }
  size_t len() const;

 private:
  void delay_loop();
  std::string name_;
  double base_, max_, qps_;
  int burst_;
  double tokens_;
  double last_refill_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Request> queue_;
  std::set<Request> dirty_, processing_;
  std::map<Request, int> failures_;
  std::map<Request, double> added_at_;  // when an item became dirty (queue-latency histogram)
  std::multimap<double, Request> delayed_;
  std::condition_variable delay_cv_;
  std::thread delay_th_;
  bool shutdown_ = false;
  std::shared_ptr<GaugeVec> depth_;
  std::shared_ptr<CounterVec> adds_, retries_;
  std::shared_ptr<HistogramVec> queue_dur_;
};

// ---- controller ------------------------------------------------------------------------------
struct Result {
  bool requeue = false;
  double requeue_after = 0;  // seconds
  static Result done() { return {}; }
  static Result after(double s) { return {false, s}; }
};
using ReconcileFn = std::function<Result(const Request& req, std::string* err)>;
using Predicate = std::function<bool(const std::string& type, const Json& obj, const Json* old)>;

class Controller {
 public:
  Controller(std::string name, ReconcileFn fn, int workers = 1);
  ~Controller();
  const std::string& name() const { return name_; }
  // For(): enqueue the object itself; Owns(): enqueue the controller owner of the given kind;
  // Watches(): arbitrary mapping.
  void For(Informer& inf, Predicate pred = nullptr);
  void Owns(Informer& inf, const std::string& owner_kind, Predicate pred = nullptr);
  void Watches(Informer& inf, std::function<std::vector<Request>(const std::string& type, const Json& obj)> map,
               Predicate pred = nullptr);
  void enqueue(const Request& r) { q_.add(r); }
  void enqueue_after(const Request& r, double s) { q_.add_after(r, s); }
  void start();
  void stop();
  WorkQueue& queue() { return q_; }
  uint64_t reconciles() const { return reconciles_.load(); }

 private:
  void worker();
  std::string name_;
  ReconcileFn fn_;
  int workers_;
  WorkQueue q_;
  std::vector<std::thread> threads_;
  std::atomic<bool> running_{false};
  std::atomic<uint64_t> reconciles_{0};
  std::shared_ptr<CounterVec> total_, errors_;
  std::shared_ptr<HistogramVec> latency_;
};

// ---- events ----------------------------------------------------------------------------------
class EventRecorder {
 public:
  EventRecorder(std::shared_ptr<Client> c, std::string component) : c_(std::move(c)), component_(std::move(component)) {}
  void event(const Json& obj, const std::string& type, const std::string& reason, const std::string& message);

 private:
  std::shared_ptr<Client> c_;
  std::string component_;
  std::mutex mu_;
  std::map<std::string, std::pair<std::string, int64_t>> seen_;  // dedup key -> (event name, count)
};

// ---- manager ---------------------------------------------------------------------------------
class Manager {
 public:
  struct Options {
    std::string metrics_addr = ":8080";  // "0" disables
    std::string probe_addr = ":8081";
    bool leader_election = false;
    std::string leader_election_id = "kfamd-controller";
    std::string leader_election_namespace = "kube-system";
    std::string identity;
  };
  Manager(std::shared_ptr<Client> c, Options o);
  ~Manager();
  std::shared_ptr<Client> client() { return c_; }
  Informer& informer(const std::string& api_version, const std::string& kind, const std::string& ns = "");
  void add(std::shared_ptr<Controller> c);
  void add_runnable(std::function<void(std::atomic<bool>& stop)> fn);
  void add_health_check(const std::string& name, std::function<bool()> fn);
  // Starts everything and returns once controllers are running (non-blocking).
  bool start(std::string* err = nullptr);
  void stop();
  bool is_leader() const { return leader_.load(); }
  int metrics_port() const { return metrics_srv_ ? metrics_srv_->port() : 0; }
  int probe_port() const { return probe_srv_ ? probe_srv_->port() : 0; }

 private:
  void leader_loop();
  bool try_acquire_or_renew();
  std::shared_ptr<Client> c_;
  Options o_;
  std::mutex mu_;
  std::map<std::string, std::unique_ptr<Informer>> informers_;
  std::vector<std::shared_ptr<Controller>> controllers_;
  std::vector<std::function<void(std::atomic<bool>&)>> runnables_;
  std::vector<std::thread> runnable_threads_;
  std::map<std::string, std::function<bool()>> checks_;
  std::unique_ptr<HttpServer> metrics_srv_, probe_srv_;
  std::atomic<bool> stop_{false}, leader_{false}, started_{false};
  std::thread leader_th_;
  std::mutex start_mu_;
  std::condition_variable start_cv_;
};

bool parse_listen_addr(const std::string& addr, std::string& host, int& port);

}  // namespace kf
