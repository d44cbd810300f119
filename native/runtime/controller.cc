// controller.cc — Controller, EventRecorder and Manager (see runtime.h).
#include <unistd.h>

#include <algorithm>
#include <chrono>

#include "core/util.h"
#include "runtime/runtime.h"

namespace kf {

// ---- Controller -----------------------------------------------------------------------------------
Controller::Controller(std::string name, ReconcileFn fn, int workers)
    : name_(std::move(name)), fn_(std::move(fn)), workers_(std::max(1, workers)), q_(name_) {
  total_ = Registry::global().counter("controller_runtime_reconcile_total",
                                      "Total number of reconciliations per controller", {"controller", "result"});
  errors_ = Registry::global().counter("controller_runtime_reconcile_errors_total",
                                       "Total number of reconciliation errors per controller", {"controller"});
  latency_ = Registry::global().histogram("controller_runtime_reconcile_time_seconds",
                                          "Length of time per reconciliation per controller", {"controller"},
                                          HistogramVec::exponential(0.0001, 2, 20));
}

Controller::~Controller() { stop(); }

void Controller::For(Informer& inf, Predicate pred) {
  inf.add_handler([this, pred](const std::string& type, const Json& obj, const Json* old) {
    if (pred && !pred(type, obj, old)) return;
    q_.add(Request{obj.str_at({"metadata", "namespace"}), obj.str_at({"metadata", "name"})});
  });
}

void Controller::Owns(Informer& inf, const std::string& owner_kind, Predicate pred) {
  inf.add_handler([this, owner_kind, pred](const std::string& type, const Json& obj, const Json* old) {
    if (pred && !pred(type, obj, old)) return;
    const Json* c = controller_of(obj);
    if (!c && old) c = controller_of(*old);
    if (!c || (*c)["kind"].as_string() != owner_kind) return;
    q_.add(Request{obj.str_at({"metadata", "namespace"}), (*c)["name"].as_string()});
  });
}

void Controller::Watches(Informer& inf, std::function<std::vector<Request>(const std::string&, const Json&)> map,
                         Predicate pred) {
  inf.add_handler([this, map, pred](const std::string& type, const Json& obj, const Json* old) {
    if (pred && !pred(type, obj, old)) return;
    for (const auto& r : map(type, obj)) q_.add(r);
  });
}

void Controller::start() {
  if (running_.exchange(true)) return;
  for (int i = 0; i < workers_; ++i) threads_.emplace_back([this] {
    set_thread_name("c:" + name_);
    worker();
  });
}

void Controller::stop() {
  if (!running_.exchange(false)) return;
  q_.shutdown();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
}

void Controller::worker() {
  while (running_) {
    Request r;
    if (!q_.get(r, 200)) continue;
    double t0 = now_seconds();
    std::string err;
    Result res;
    try {
      res = fn_(r, &err);
    } catch (const std::exception& e) {
      err = std::string("panic: ") + e.what();
    }
    latency_->observe({name_}, now_seconds() - t0);
    reconciles_++;
    if (!err.empty()) {
      total_->inc({name_, "error"});
      errors_->inc({name_});
      KF_ERROR(name_, "Reconciler error", Json{{"request", r.str()}, {"error", err}});
      q_.add_rate_limited(r);
    } else if (res.requeue_after > 0) {
      total_->inc({name_, "requeue_after"});
      q_.forget(r);
      q_.add_after(r, res.requeue_after);
    } else if (res.requeue) {
      total_->inc({name_, "requeue"});
      q_.add_rate_limited(r);
    } else {
      total_->inc({name_, "success"});
      q_.forget(r);
    }
    q_.done(r);
  }
}

// ---- EventRecorder ----------------------------------------------------------------------------------
void EventRecorder::event(const Json& obj, const std::string& type, const std::string& reason, const std::string& message) {
  const std::string ns = obj.str_at({"metadata", "namespace"}, "default");
  const std::string key = obj.str_at({"metadata", "uid"}) + "|" + reason + "|" + message + "|" + type;
  std::string existing;
  int64_t count = 1;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = seen_.find(key);
    if (it != seen_.end()) {
      existing = it->second.first;
      count = ++it->second.second;
    }
  }
  if (!existing.empty()) {
    Json out;
    ApiError e = c_->patch("v1", "Event", ns, existing, "merge", Json{{"count", count}, {"lastTimestamp", rfc3339_now()}}, out);
    if (!e) return;
  }
  const std::string name = obj.str_at({"metadata", "name"}) + "." + random_hex(8);
  Json ev{{"apiVersion", "v1"},
          {"kind", "Event"},
          {"metadata", Json{{"name", name}, {"namespace", ns}}},
          {"involvedObject", Json{{"apiVersion", obj["apiVersion"]}, {"kind", obj["kind"]}, {"name", obj.at_path({"metadata", "name"})},
                                  {"namespace", ns}, {"uid", obj.at_path({"metadata", "uid"})},
                                  {"resourceVersion", obj.at_path({"metadata", "resourceVersion"})}}},
          {"reason", reason},
          {"message", message},
          {"type", type},
          {"count", 1},
          {"firstTimestamp", rfc3339_now()},
          {"lastTimestamp", rfc3339_now()},
          {"source", Json{{"component", component_}}},
          {"reportingComponent", component_}};
  if (!c_->create(ev)) {
    std::lock_guard<std::mutex> g(mu_);
    seen_[key] = {name, 1};
    if (seen_.size() > 10000) seen_.clear();
  }
}

// ---- Manager ------------------------------------------------------------------------------------------
bool parse_listen_addr(const std::string& addr, std::string& host, int& port) {
  if (addr.empty() || addr == "0") return false;
  size_t c = addr.rfind(':');
  if (c == std::string::npos) {
    host = "0.0.0.0";
    port = std::atoi(addr.c_str());
    return true;
  }
  host = addr.substr(0, c);
  if (host.empty()) host = "0.0.0.0";
  port = std::atoi(addr.substr(c + 1).c_str());
  return true;
}

Manager::Manager(std::shared_ptr<Client> c, Options o) : c_(std::move(c)), o_(std::move(o)) {
  if (o_.identity.empty()) {
    char host[256] = {0};
    ::gethostname(host, sizeof host - 1);
    o_.identity = std::string(host) + "_" + random_hex(6);
  }
}

Manager::~Manager() { stop(); }

Informer& Manager::informer(const std::string& av, const std::string& kind, const std::string& ns) {
  std::lock_guard<std::mutex> g(mu_);
  const std::string key = av + "|" + kind + "|" + ns;
  auto it = informers_.find(key);
  if (it != informers_.end()) return *it->second;
  auto inf = std::make_unique<Informer>(c_, av, kind, ns);
  Informer& ref = *inf;
  informers_[key] = std::move(inf);
  if (started_) ref.start();
  return ref;
}

void Manager::add(std::shared_ptr<Controller> c) {
  std::lock_guard<std::mutex> g(mu_);
  controllers_.push_back(c);
  if (started_ && leader_) c->start();
}

void Manager::add_runnable(std::function<void(std::atomic<bool>&)> fn) {
  std::lock_guard<std::mutex> g(mu_);
  runnables_.push_back(std::move(fn));
}

void Manager::add_health_check(const std::string& name, std::function<bool()> fn) {
  std::lock_guard<std::mutex> g(mu_);
  checks_[name] = std::move(fn);
}

bool Manager::start(std::string* err) {
  std::string host;
  int port = 0;
  if (parse_listen_addr(o_.metrics_addr, host, port)) {
    metrics_srv_ = std::make_unique<HttpServer>();
    if (!metrics_srv_->listen(host, port, err)) return false;
    metrics_srv_->set_handler([](HttpRequest& req, HttpResponse& resp) {
      if (req.path == "/metrics") resp.text(200, Registry::global().expose(), "text/plain; version=0.0.4");
      else resp.text(404, "not found");
    });
    metrics_srv_->start();
  }
  if (parse_listen_addr(o_.probe_addr, host, port)) {
    probe_srv_ = std::make_unique<HttpServer>();
    if (!probe_srv_->listen(host, port, err)) return false;
    probe_srv_->set_handler([this](HttpRequest& req, HttpResponse& resp) {
      if (req.path == "/healthz" || req.path == "/readyz") {
        std::lock_guard<std::mutex> g(mu_);
        for (auto& kv : checks_)
          if (!kv.second()) {
            resp.text(500, "[-]" + kv.first + " failed");
            return;
          }
        if (req.path == "/readyz") {
          for (auto& kv : informers_)
            if (!kv.second->synced()) {
              resp.text(500, "[-]informers not synced");
              return;
            }
        }
        resp.text(200, "ok");
      } else {
        resp.text(404, "not found");
      }
    });
    probe_srv_->start();
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    started_ = true;
    for (auto& kv : informers_) kv.second->start();
  }
  // wait for caches
  std::vector<Informer*> infs;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : informers_) infs.push_back(kv.second.get());
  }
  for (auto* i : infs)
    if (!i->wait_synced(30)) {
      if (err) *err = "timed out waiting for informer " + i->kind() + " to sync";
      return false;
    }
  if (o_.leader_election) {
    leader_th_ = std::thread([this] { leader_loop(); });
  } else {
    leader_ = true;
  }
  auto launch = [this]() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& c : controllers_) c->start();
    for (auto& r : runnables_) {
      auto fn = r;
      runnable_threads_.emplace_back([this, fn] { fn(stop_); });
    }
  };
  if (leader_) {
    launch();
  } else {
    std::thread([this, launch] {
      while (!stop_ && !leader_) ::usleep(50000);
      if (!stop_) launch();
    }).detach();
  }
  return true;
}

bool Manager::try_acquire_or_renew() {
  Json lease;
  const std::string now = rfc3339_ms_now();
  ApiError e = c_->get("coordination.k8s.io/v1", "Lease", o_.leader_election_namespace, o_.leader_election_id, lease);
  if (e.code == 404) {
    Json l{{"apiVersion", "coordination.k8s.io/v1"}, {"kind", "Lease"},
           {"metadata", Json{{"name", o_.leader_election_id}, {"namespace", o_.leader_election_namespace}}},
           {"spec", Json{{"holderIdentity", o_.identity}, {"leaseDurationSeconds", 15}, {"acquireTime", now},
                         {"renewTime", now}, {"leaseTransitions", 0}}}};
    return !c_->create(l);
  }
  if (e) return false;
  const std::string holder = lease.str_at({"spec", "holderIdentity"});
  auto renew = parse_rfc3339_ms(lease.str_at({"spec", "renewTime"}));
  int64_t dur = lease.at_path({"spec", "leaseDurationSeconds"}).as_int(15) * 1000;
  bool expired = !renew || now_unix_ms() - *renew > dur;
  if (holder != o_.identity && !expired) return false;
  if (holder != o_.identity) {
    lease["spec"]["acquireTime"] = now;
    lease["spec"]["leaseTransitions"] = lease.at_path({"spec", "leaseTransitions"}).as_int(0) + 1;
  }
  lease["spec"]["holderIdentity"] = o_.identity;
  lease["spec"]["renewTime"] = now;
  return !c_->update(lease);
}

void Manager::leader_loop() {
  while (!stop_) {
    bool ok = try_acquire_or_renew();
    if (ok && !leader_) KF_INFO("leader-election", "successfully acquired lease", Json{{"id", o_.leader_election_id}});
    if (!ok && leader_) {
      KF_ERROR("leader-election", "lost lease; stopping", Json{{"id", o_.leader_election_id}});
      leader_ = false;
      stop_ = true;
      break;
    }
    leader_ = ok;
    for (int i = 0; i < 20 && !stop_; ++i) ::usleep(100000);
  }
}

void Manager::stop() {
  stop_ = true;
  if (leader_th_.joinable()) leader_th_.join();
  std::vector<std::shared_ptr<Controller>> cs;
  {
    std::lock_guard<std::mutex> g(mu_);
    cs = controllers_;
  }
  for (auto& c : cs) c->stop();
  for (auto& t : runnable_threads_)
    if (t.joinable()) t.join();
  runnable_threads_.clear();
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : informers_) kv.second->stop();
  }
  if (metrics_srv_) metrics_srv_->stop();
  if (probe_srv_) probe_srv_->stop();
}

}  // namespace kf
