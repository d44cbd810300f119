// informer.cc — list+watch cache (see runtime.h).
#include <unistd.h>

#include <chrono>

#include "core/util.h"
#include "runtime/runtime.h"

namespace kf {

Informer::Informer(std::shared_ptr<Client> c, std::string av, std::string kind, std::string ns, std::string labels)
    : c_(std::move(c)), av_(std::move(av)), kind_(std::move(kind)), ns_(std::move(ns)), labels_(std::move(labels)) {}

Informer::~Informer() { stop(); }

void Informer::add_handler(Handler h) {
  std::vector<Json> snapshot;
  {
    std::lock_guard<std::mutex> g(handlers_mu_);
    handlers_.push_back(h);
  }
  if (synced_) {
    // late registration: replay the cache as ADDED events, like SharedInformer does
    for (const auto& o : list()) h("ADDED", o, nullptr);
  }
}

void Informer::add_index(const std::string& name, IndexFn fn) {
  std::lock_guard<std::mutex> g(mu_);
  auto& idx = indexes_[name];
  idx.first = std::move(fn);
  for (const auto& kv : items_)
    for (const auto& v : idx.first(kv.second)) idx.second[v].insert(kv.first);
}

void Informer::start() {
  if (running_.exchange(true)) return;
  th_ = std::thread([this] {
    set_thread_name("i:" + kind_);
    run();
  });
}

void Informer::stop() {
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> g(watch_mu_);
    if (cur_watch_) cur_watch_->stop();
  }
  if (th_.joinable()) th_.join();
}

bool Informer::wait_synced(double timeout_s) {
  double end = now_seconds() + timeout_s;
  while (!synced_ && now_seconds() < end) ::usleep(2000);
  return synced_;
}

size_t Informer::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return items_.size();
}

bool Informer::get(const std::string& ns, const std::string& name, Json& out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = items_.find(ns + "/" + name);
  if (it == items_.end()) return false;
  out = it->second;
  return true;
}

std::vector<Json> Informer::list(const std::string& ns, const LabelSelector& sel) const {
  std::vector<Json> out;
  std::lock_guard<std::mutex> g(mu_);
  auto it = ns.empty() ? items_.begin() : items_.lower_bound(ns + "/");
  for (; it != items_.end(); ++it) {
    if (!ns.empty() && !starts_with(it->first, ns + "/")) break;
    if (sel.matches(it->second.at_path({"metadata", "labels"}))) out.push_back(it->second);
  }
  return out;
}

void Informer::visit(const std::string& ns, const std::function<void(const Json&)>& fn) const {
  std::lock_guard<std::mutex> g(mu_);
  const std::string prefix = ns + "/";
  auto it = ns.empty() ? items_.begin() : items_.lower_bound(prefix);
  for (; it != items_.end(); ++it) {
    if (!ns.empty() && it->first.compare(0, prefix.size(), prefix) != 0) break;
    fn(it->second);
  }
}

std::vector<Json> Informer::by_index(const std::string& index, const std::string& value) const {
  std::vector<Json> out;
  std::lock_guard<std::mutex> g(mu_);
  auto it = indexes_.find(index);
  if (it == indexes_.end()) return out;
  auto v = it->second.second.find(value);
  if (v == it->second.second.end()) return out;
  for (const auto& k : v->second) {
    auto o = items_.find(k);
    if (o != items_.end()) out.push_back(o->second);
  }
  return out;
}

void Informer::apply(const std::string& type, const Json& obj) {
  const std::string key = obj.str_at({"metadata", "namespace"}) + "/" + obj.str_at({"metadata", "name"});
  Json old;
  bool had = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = items_.find(key);
    if (it != items_.end()) {
      old = it->second;
      had = true;
      for (auto& idx : indexes_)
        for (const auto& v : idx.second.first(old)) idx.second.second[v].erase(key);
    }
    if (type == "DELETED") {
      items_.erase(key);
    } else {
      items_[key] = obj;
      for (auto& idx : indexes_)
        for (const auto& v : idx.second.first(obj)) idx.second.second[v].insert(key);
    }
  }
  std::vector<Handler> hs;
  {
    std::lock_guard<std::mutex> g(handlers_mu_);
    hs = handlers_;
  }
  std::string t = type;
  if (type == "ADDED" && had) t = "MODIFIED";
  for (auto& h : hs) h(t, obj, had ? &old : nullptr);
}

bool Informer::relist(int64_t& rv) {
  ListOptions lo;
  lo.label_selector = labels_;
  Json lst;
  ApiError e = c_->list(av_, kind_, ns_, lo, lst);
  if (e) return false;
  rv = std::atoll(lst.str_at({"metadata", "resourceVersion"}).c_str());
  std::set<std::string> seen;
  for (const auto& o : lst["items"].as_array()) {
    Json obj = o;
    if (!obj.has("apiVersion")) obj["apiVersion"] = av_;
    if (!obj.has("kind")) obj["kind"] = kind_;
    seen.insert(obj.str_at({"metadata", "namespace"}) + "/" + obj.str_at({"metadata", "name"}));
    Json cur;
    bool same = get(obj.str_at({"metadata", "namespace"}), obj.str_at({"metadata", "name"}), cur) &&
                cur.str_at({"metadata", "resourceVersion"}) == obj.str_at({"metadata", "resourceVersion"});
    if (!same) apply("ADDED", obj);
  }
  std::vector<Json> gone;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& kv : items_)
      if (!seen.count(kv.first)) gone.push_back(kv.second);
  }
  for (const auto& o : gone) apply("DELETED", o);
  return true;
}

void Informer::run() {
  double backoff = 0.05;
  while (running_) {
    int64_t rv = 0;
    if (!relist(rv)) {
      ::usleep(static_cast<useconds_t>(backoff * 1e6));
      backoff = std::min(backoff * 2, 5.0);
      continue;
    }
    synced_ = true;
    backoff = 0.05;
    ListOptions lo;
    lo.label_selector = labels_;
    lo.resource_version = std::to_string(rv);
    lo.allow_bookmarks = true;
    ApiError err;
    auto w = c_->watch(av_, kind_, ns_, lo, &err);
    if (!w) {
      ::usleep(100000);
      continue;
    }
    {
      std::lock_guard<std::mutex> g(watch_mu_);
      cur_watch_ = w;
    }
    while (running_) {
      WatchEvent ev;
      if (!w->next(ev, 200)) {
        if (w->closed()) break;
        continue;
      }
      if (ev.type == "ERROR") break;  // e.g. 410 Gone -> relist
      if (ev.type == "BOOKMARK") continue;
      if (!ev.object.has("apiVersion")) ev.object["apiVersion"] = av_;
      apply(ev.type, ev.object);
    }
    w->stop();
    {
      std::lock_guard<std::mutex> g(watch_mu_);
      cur_watch_.reset();
    }
  }
}

}  // namespace kf
