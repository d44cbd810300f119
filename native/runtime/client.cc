// client.cc — LocalClient / RestClient / object helpers (see runtime.h).
#include <unistd.h>

#include <deque>

#include "core/util.h"
#include "runtime/runtime.h"

namespace kf {

// ---- Client helpers -------------------------------------------------------------------------------
ApiError Client::merge_patch(const Json& obj, const Json& p, Json* out) {
  Json o;
  ApiError e = patch(obj["apiVersion"].as_string(), obj["kind"].as_string(), obj.str_at({"metadata", "namespace"}),
                     obj.str_at({"metadata", "name"}), "application/merge-patch+json", p, o);
  if (!e && out) *out = o;
  return e;
}

ApiError Client::update_with_retry(const std::string& av, const std::string& kind, const std::string& ns,
                                   const std::string& name, const std::function<bool(Json&)>& mutate, bool status) {
  ApiError e;
  for (int i = 0; i < 5; ++i) {
    Json cur;
    e = get(av, kind, ns, name, cur);
    if (e) return e;
    if (!mutate(cur)) return {};
    e = status ? update_status(cur) : update(cur);
    if (e.code != 409) return e;
    ::usleep(10000 * (i + 1));
  }
  return e;
}

ApiError Client::update_with_retry_from(Json cur, const std::function<bool(Json&)>& mutate, bool status) {
  if (!mutate(cur)) return {};
  ApiError e = status ? update_status(cur) : update(cur);
  if (e.code != 409) return e;
  return update_with_retry(cur["apiVersion"].as_string(), cur["kind"].as_string(), cur.str_at({"metadata", "namespace"}),
                           cur.str_at({"metadata", "name"}), mutate, status);
}

// ---- LocalClient ------------------------------------------------------------------------------------
namespace {
class LocalWatch : public WatchSource {
 public:
  explicit LocalWatch(WatchPtr w) : w_(std::move(w)) {}
  bool next(WatchEvent& ev, int timeout_ms) override { return w_->next(ev, timeout_ms); }
  void stop() override { w_->stop(); }
  bool closed() override { return w_->closed(); }

 private:
  WatchPtr w_;
};
}  // namespace

ApiError LocalClient::get(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name, Json& out) {
  return s_->get(av, kind, ns, name, out);
}
ApiError LocalClient::list(const std::string& av, const std::string& kind, const std::string& ns, const ListOptions& lo, Json& out) {
  return s_->list(av, kind, ns, lo, out);
}
ApiError LocalClient::create(Json& obj, bool dry_run) {
  WriteOptions o;
  o.user = user_;
  o.dry_run = dry_run;
  return s_->create(obj, o);
}
ApiError LocalClient::update(Json& obj) {
  WriteOptions o;
  o.user = user_;
  return s_->update(obj, o);
}
ApiError LocalClient::update_status(Json& obj) {
  WriteOptions o;
  o.user = user_;
  return s_->update_status(obj, o);
}
ApiError LocalClient::patch(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name,
                            const std::string& pt, const Json& p, Json& out, const std::string& sub) {
  WriteOptions o;
  o.user = user_;
  return s_->patch(av, kind, ns, name, pt, p, out, o, sub);
}
ApiError LocalClient::remove(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name,
                             const std::string& propagation, int64_t grace) {
  DeleteOptions d;
  d.user = user_;
  d.propagation = propagation;
  d.grace_seconds = grace;
  return s_->remove(av, kind, ns, name, d);
}
std::shared_ptr<WatchSource> LocalClient::watch(const std::string& av, const std::string& kind, const std::string& ns,
                                                const ListOptions& lo, ApiError* err) {
  WatchPtr w = s_->watch(av, kind, ns, lo, err);
  if (!w) return nullptr;
  return std::make_shared<LocalWatch>(w);
}

// ---- RestClient -------------------------------------------------------------------------------------
RestClient::RestClient(std::string base_url, std::string token, int qps) : base_(std::move(base_url)), token_(std::move(token)) {
  while (!base_.empty() && base_.back() == '/') base_.pop_back();
  (void)qps;
}

ApiError RestClient::do_req(const std::string& method, const std::string& path, const std::string& body, Json& out,
                            const std::string& ctype) {
  Headers h;
  if (!token_.empty()) h["Authorization"] = "Bearer " + token_;
  if (!body.empty()) h["Content-Type"] = ctype;
  h["Accept"] = "application/json";
  HttpResult r = http_request(method, base_ + path, body, h, 30000);
  if (r.status == 0) return ApiError{503, "ServiceUnavailable", "apiserver unreachable: " + r.error};
  if (!Json::try_parse(r.body, out)) out = Json();
  if (r.status >= 400) {
    ApiError e;
    e.code = r.status;
    e.reason = out["reason"].as_string_or("Unknown");
    e.message = out["message"].as_string_or(r.body);
    return e;
  }
  return {};
}

bool RestClient::resolve(const std::string& av, const std::string& kind, Res& out, ApiError* err) {
  const std::string key = av + "|" + kind;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = cache_.find(key);
    if (it != cache_.end()) {
      out = it->second;
      return true;
    }
  }
  std::string path = av.find('/') == std::string::npos ? "/api/" + av : "/apis/" + av;
  Json disc;
  ApiError e = do_req("GET", path, "", disc);
  if (e) {
    if (err) *err = e;
    return false;
  }
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& r : disc["resources"].as_array()) {
    const std::string& name = r["name"].as_string();
    if (name.find('/') != std::string::npos) continue;
    cache_[av + "|" + r["kind"].as_string()] = Res{name, r["namespaced"].as_bool()};
  }
  auto it = cache_.find(key);
  if (it == cache_.end()) {
    if (err) *err = ApiError::NotFound("kind", av + "/" + kind);
    return false;
  }
  out = it->second;
  return true;
}

std::string RestClient::path_for(const std::string& av, const Res& r, const std::string& ns, const std::string& name,
                                 const std::string& sub) const {
  std::string p = av.find('/') == std::string::npos ? "/api/" + av : "/apis/" + av;
  if (r.namespaced && !ns.empty()) p += "/namespaces/" + url_encode(ns);
  p += "/" + r.plural;
  if (!name.empty()) p += "/" + url_encode(name);
  if (!sub.empty()) p += "/" + sub;
  return p;
}

ApiError RestClient::get(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name, Json& out) {
  Res r;
  ApiError e;
  if (!resolve(av, kind, r, &e)) return e;
  return do_req("GET", path_for(av, r, ns, name), "", out);
}

namespace {
std::string list_query(const ListOptions& lo) {
  std::vector<std::string> q;
  if (!lo.label_selector.empty()) q.push_back("labelSelector=" + url_encode(lo.label_selector));
  if (!lo.field_selector.empty()) q.push_back("fieldSelector=" + url_encode(lo.field_selector));
  if (!lo.resource_version.empty()) q.push_back("resourceVersion=" + url_encode(lo.resource_version));
  if (lo.limit > 0) q.push_back("limit=" + std::to_string(lo.limit));
  if (!lo.continue_token.empty()) q.push_back("continue=" + url_encode(lo.continue_token));
  if (lo.timeout_seconds > 0) q.push_back("timeoutSeconds=" + std::to_string(lo.timeout_seconds));
  if (lo.allow_bookmarks) q.push_back("allowWatchBookmarks=true");
  return q.empty() ? "" : "?" + join(q, "&");
}
}  // namespace

ApiError RestClient::list(const std::string& av, const std::string& kind, const std::string& ns, const ListOptions& lo, Json& out) {
  Res r;
  ApiError e;
  if (!resolve(av, kind, r, &e)) return e;
  return do_req("GET", path_for(av, r, ns, "") + list_query(lo), "", out);
}
ApiError RestClient::create(Json& obj, bool dry_run) {
  Res r;
  ApiError e;
  const std::string av = obj["apiVersion"].as_string();
  if (!resolve(av, obj["kind"].as_string(), r, &e)) return e;
  Json out;
  e = do_req("POST", path_for(av, r, obj.str_at({"metadata", "namespace"}), "") + (dry_run ? "?dryRun=All" : ""), obj.dump(), out);
  if (!e) obj = out;
  return e;
}
ApiError RestClient::update(Json& obj) {
  Res r;
  ApiError e;
  const std::string av = obj["apiVersion"].as_string();
  if (!resolve(av, obj["kind"].as_string(), r, &e)) return e;
  Json out;
  e = do_req("PUT", path_for(av, r, obj.str_at({"metadata", "namespace"}), obj.str_at({"metadata", "name"})), obj.dump(), out);
  if (!e) obj = out;
  return e;
}
ApiError RestClient::update_status(Json& obj) {
  Res r;
  ApiError e;
  const std::string av = obj["apiVersion"].as_string();
  if (!resolve(av, obj["kind"].as_string(), r, &e)) return e;
  Json out;
  e = do_req("PUT", path_for(av, r, obj.str_at({"metadata", "namespace"}), obj.str_at({"metadata", "name"}), "status"),
             obj.dump(), out);
  if (!e) obj = out;
  return e;
}
ApiError RestClient::patch(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name,
                           const std::string& pt, const Json& p, Json& out, const std::string& sub) {
  Res r;
  ApiError e;
  if (!resolve(av, kind, r, &e)) return e;
  std::string ct = pt;
  if (ct == "merge") ct = "application/merge-patch+json";
  if (ct == "json") ct = "application/json-patch+json";
  if (ct == "strategic") ct = "application/strategic-merge-patch+json";
  return do_req("PATCH", path_for(av, r, ns, name, sub), p.dump(), out, ct);
}
ApiError RestClient::remove(const std::string& av, const std::string& kind, const std::string& ns, const std::string& name,
                            const std::string& propagation, int64_t grace) {
  Res r;
  ApiError e;
  if (!resolve(av, kind, r, &e)) return e;
  std::vector<std::string> q;
  if (!propagation.empty()) q.push_back("propagationPolicy=" + propagation);
  if (grace >= 0) q.push_back("gracePeriodSeconds=" + std::to_string(grace));
  Json out;
  return do_req("DELETE", path_for(av, r, ns, name) + (q.empty() ? "" : "?" + join(q, "&")), "", out);
}

namespace {
class RestWatch : public WatchSource {
 public:
  RestWatch(std::string url, Headers h) {
    th_ = std::thread([this, url, h] {
      std::string err;
      int st = http_stream_lines("GET", url, h,
                                 [this](const std::string& line) {
                                   Json j;
                                   if (!Json::try_parse(line, j)) return true;
                                   WatchEvent ev;
                                   ev.type = j["type"].as_string();
                                   ev.object = j["object"];
                                   ev.rv = std::atoll(ev.object.str_at({"metadata", "resourceVersion"}).c_str());
                                   std::lock_guard<std::mutex> g(mu_);
                                   q_.push_back(std::move(ev));
                                   cv_.notify_one();
                                   return !stop_.load();
                                 },
                                 &stop_, 5000, &err);
      (void)st;
      std::lock_guard<std::mutex> g(mu_);
      done_ = true;
      cv_.notify_all();
    });
  }
  ~RestWatch() override {
    stop();
    if (th_.joinable()) th_.join();
  }
  bool next(WatchEvent& ev, int timeout_ms) override {
    std::unique_lock<std::mutex> g(mu_);
    if (!cv_.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return !q_.empty() || done_; })) return false;
    if (q_.empty()) return false;
    ev = std::move(q_.front());
    q_.pop_front();
    return true;
  }
  void stop() override { stop_ = true; }
  bool closed() override {
    std::lock_guard<std::mutex> g(mu_);
    return done_ && q_.empty();
  }

 private:
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<WatchEvent> q_;
  bool done_ = false;
  std::atomic<bool> stop_{false};
};
}  // namespace

std::shared_ptr<WatchSource> RestClient::watch(const std::string& av, const std::string& kind, const std::string& ns,
                                               const ListOptions& lo, ApiError* err) {
  Res r;
  if (!resolve(av, kind, r, err)) return nullptr;
  std::string q = list_query(lo);
  std::string url = base_ + path_for(av, r, ns, "") + (q.empty() ? "?watch=true" : q + "&watch=true");
  Headers h;
  if (!token_.empty()) h["Authorization"] = "Bearer " + token_;
  return std::make_shared<RestWatch>(url, h);
}

std::shared_ptr<Client> make_client(const std::string& url, ApiServer* local, const std::string& token) {
  if (!url.empty()) return std::make_shared<RestClient>(url, token);
  return std::make_shared<LocalClient>(local);
}

// ---- object helpers -------------------------------------------------------------------------------
Json owner_ref(const Json& owner, bool controller, bool block) {
  return Json{{"apiVersion", owner["apiVersion"]}, {"kind", owner["kind"]}, {"name", owner.at_path({"metadata", "name"})},
              {"uid", owner.at_path({"metadata", "uid"})}, {"controller", controller}, {"blockOwnerDeletion", block}};
}
void set_controller_reference(const Json& owner, Json& obj) {
  Json& refs = obj["metadata"]["ownerReferences"];
  Json ref = owner_ref(owner);
  if (refs.is_array())
    for (auto& r : refs.mut_array())
      if (r["uid"] == ref["uid"]) {
        r = ref;
        return;
      }
  refs.push_back(ref);
}
const Json* controller_of(const Json& obj) {
  for (const auto& r : obj.at_path({"metadata", "ownerReferences"}).as_array())
    if (r["controller"].as_bool()) return &r;
  return nullptr;
}
bool is_controlled_by(const Json& obj, const Json& owner) {
  const Json* c = controller_of(obj);
  return c && (*c)["uid"] == owner.at_path({"metadata", "uid"});
}
std::string ns_name(const Json& obj) {
  const std::string& ns = obj.str_at({"metadata", "namespace"});
  return ns.empty() ? obj.str_at({"metadata", "name"}) : ns + "/" + obj.str_at({"metadata", "name"});
}
bool has_annotation(const Json& obj, const std::string& key) {
  return obj.at_path({"metadata", "annotations"}).has(key);
}
std::string annotation(const Json& obj, const std::string& key, const std::string& def) {
  const Json& v = obj.at_path({"metadata", "annotations"}).get(key);
  return v.is_string() ? v.as_string() : def;
}
void set_annotation(Json& obj, const std::string& key, const std::string& value) {
  obj["metadata"]["annotations"][key] = value;
}
std::string label(const Json& obj, const std::string& key, const std::string& def) {
  const Json& v = obj.at_path({"metadata", "labels"}).get(key);
  return v.is_string() ? v.as_string() : def;
}

}  // namespace kf

namespace kf {
// Cluster-DNS equivalent for processes that talk to a remote API server (split binaries):
// <svc>.<ns>[.svc[.<domain>]] -> a Ready pod of the service's selector + resolved targetPort.
bool resolve_service_via(Client& c, const std::string& host, int port, std::string& ip, int& out_port) {
  auto parts = split(host, '.');
  if (parts.size() < 2 || (parts.size() > 2 && parts[2] != "svc") || host == "localhost" || starts_with(host, "127.")) return false;
  Json s;
  if (c.get("v1", "Service", parts[1], parts[0], s)) return false;
  Json target;
  for (const auto& p : s.at_path({"spec", "ports"}).as_array())
    if (p["port"].as_int() == port || s.at_path({"spec", "ports"}).size() == 1) target = p["targetPort"];
  if (target.is_null()) target = port;
  if (s.at_path({"spec", "selector"}).empty()) return false;
  LabelSelector sel = LabelSelector::from_json(Json{{"matchLabels", s.at_path({"spec", "selector"})}}, true);
  Json pods;
  if (c.list("v1", "Pod", parts[1], ListOptions(), pods)) return false;
  for (const auto& p : pods["items"].as_array()) {
    if (!sel.matches(p.at_path({"metadata", "labels"})) || p.at_path({"metadata", "deletionTimestamp"}).is_string()) continue;
    const std::string pip = p.at_path({"status", "podIP"}).as_string();
    bool ready = false;
    for (const auto& cond : p.at_path({"status", "conditions"}).as_array())
      ready = ready || (cond["type"].as_string() == "Ready" && cond["status"].as_string() == "True");
    if (pip.empty() || !ready) continue;
    int tp = target.is_number() ? static_cast<int>(target.as_int()) : 0;
    if (!target.is_number())
      for (const auto& ct : p.at_path({"spec", "containers"}).as_array())
        for (const auto& cp : ct["ports"].as_array())
          if (cp["name"].as_string() == target.as_string()) tp = static_cast<int>(cp["containerPort"].as_int());
    if (tp == 0) continue;
    ip = pip;
    out_port = tp;
    return true;
  }
  return false;
}
}  // namespace kf
