// apiserver.cc — core storage / admission / CRUD pipeline of kube-lite (see apiserver.h).
#include "apiserver/apiserver.h"

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>

#include "apiserver/schemas.h"
#include "core/metrics.h"
#include "core/resources.h"
#include "core/util.h"

namespace kf {

// ---- errors -------------------------------------------------------------------------------------
Json ApiError::status_json(const std::string& kind, const std::string& name) const {
  Json s{{"kind", "Status"}, {"apiVersion", "v1"}, {"metadata", Json::object()}, {"status", code ? "Failure" : "Success"},
         {"message", message}, {"reason", reason}, {"code", code ? code : 200}};
  if (!kind.empty() || !name.empty()) s["details"] = Json{{"name", name}, {"kind", kind}};
  return s;
}
ApiError ApiError::NotFound(const std::string& what, const std::string& name) {
  return {404, "NotFound", what + " \"" + name + "\" not found"};
}
ApiError ApiError::AlreadyExists(const std::string& what, const std::string& name) {
  return {409, "AlreadyExists", what + " \"" + name + "\" already exists"};
}
ApiError ApiError::Conflict(const std::string& msg) { return {409, "Conflict", msg}; }
ApiError ApiError::Invalid(const std::string& msg) { return {422, "Invalid", msg}; }
ApiError ApiError::BadRequest(const std::string& msg) { return {400, "BadRequest", msg}; }
ApiError ApiError::Forbidden(const std::string& msg) { return {403, "Forbidden", msg}; }
ApiError ApiError::Internal(const std::string& msg) { return {500, "InternalError", msg}; }

// ---- watch ----------------------------------------------------------------------------------------
bool Watch::next(WatchEvent& ev, int timeout_ms) {
  std::unique_lock<std::mutex> g(mu_);
  if (!cv_.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return !q_.empty() || closed_; })) return false;
  if (q_.empty()) return false;
  Item it = std::move(q_.front());
  q_.pop_front();
  g.unlock();
  ev.type = std::move(it.type);
  ev.object = *it.obj;
  ev.rv = it.rv;
  return true;
}
void Watch::stop() {
  std::lock_guard<std::mutex> g(mu_);
  closed_ = true;
  cv_.notify_all();
}
bool Watch::closed() const {
  std::lock_guard<std::mutex> g(mu_);
  return closed_ && q_.empty();
}
void Watch::push(Item ev) {
  std::lock_guard<std::mutex> g(mu_);
  if (closed_) return;
  if (q_.size() >= max_queue_) {  // slow consumer: terminate the watch (client re-lists)
    closed_ = true;
    cv_.notify_all();
    return;
  }
  q_.push_back(std::move(ev));
  cv_.notify_one();
}

// ---- metrics ------------------------------------------------------------------------------------
namespace {
std::shared_ptr<CounterVec> req_counter() {
  static auto c = Registry::global().counter("apiserver_request_total", "kube-lite API requests",
                                              {"verb", "resource", "code"});
  return c;
}
std::shared_ptr<HistogramVec> req_latency() {
  static auto h = Registry::global().histogram("apiserver_request_duration_seconds", "kube-lite request latency",
                                                {"verb", "resource"}, HistogramVec::exponential(0.0001, 2, 18));
  return h;
}

bool spec_changed(const Json& a, const Json& b) {
  // generation bumps when anything but metadata / status changes
  for (const auto& m : a.as_object()) {
    if (m.first == "metadata" || m.first == "status" || m.first == "apiVersion" || m.first == "kind") continue;
    if (b.get(m.first) != m.second) return true;
  }
  for (const auto& m : b.as_object()) {
    if (m.first == "metadata" || m.first == "status" || m.first == "apiVersion" || m.first == "kind") continue;
    if (!a.has(m.first)) return true;
  }
  return false;
}

std::string version_of(const std::string& api_version) {
  size_t s = api_version.find('/');
  return s == std::string::npos ? api_version : api_version.substr(s + 1);
}
}  // namespace

// ---- construction / persistence -------------------------------------------------------------------
ApiServer::ApiServer(Config cfg) : cfg_(std::move(cfg)) {}

ApiServer::~ApiServer() { stop(); }

void ApiServer::stop() {
  if (running_.exchange(false)) {
    {
      std::lock_guard<std::mutex> g(bg_mu_);
      bg_kick_ = true;
    }
    bg_cv_.notify_all();
    if (bg_.joinable()) bg_.join();
  }
  std::lock_guard<std::mutex> g(mu_);
  for (auto& w : watchers_)
    if (auto p = w.lock()) p->stop();
  watchers_.clear();
}

int64_t ApiServer::current_rv() const {
  std::lock_guard<std::mutex> g(mu_);
  return rv_;
}

void ApiServer::wal_append(const Json& rec) {
  if (cfg_.data_dir.empty()) return;
  std::lock_guard<std::mutex> g(wal_mu_);
  if (!wal_.is_open()) return;
  wal_ << rec.dump() << '\n';
  wal_.flush();
  wal_records_++;
}

void ApiServer::load_wal() {
  if (cfg_.data_dir.empty()) return;
  make_dirs(cfg_.data_dir);
  const std::string path = cfg_.data_dir + "/store.wal";
  std::string text;
  if (read_file(path, text)) {
    size_t start = 0;
    while (start < text.size()) {
      size_t nl = text.find('\n', start);
      if (nl == std::string::npos) nl = text.size();
      std::string line = text.substr(start, nl - start);
      start = nl + 1;
      if (line.empty()) continue;
      Json rec;
      if (!Json::try_parse(line, rec)) continue;  // torn tail write
      const std::string& rk = rec["r"].as_string();
      const std::string& id = rec["id"].as_string();
      if (rec["op"].as_string() == "put") {
        data_[rk][id] = rec["o"];
        uid_index_[rec["o"].str_at({"metadata", "uid"})] = rk + "|" + id;
      } else {
        auto it = data_[rk].find(id);
        if (it != data_[rk].end()) {
          uid_index_.erase(it->second.str_at({"metadata", "uid"}));
          data_[rk].erase(it);
        }
      }
      rv_ = std::max(rv_, rec["rv"].as_int());
    }
  }
  // register CRDs that were persisted
  auto crds = data_.find("apiextensions.k8s.io/customresourcedefinitions");
  if (crds != data_.end())
    for (const auto& kv : crds->second) reg_.add_crd(kv.second);
  // compact: rewrite the WAL as a snapshot of the live objects
  std::string snap;
  for (const auto& rk : data_)
    for (const auto& kv : rk.second)
      snap += Json{{"op", "put"}, {"r", rk.first}, {"id", kv.first}, {"o", kv.second}, {"rv", rv_}}.dump() + "\n";
  write_file(path, snap);
  wal_.open(path, std::ios::app);
}

// ---- bootstrap ----------------------------------------------------------------------------------
void ApiServer::bootstrap() {
  {
    std::lock_guard<std::mutex> g(mu_);
    load_wal();
  }
  WriteOptions sys;
  for (Json crd : builtin_crds()) {
    Json existing;
    if (get("apiextensions.k8s.io/v1", "CustomResourceDefinition", "", crd.str_at({"metadata", "name"}), existing).ok()) {
      if (existing["spec"] != crd["spec"]) {  // a data dir from an older build: serve this build's schemas
        existing["spec"] = crd["spec"];
        if (ApiError e = update(existing, sys))
          KF_ERROR("apiserver", "bootstrap CRD update failed", Json{{"crd", crd.str_at({"metadata", "name"})}, {"error", e.message}});
      }
      reg_.add_crd(existing);
      continue;
    }
    ApiError e = create(crd, sys);
    if (e) KF_ERROR("apiserver", "bootstrap CRD failed", Json{{"crd", crd.str_at({"metadata", "name"})}, {"error", e.message}});
  }
  for (const char* ns : {"default", "kube-system", "kube-public", "kubeflow"}) {
    Json n{{"apiVersion", "v1"}, {"kind", "Namespace"}, {"metadata", Json{{"name", ns}}}};
    Json existing;
    if (!get("v1", "Namespace", "", ns, existing).ok()) create(n, sys);
  }
  {
    Json sc{{"apiVersion", "storage.k8s.io/v1"}, {"kind", "StorageClass"},
            {"metadata", Json{{"name", "standard"},
                              {"annotations", Json{{"storageclass.kubernetes.io/is-default-class", "true"}}}}},
            {"provisioner", "kflite.io/hostpath"}, {"reclaimPolicy", "Delete"},
            {"volumeBindingMode", "Immediate"}};
    Json existing;
    if (!get("storage.k8s.io/v1", "StorageClass", "", "standard", existing).ok()) create(sc, sys);
  }
  bootstrap_rbac();
}

void ApiServer::start_background() {
  if (running_.exchange(true)) return;
  bg_ = std::thread([this] {
    set_thread_name("apiserver-bg");
    background_loop();
  });
}

// ---- conversion ---------------------------------------------------------------------------------
void ApiServer::convert_out(std::shared_ptr<const ResourceInfo> res, const std::string& version, Json& obj) const {
  std::string v = version.empty() ? res->storage_version : version;
  obj["apiVersion"] = res->api_version(v);
  obj["kind"] = res->kind;
}
void ApiServer::to_storage(std::shared_ptr<const ResourceInfo> res, Json& obj) const {
  prune_nulls(obj);
  obj["apiVersion"] = res->storage_api_version();
  obj["kind"] = res->kind;
}

// ---- faults ---------------------------------------------------------------------------------------
std::string ApiServer::inject_fault(const std::string& spec) {
  auto parts = split(spec, ':');
  if (parts.size() < 3) return "fault spec must be kind:plural:count[:arg]";
  Fault f;
  f.kind = parts[0];
  f.plural = parts[1];
  f.count = std::atoi(parts[2].c_str());
  f.arg = parts.size() > 3 ? std::atoll(parts[3].c_str()) : 0;
  // commitdelay: sleep arg ms between admission and the store commit of a create (widens the
  // check-then-commit window for admission race tests)
  if (f.kind != "conflict" && f.kind != "error" && f.kind != "delay" && f.kind != "dropwatch" && f.kind != "commitdelay")
    return "unknown fault kind " + f.kind;
  std::lock_guard<std::mutex> g(fault_mu_);
  faults_.push_back(f);
  return "";
}
void ApiServer::clear_faults() {
  std::lock_guard<std::mutex> g(fault_mu_);
  faults_.clear();
}
bool ApiServer::take_fault(const std::string& kind, const std::string& plural, int64_t* arg) {
  std::lock_guard<std::mutex> g(fault_mu_);
  for (auto it = faults_.begin(); it != faults_.end(); ++it) {
    if (it->kind == kind && (it->plural == "*" || it->plural == plural) && it->count > 0) {
      if (arg) *arg = it->arg;
      if (--it->count == 0) faults_.erase(it);
      return true;
    }
  }
  return false;
}

// ---- namespace lifecycle ------------------------------------------------------------------------
bool ApiServer::check_namespace(std::shared_ptr<const ResourceInfo> res, const std::string& ns, bool creating,
                                ApiError& err) {
  if (!res->namespaced) {
    if (!ns.empty()) {
      err = ApiError::BadRequest(res->plural + " is cluster-scoped; namespace must be empty");
      return false;
    }
    return true;
  }
  if (ns.empty()) {
    err = ApiError::BadRequest("namespace is required for " + res->plural);
    return false;
  }
  if (!creating) return true;
  std::lock_guard<std::mutex> g(mu_);
  auto& nss = data_["/namespaces"];
  auto it = nss.find("/" + ns);
  if (it == nss.end()) {
    err = ApiError::NotFound("namespaces", ns);
    return false;
  }
  if (it->second.at_path({"metadata", "deletionTimestamp"}).is_string()) {
    err = {403, "Forbidden", "unable to create new content in namespace " + ns + " because it is being terminated"};
    return false;
  }
  return true;
}

std::string ApiServer::alloc_cluster_ip() {
  uint32_t n = next_ip_++;
  return "10.96." + std::to_string((n >> 8) & 0xFF) + "." + std::to_string(n & 0xFF);
}

// ---- defaulting ---------------------------------------------------------------------------------
namespace {
void default_pod_spec(Json& spec) {
  if (!spec.has("restartPolicy")) spec["restartPolicy"] = "Always";
  if (!spec.has("terminationGracePeriodSeconds")) spec["terminationGracePeriodSeconds"] = 30;
  if (!spec.has("dnsPolicy")) spec["dnsPolicy"] = "ClusterFirst";
  if (!spec.has("schedulerName")) spec["schedulerName"] = "default-scheduler";
  if (!spec.has("securityContext")) spec["securityContext"] = Json::object();
  for (const char* list : {"containers", "initContainers"}) {
    Json* cs = spec.find(list);
    if (!cs || !cs->is_array()) continue;
    for (auto& c : cs->mut_array()) {
      if (!c.has("imagePullPolicy")) {
        const std::string& img = c["image"].as_string();
        c["imagePullPolicy"] = (ends_with(img, ":latest") || img.find(':') == std::string::npos) ? "Always" : "IfNotPresent";
      }
      if (!c.has("terminationMessagePath")) c["terminationMessagePath"] = "/dev/termination-log";
      if (!c.has("terminationMessagePolicy")) c["terminationMessagePolicy"] = "File";
      if (!c.has("resources")) c["resources"] = Json::object();
      Json* ports = c.find("ports");
      if (ports)
        for (auto& p : ports->mut_array())
          if (!p.has("protocol")) p["protocol"] = "TCP";
    }
  }
}
}  // namespace

void ApiServer::apply_defaults(std::shared_ptr<const ResourceInfo> res, Json& obj, bool create) {
  const std::string& k = res->kind;
  if (res->group.empty()) {
    if (k == "Pod") {
      default_pod_spec(obj["spec"]);
      default_requests_from_limits(obj["spec"]);  // SetDefaults_Pod: quota / scheduler read requests
      if (create) {
        obj["status"] = Json{{"phase", "Pending"}, {"qosClass", "BestEffort"}};
        bool any = false;
        for (const auto& c : obj.at_path({"spec", "containers"}).as_array())
          any = any || !c.at_path({"resources", "requests"}).empty() || !c.at_path({"resources", "limits"}).empty();
        if (any) obj["status"]["qosClass"] = "Burstable";
      }
    } else if (k == "Secret") {
      // stringData is write-only convenience: merged into data (base64) and dropped
      if (obj["stringData"].is_object()) {
        for (const auto& kv : obj["stringData"].as_object()) obj["data"][kv.first] = base64_encode(kv.second.as_string());
        obj.erase("stringData");
      }
      if (!obj.has("type")) obj["type"] = "Opaque";
    } else if (k == "Service") {
      Json& spec = obj["spec"];
      if (!spec.has("type")) spec["type"] = "ClusterIP";
      if (!spec.has("sessionAffinity")) spec["sessionAffinity"] = "None";
      if (create && !spec.has("clusterIP")) {
        std::lock_guard<std::mutex> g(mu_);
        spec["clusterIP"] = alloc_cluster_ip();
      }
      Json* ports = spec.find("ports");
      if (ports)
        for (auto& p : ports->mut_array()) {
          if (!p.has("protocol")) p["protocol"] = "TCP";
          if (!p.has("targetPort")) p["targetPort"] = p["port"];
        }
    } else if (k == "Namespace") {
      if (create) {
        obj["spec"]["finalizers"] = Json::array({"kubernetes"});
        obj["status"] = Json{{"phase", "Active"}};
      }
      obj.mut_path({"metadata", "labels"})["kubernetes.io/metadata.name"] = obj.str_at({"metadata", "name"});
    } else if (k == "PersistentVolumeClaim") {
      if (create) obj["status"] = Json{{"phase", "Pending"}};
      Json& spec = obj["spec"];
      if (!spec.has("volumeMode")) spec["volumeMode"] = "Filesystem";
    } else if (k == "ServiceAccount" && create && cfg_.openshift_sa_pull_secrets) {
      // OpenShift's token controller attaches a dockercfg pull secret to every SA; the ODH
      // reconciliation-lock removal waits for it (odh-notebook-controller/controllers/notebook_controller.go:118-146).
      Json& ips = obj["imagePullSecrets"];
      if (!ips.is_array() || ips.empty()) {
        ips = Json::array();
        ips.push_back(Json{{"name", obj.str_at({"metadata", "name"}) + "-dockercfg-" + random_alnum(5)}});
      }
    } else if (k == "Event") {
      if (!obj.has("count")) obj["count"] = 1;
      if (!obj.has("firstTimestamp")) obj["firstTimestamp"] = rfc3339_now();
      if (!obj.has("lastTimestamp")) obj["lastTimestamp"] = obj["firstTimestamp"];
      if (!obj.has("type")) obj["type"] = "Normal";
    } else if (k == "Node" && create) {
      if (!obj.has("status")) obj["status"] = Json::object();
    }
  } else if (res->group == "apps") {
    Json& spec = obj["spec"];
    if (!spec.has("replicas")) spec["replicas"] = 1;
    if (!spec.has("revisionHistoryLimit")) spec["revisionHistoryLimit"] = 10;
    if (k == "StatefulSet") {
      if (!spec.has("podManagementPolicy")) spec["podManagementPolicy"] = "OrderedReady";
      if (!spec.has("updateStrategy"))
        spec["updateStrategy"] = Json{{"type", "RollingUpdate"}, {"rollingUpdate", Json{{"partition", 0}}}};
    } else if (k == "Deployment") {
      if (!spec.has("strategy"))
        spec["strategy"] = Json{{"type", "RollingUpdate"},
                                {"rollingUpdate", Json{{"maxSurge", "25%"}, {"maxUnavailable", "25%"}}}};
      if (!spec.has("progressDeadlineSeconds")) spec["progressDeadlineSeconds"] = 600;
    }
    if (spec.at_path({"template", "spec"}).is_object()) default_pod_spec(spec["template"]["spec"]);
    if (create && !obj.has("status")) obj["status"] = Json::object();
  }
}

// ---- structural schemas (CRDs) ----------------------------------------------------------------------
ApiError ApiServer::structural(std::shared_ptr<const ResourceInfo> res, Json& obj, const WriteOptions& o, bool report) {
  if (!res->is_crd) return {};
  auto it = res->schemas.find(version_of(obj["apiVersion"].as_string()));
  if (it == res->schemas.end()) it = res->schemas.find(res->storage_version);
  if (it == res->schemas.end()) return {};
  std::vector<std::string> pruned;
  prune_unknown_fields(it->second, obj, report ? &pruned : nullptr);
  apply_schema_defaults(it->second, obj);
  if (pruned.empty()) return {};
  if (o.field_validation == "Strict") {
    std::vector<std::string> msgs;
    for (const auto& p : pruned) msgs.push_back("unknown field \"" + p + "\"");
    return ApiError::BadRequest(res->kind + " in version \"" + version_of(obj["apiVersion"].as_string()) +
                                "\" cannot be handled as a " + res->kind + ": strict decoding error: " + join(msgs, ", "));
  }
  if (o.field_validation != "Ignore" && o.warnings)
    for (const auto& p : pruned) o.warnings->push_back("unknown field \"" + p + "\"");
  return {};
}

// ---- validation ---------------------------------------------------------------------------------
// Resource requirements of a Pod or of the pod template of a StatefulSet / Deployment / ReplicaSet,
// with kube-apiserver's outcomes (core/resources.h): an unparsable quantity is a decode error (400,
// "cannot be handled as a Pod"), every other violation is one 422 listing all field errors.
ApiError ApiServer::validate_workload_resources(std::shared_ptr<const ResourceInfo> res, const Json& obj) {
  std::string path;
  if (res->group.empty() && res->kind == "Pod") path = "spec";
  else if (res->group == "apps" && (res->kind == "StatefulSet" || res->kind == "Deployment" || res->kind == "ReplicaSet"))
    path = "spec.template.spec";
  else return {};
  const Json& spec = path == "spec" ? obj["spec"] : obj.at_path({"spec", "template", "spec"});
  ResourceErrors errs;
  validate_pod_spec_resources(spec, path, errs);
  if (!errs.decode.empty())
    return ApiError::BadRequest(res->kind + " in version \"" + version_of(obj["apiVersion"].as_string()) +
                                "\" cannot be handled as a " + res->kind + ": " + errs.decode.front());
  if (errs.invalid.empty()) return {};
  const std::string what = res->group.empty() ? res->kind : res->kind + "." + res->group;
  const std::string list = errs.invalid.size() == 1 ? errs.invalid.front() : "[" + join(errs.invalid, ", ") + "]";
  return ApiError::Invalid(what + " \"" + obj.str_at({"metadata", "name"}) + "\" is invalid: " + list);
}

ApiError ApiServer::validate(std::shared_ptr<const ResourceInfo> res, const Json& obj, const Json* old,
                             const std::string& subresource) {
  const std::string& name = obj.str_at({"metadata", "name"});
  if (name.empty()) return ApiError::Invalid(res->kind + ": metadata.name: Required value: name or generateName is required");
  if (name.size() > 253) return ApiError::Invalid(res->kind + " \"" + name + "\": metadata.name: Too long");
  for (char c : name) {
    if (!(std::islower(static_cast<unsigned char>(c)) || std::isdigit(static_cast<unsigned char>(c)) || c == '-' ||
          c == '.' || (res->kind == "ClusterRole" || res->kind == "ClusterRoleBinding" || res->kind == "Role" ||
                       res->kind == "RoleBinding" ? (c == ':' || c == '_' || std::isupper(static_cast<unsigned char>(c))) : false))) {
      return ApiError::Invalid(res->kind + " \"" + name +
                               "\" is invalid: metadata.name: Invalid value: a lowercase RFC 1123 subdomain must consist of "
                               "lower case alphanumeric characters, '-' or '.'");
    }
  }
  if (subresource == "status") return {};
  if (res->is_crd) {
    auto it = res->schemas.find(version_of(obj["apiVersion"].as_string()));
    if (it == res->schemas.end()) it = res->schemas.find(res->storage_version);
    if (it != res->schemas.end()) {
      auto errs = validate_schema(it->second, obj);
      if (!errs.empty())
        return ApiError::Invalid(res->kind + ".kubeflow.org \"" + name + "\" is invalid: " + join(errs, ", "));
    }
  }
  if (ApiError re = validate_workload_resources(res, obj)) return re;
  if (res->group.empty() && res->kind == "Pod") {
    const Json& cs = obj.at_path({"spec", "containers"});
    if (!cs.is_array() || cs.empty()) return ApiError::Invalid("Pod \"" + name + "\" is invalid: spec.containers: Required value");
    for (const auto& c : cs.as_array())
      if (c["name"].as_string().empty() || c["image"].as_string().empty())
        return ApiError::Invalid("Pod \"" + name + "\" is invalid: spec.containers: name and image are required");
    if (old) {
      // pod spec is immutable except image fields / activeDeadlineSeconds / tolerations additions
      Json a = obj["spec"], b = (*old)["spec"];
      for (Json* s : {&a, &b}) {
        for (auto& c : (*s)["containers"].mut_array()) c.erase("image");
        for (auto& c : (*s)["initContainers"].mut_array()) c.erase("image");
        s->erase("activeDeadlineSeconds");
        s->erase("tolerations");
        s->erase("nodeName");  // binding subresource
      }
      if (a != b) return ApiError::Invalid("Pod \"" + name + "\" is invalid: spec: Forbidden: pod updates may not change fields other than image");
    }
  }
  if (res->group == "apps" && (res->kind == "StatefulSet" || res->kind == "Deployment")) {
    if (obj.at_path({"spec", "replicas"}).as_int(0) < 0) return ApiError::Invalid(res->kind + ": spec.replicas must be >= 0");
    const Json& cs = obj.at_path({"spec", "template", "spec", "containers"});
    if (!cs.is_array() || cs.empty()) return ApiError::Invalid(res->kind + " \"" + name + "\" is invalid: spec.template.spec.containers: Required value");
    if (old && res->kind == "StatefulSet") {
      if (obj.at_path({"spec", "selector"}) != (*old).at_path({"spec", "selector"}) ||
          obj.at_path({"spec", "serviceName"}) != (*old).at_path({"spec", "serviceName"}))
        return ApiError::Invalid("StatefulSet.apps \"" + name + "\" is invalid: spec: Forbidden: updates to statefulset spec for fields other than 'replicas', 'template', 'updateStrategy' and 'minReadySeconds' are forbidden");
    }
  }
  if (res->group.empty() && res->kind == "Service" && old) {
    const Json& a = obj.at_path({"spec", "clusterIP"});
    const Json& b = (*old).at_path({"spec", "clusterIP"});
    if (a.is_string() && b.is_string() && a != b && !a.as_string().empty())
      return ApiError::Invalid("Service \"" + name + "\" is invalid: spec.clusterIP: Invalid value: field is immutable");
  }
  return {};
}

// ---- admission ------------------------------------------------------------------------------------
void ApiServer::add_mutating_plugin(const std::string& name, AdmissionFn fn) {
  std::lock_guard<std::mutex> g(mu_);
  mutating_.emplace_back(name, std::move(fn));
}
void ApiServer::add_validating_plugin(const std::string& name, AdmissionFn fn) {
  std::lock_guard<std::mutex> g(mu_);
  validating_.emplace_back(name, std::move(fn));
}

// kube-apiserver's admission latency families: one observation per in-process plugin
// (GPU placement, quota, PodDefault, readiness injection, ...) and per webhook call, labelled with
// the plugin/webhook name, operation, mutating|validating and whether it rejected the request.
std::shared_ptr<HistogramVec> admission_latency(bool webhook) {
  static auto plugin_h = Registry::global().histogram(
      "apiserver_admission_controller_admission_duration_seconds", "in-process admission plugin latency",
      {"name", "operation", "type", "rejected"}, HistogramVec::exponential(0.00001, 2, 22));
  static auto webhook_h = Registry::global().histogram(
      "apiserver_admission_webhook_admission_duration_seconds", "admission webhook call latency (AdmissionReview round trip)",
      {"name", "operation", "type", "rejected"}, HistogramVec::exponential(0.0001, 2, 18));
  return webhook ? webhook_h : plugin_h;
}

ApiError ApiServer::run_admission(AdmissionAttrs& a, bool mutating) {
  std::vector<std::pair<std::string, AdmissionFn>> plugins;
  {
    std::lock_guard<std::mutex> g(mu_);
    plugins = mutating ? mutating_ : validating_;
  }
  const char* type = mutating ? "admit" : "validate";
  for (auto& p : plugins) {
    const double t0 = now_seconds();
    ApiError e = p.second(a);
    admission_latency(false)->observe({p.first, a.operation, type, e ? "true" : "false"}, now_seconds() - t0);
    if (e) {
      if (e.message.find("admission webhook") == std::string::npos && e.reason != "Forbidden")
        e.message = "admission webhook \"" + p.first + "\" denied the request: " + e.message;
      return e;
    }
  }
  return call_webhooks(a, mutating);
}

// ---- CRUD ------------------------------------------------------------------------------------------
void ApiServer::broadcast(std::shared_ptr<const ResourceInfo> res, const std::string& type, const Json& obj,
                          const Json* old_obj, int64_t rv) {
  // caller holds mu_
  const std::string rk = res->key();
  const std::string& ns = obj.str_at({"metadata", "namespace"});
  auto snap = std::make_shared<const Json>(obj);
  log_.push_back(LogEntry{rk, type, snap, rv});
  while (log_.size() > cfg_.watch_log_size) log_.pop_front();
  std::map<std::string, std::shared_ptr<const Json>> converted;  // served version -> snapshot
  int64_t drop = 0;
  bool dropping = take_fault("dropwatch", res->plural, &drop);
  for (auto it = watchers_.begin(); it != watchers_.end();) {
    auto w = it->lock();
    if (!w || w->closed()) {
      it = watchers_.erase(it);
      continue;
    }
    ++it;
    if (w->res_key_ != rk) continue;
    if (!w->ns_.empty() && w->ns_ != ns) continue;
    if (dropping) continue;
    bool now = w->labels_.matches(obj.at_path({"metadata", "labels"})) && w->fields_.matches(obj);
    bool before = old_obj && w->labels_.matches(old_obj->at_path({"metadata", "labels"})) && w->fields_.matches(*old_obj);
    std::string t = type;
    if (type == "MODIFIED") {
      if (now && !before) t = "ADDED";
      else if (!now && before) t = "DELETED";
      else if (!now && !before) continue;
    } else if (!now) {
      continue;
    }
    std::shared_ptr<const Json> out = snap;
    if (!w->version_.empty()) {
      auto& cv = converted[w->version_];
      if (!cv) {
        Json o = obj;
        convert_out(res, w->version_, o);
        cv = o == obj ? snap : std::make_shared<const Json>(std::move(o));
      }
      out = cv;
    }
    w->push(Watch::Item{t, std::move(out), rv});
  }
}

void ApiServer::commit_put(std::shared_ptr<const ResourceInfo> res, const std::string& key, Json& obj,
                           const std::string& type) {
  // caller holds mu_
  const std::string rk = res->key();
  auto& m = data_[rk];
  auto it = m.find(key);
  Json old;
  bool had = it != m.end();
  if (had) old = it->second;
  int64_t rv = ++rv_;
  obj["metadata"]["resourceVersion"] = std::to_string(rv);
  uid_index_[obj.str_at({"metadata", "uid"})] = rk + "|" + key;
  m[key] = obj;
  wal_append(Json{{"op", "put"}, {"r", rk}, {"id", key}, {"o", obj}, {"rv", rv}});
  broadcast(res, type, obj, had ? &old : nullptr, rv);
}

void ApiServer::commit_delete(std::shared_ptr<const ResourceInfo> res, const std::string& key) {
  // caller holds mu_
  const std::string rk = res->key();
  auto& m = data_[rk];
  auto it = m.find(key);
  if (it == m.end()) return;
  Json obj = it->second;
  m.erase(it);
  uid_index_.erase(obj.str_at({"metadata", "uid"}));
  int64_t rv = ++rv_;
  obj["metadata"]["resourceVersion"] = std::to_string(rv);
  wal_append(Json{{"op", "del"}, {"r", rk}, {"id", key}, {"rv", rv}});
  broadcast(res, "DELETED", obj, &obj, rv);
  if (res->is_crd == false && res->kind == "CustomResourceDefinition") reg_.remove_crd(obj);
  {
    std::lock_guard<std::mutex> g(bg_mu_);
    bg_kick_ = true;
  }
  bg_cv_.notify_all();
}

void ApiServer::post_commit(std::shared_ptr<const ResourceInfo> res, const std::string& type, const Json& obj) {
  if (res->kind == "CustomResourceDefinition" && type != "DELETED") {
    std::string err = reg_.add_crd(obj);
    Json st = obj;
    Json cond{{"type", "Established"}, {"status", err.empty() ? "True" : "False"},
              {"reason", err.empty() ? "InitialNamesAccepted" : "NotAccepted"}, {"message", err},
              {"lastTransitionTime", rfc3339_now()}};
    if (!obj.at_path({"status", "conditions"}).is_array()) {
      st["status"]["conditions"] = Json::array({cond});
      st["status"]["acceptedNames"] = obj.at_path({"spec", "names"});
      std::lock_guard<std::mutex> g(mu_);
      commit_put(res, object_key("", obj.str_at({"metadata", "name"})), st, "MODIFIED");
    }
  }
  if (res->kind == "ClusterRole") aggregate_clusterroles();
}

ApiError ApiServer::r_create(std::shared_ptr<const ResourceInfo> res, const std::string& version,
                             const std::string& ns_in, Json& obj, const WriteOptions& o) {
  double t0 = now_seconds();
  int64_t delay = 0;
  if (take_fault("delay", res->plural, &delay)) ::usleep(static_cast<useconds_t>(delay * 1000));
  if (take_fault("error", res->plural)) return ApiError::Internal("injected fault");
  if (!obj.is_object()) return ApiError::BadRequest("request body must be a JSON object");
  Json& md = obj["metadata"];
  if (!md.is_object()) md = Json::object();
  std::string ns = res->namespaced ? (ns_in.empty() ? md["namespace"].as_string() : ns_in) : "";
  if (res->namespaced && !md["namespace"].as_string().empty() && md["namespace"].as_string() != ns)
    return ApiError::BadRequest("the namespace of the provided object does not match the namespace sent on the request");
  if (res->namespaced) md["namespace"] = ns;
  else md.erase("namespace");
  if (md["name"].as_string().empty() && !md["generateName"].as_string().empty())
    md["name"] = md["generateName"].as_string() + random_alnum(5);
  ApiError err;
  if (!check_namespace(res, ns, true, err)) return err;
  const std::string& api_version = obj["apiVersion"].as_string();
  if (!api_version.empty() && version_of(api_version) != version && !res->serves(version_of(api_version)))
    return ApiError::BadRequest("apiVersion " + api_version + " is not served for " + res->plural);
  obj["apiVersion"] = res->api_version(version);
  obj["kind"] = res->kind;

  if (res->virtual_only) {
    // SubjectAccessReview & friends: evaluate, never store
    Json& spec = obj["spec"];
    if (res->kind == "TokenReview") {
      UserInfo tu;
      if (authenticate_token(spec["token"].as_string(), tu)) {
        Json groups = Json::array();
        for (const auto& g : tu.groups) groups.push_back(g);
        obj["status"] = Json{{"authenticated", true}, {"user", Json{{"username", tu.username}, {"groups", groups}}}};
      } else {
        obj["status"] = Json{{"authenticated", false}, {"error", "invalid bearer token"}};
      }
      spec.erase("token");  // never echo a credential back
      return {};
    }
    UserInfo u;
    if (res->kind == "SelfSubjectAccessReview") {
      u = o.user;
    } else {
      u.username = spec["user"].as_string();
      u.groups.clear();
      for (const auto& g : spec["groups"].as_array()) u.groups.push_back(g.as_string());
    }
    const Json& ra = spec["resourceAttributes"];
    std::string reason;
    bool allowed;
    if (ra.is_object()) {
      std::string resource = ra["resource"].as_string();
      allowed = authorize(u, ra["verb"].as_string(), ra["group"].as_string(), resource, ra["subresource"].as_string(),
                          ra["namespace"].as_string(), ra["name"].as_string(), &reason);
    } else {
      allowed = authorize(u, spec.at_path({"nonResourceAttributes", "verb"}).as_string(), "",
                          spec.at_path({"nonResourceAttributes", "path"}).as_string(), "", "", "", &reason);
    }
    obj["status"] = Json{{"allowed", allowed}, {"reason", reason}};
    return {};
  }

  if (ApiError se = structural(res, obj, o, true)) return se;
  apply_defaults(res, obj, true);
  AdmissionAttrs a;
  a.operation = "CREATE";
  a.res = res;
  a.ns = ns;
  a.name = md["name"].as_string();
  a.version = version;
  a.object = &obj;
  a.user = &o.user;
  a.dry_run = o.dry_run;
  // fires every admission completion hook on every exit path below
  struct DoneGuard {
    AdmissionAttrs& a;
    bool committed = false;
    ~DoneGuard() {
      for (auto& f : a.on_done) f(committed);
    }
  } done{a};
  err = run_admission(a, true);
  if (err) return err;
  apply_defaults(res, obj, false);  // mutating admission may add containers: default them too
  structural(res, obj, o, false);    // ... and fields a webhook added are pruned too (silently)
  to_storage(res, obj);
  obj["metadata"]["namespace"] = ns;
  if (!res->namespaced) obj["metadata"].erase("namespace");
  err = validate(res, obj, nullptr, "");
  if (err) return err;
  err = run_admission(a, false);
  if (err) return err;
  if (take_fault("commitdelay", res->plural, &delay)) ::usleep(static_cast<useconds_t>(delay * 1000));

  const std::string name = obj.str_at({"metadata", "name"});
  const std::string key = object_key(ns, name);
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& m = data_[res->key()];
    if (m.count(key)) return ApiError::AlreadyExists(res->plural + (res->group.empty() ? "" : "." + res->group), name);
    Json& md2 = obj["metadata"];
    md2["uid"] = uuid4();
    md2["creationTimestamp"] = rfc3339_now();
    md2["generation"] = 1;
    md2.erase("deletionTimestamp");
    md2.erase("resourceVersion");
    if (!o.dry_run) {
      commit_put(res, key, obj, "ADDED");
      done.committed = true;
    } else {
      obj["metadata"]["resourceVersion"] = std::to_string(rv_);
    }
  }
  if (!o.dry_run) post_commit(res, "ADDED", obj);
  convert_out(res, version, obj);
  req_counter()->inc({"create", res->plural, "201"});
  req_latency()->observe({"create", res->plural}, now_seconds() - t0);
  return {};
}

ApiError ApiServer::r_get(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                          const std::string& name, Json& out) {
  std::lock_guard<std::mutex> g(mu_);
  auto rit = data_.find(res->key());
  if (rit == data_.end()) return ApiError::NotFound(res->plural + (res->group.empty() ? "" : "." + res->group), name);
  auto it = rit->second.find(object_key(res->namespaced ? ns : "", name));
  if (it == rit->second.end()) return ApiError::NotFound(res->plural + (res->group.empty() ? "" : "." + res->group), name);
  out = it->second;
  convert_out(res, version, out);
  return {};
}

ApiError ApiServer::r_list(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                           const ListOptions& lo, Json& out) {
  LabelSelector ls;
  FieldSelector fs;
  std::string perr;
  if (!LabelSelector::parse(lo.label_selector, ls, &perr)) return ApiError::BadRequest(perr);
  if (!FieldSelector::parse(lo.field_selector, fs, &perr)) return ApiError::BadRequest(perr);
  Json items = Json::array();
  int64_t rv;
  std::string next_token;
  {
    std::lock_guard<std::mutex> g(mu_);
    rv = rv_;
    auto rit = data_.find(res->key());
    if (rit != data_.end()) {
      auto& m = rit->second;
      std::string prefix = res->namespaced && !ns.empty() ? ns + "/" : "";
      auto it = prefix.empty() ? m.begin() : m.lower_bound(prefix);
      if (!lo.continue_token.empty()) it = m.upper_bound(base64_decode(lo.continue_token));
      for (; it != m.end(); ++it) {
        if (!prefix.empty() && !starts_with(it->first, prefix)) break;
        if (!ls.matches(it->second.at_path({"metadata", "labels"})) || !fs.matches(it->second)) continue;
        if (lo.limit > 0 && static_cast<int64_t>(items.size()) >= lo.limit) {
          auto prev = it;
          --prev;
          next_token = base64_encode(prev->first);
          break;
        }
        Json o = it->second;
        convert_out(res, version, o);
        items.push_back(std::move(o));
      }
    }
  }
  out = Json{{"apiVersion", res->api_version(version.empty() ? res->storage_version : version)},
             {"kind", res->list_kind},
             {"metadata", Json{{"resourceVersion", std::to_string(rv)}}},
             {"items", items}};
  if (!next_token.empty()) out["metadata"]["continue"] = next_token;
  return {};
}

ApiError ApiServer::r_update(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns_in,
                             const std::string& name_in, Json& obj, const WriteOptions& o, const std::string& subresource) {
  double t0 = now_seconds();
  int64_t delay = 0;
  if (take_fault("delay", res->plural, &delay)) ::usleep(static_cast<useconds_t>(delay * 1000));
  if (take_fault("error", res->plural)) return ApiError::Internal("injected fault");
  if (take_fault("conflict", res->plural))
    return ApiError::Conflict("Operation cannot be fulfilled on " + res->plural + " \"" + name_in +
                              "\": the object has been modified; please apply your changes to the latest version and try again");
  if (!obj.is_object()) return ApiError::BadRequest("request body must be a JSON object");
  std::string ns = res->namespaced ? ns_in : "";
  std::string name = name_in.empty() ? obj.str_at({"metadata", "name"}) : name_in;
  if (!obj.str_at({"metadata", "name"}).empty() && obj.str_at({"metadata", "name"}) != name)
    return ApiError::BadRequest("the name of the object (" + obj.str_at({"metadata", "name"}) +
                                ") does not match the name on the URL (" + name + ")");
  if (subresource == "scale") {
    Json cur;
    ApiError e = r_get(res, "", ns, name, cur);
    if (e) return e;
    cur["spec"]["replicas"] = obj.at_path({"spec", "replicas"});
    Json out = cur;
    e = r_update(res, version, ns, name, out, o, "");
    if (e) return e;
    obj = Json{{"apiVersion", "autoscaling/v1"}, {"kind", "Scale"},
               {"metadata", Json{{"name", name}, {"namespace", ns}}},
               {"spec", Json{{"replicas", out.at_path({"spec", "replicas"})}}},
               {"status", Json{{"replicas", out.at_path({"status", "replicas"})}}}};
    return {};
  }
  const std::string key = object_key(ns, name);
  Json old;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& m = data_[res->key()];
    auto it = m.find(key);
    if (it == m.end()) return ApiError::NotFound(res->plural + (res->group.empty() ? "" : "." + res->group), name);
    old = it->second;
  }
  const std::string want_rv = obj.str_at({"metadata", "resourceVersion"});
  if (!want_rv.empty() && want_rv != old.str_at({"metadata", "resourceVersion"}))
    return ApiError::Conflict("Operation cannot be fulfilled on " + res->plural + (res->group.empty() ? "" : "." + res->group) +
                              " \"" + name + "\": the object has been modified; please apply your changes to the latest version and try again");
  Json next = obj;
  // status subresource semantics
  if (res->has_status) {
    if (subresource == "status") {
      Json s = obj["status"];
      next = old;
      next["status"] = s;
      // metadata changes through /status are limited to labels/annotations? k8s ignores them: keep old
    } else {
      if (old.has("status")) next["status"] = old["status"];
      else next.erase("status");
    }
  }
  // immutable metadata
  Json& md = next["metadata"];
  const Json& omd = old["metadata"];
  md["name"] = name;
  if (res->namespaced) md["namespace"] = ns;
  md["uid"] = omd["uid"];
  md["creationTimestamp"] = omd["creationTimestamp"];
  if (omd.has("deletionTimestamp")) {
    md["deletionTimestamp"] = omd["deletionTimestamp"];
    if (omd.has("deletionGracePeriodSeconds")) md["deletionGracePeriodSeconds"] = omd["deletionGracePeriodSeconds"];
  } else {
    md.erase("deletionTimestamp");
  }
  md["generation"] = omd["generation"].as_int(1);
  next["apiVersion"] = res->api_version(version);
  next["kind"] = res->kind;
  if (ApiError se = structural(res, next, o, subresource.empty())) return se;
  if (subresource.empty()) apply_defaults(res, next, false);

  AdmissionAttrs a;
  a.operation = "UPDATE";
  a.res = res;
  a.subresource = subresource;
  a.ns = ns;
  a.name = name;
  a.version = version;
  a.object = &next;
  a.old_object = &old;
  a.user = &o.user;
  a.dry_run = o.dry_run;
  ApiError err = run_admission(a, true);
  if (err) return err;
  if (subresource.empty()) apply_defaults(res, next, false);
  structural(res, next, o, false);
  to_storage(res, next);
  err = validate(res, next, &old, subresource);
  if (err) return err;
  err = run_admission(a, false);
  if (err) return err;
  if (subresource.empty() && spec_changed(old, next)) next["metadata"]["generation"] = omd["generation"].as_int(1) + 1;

  bool finalize = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& m = data_[res->key()];
    auto it = m.find(key);
    if (it == m.end()) return ApiError::NotFound(res->plural, name);
    if (it->second.str_at({"metadata", "resourceVersion"}) != old.str_at({"metadata", "resourceVersion"})) {
      if (!want_rv.empty())
        return ApiError::Conflict("Operation cannot be fulfilled on " + res->plural + " \"" + name +
                                  "\": the object has been modified; please apply your changes to the latest version and try again");
    }
    if (o.dry_run) {
      obj = next;
      convert_out(res, version, obj);
      return {};
    }
    if (next == it->second) {  // no-op update: no new resourceVersion, no event
      obj = it->second;
      convert_out(res, version, obj);
      return {};
    }
    finalize = next.at_path({"metadata", "deletionTimestamp"}).is_string() &&
               next.at_path({"metadata", "finalizers"}).empty() &&
               !(res->kind == "Pod" && res->group.empty() && next.at_path({"spec", "nodeName"}).is_string() &&
                 !next.at_path({"status", "phase"}).as_string().empty() &&
                 next.at_path({"status", "phase"}).as_string() != "Succeeded" &&
                 next.at_path({"status", "phase"}).as_string() != "Failed" &&
                 next.at_path({"metadata", "deletionGracePeriodSeconds"}).as_int(0) > 0);
    commit_put(res, key, next, "MODIFIED");
    if (finalize) {
      finalize_delete_locked(res, key);
    }
  }
  if (!finalize) post_commit(res, "MODIFIED", next);
  obj = next;
  convert_out(res, version, obj);
  req_counter()->inc({"update", res->plural, "200"});
  req_latency()->observe({"update", res->plural}, now_seconds() - t0);
  return {};
}

ApiError ApiServer::r_patch(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                            const std::string& name, const std::string& patch_type, const Json& patch, Json& out,
                            const WriteOptions& o, const std::string& subresource) {
  for (int attempt = 0; attempt < 5; ++attempt) {
    Json cur;
    ApiError e = r_get(res, version, ns, name, cur);
    if (e) return e;
    Json next;
    try {
      std::string pt = to_lower(patch_type);
      if (contains(pt, "json-patch")) next = apply_json_patch(cur, patch);
      else if (contains(pt, "strategic")) next = strategic_merge_patch(cur, patch);
      else next = merge_patch(cur, patch);
    } catch (const JsonError& je) {
      return ApiError{422, "Invalid", std::string("the server rejected our request due to an error in our request: ") + je.what()};
    }
    // the patch is applied against the current rv: keep it for optimistic concurrency unless the
    // patch itself pinned a resourceVersion
    if (!patch.is_object() || !patch.at_path({"metadata", "resourceVersion"}).is_string())
      next["metadata"]["resourceVersion"] = cur.str_at({"metadata", "resourceVersion"});
    e = r_update(res, version, ns, name, next, o, subresource);
    if (e.code == 409 && e.reason == "Conflict" &&
        !(patch.is_object() && patch.at_path({"metadata", "resourceVersion"}).is_string()))
      continue;
    if (e) return e;
    out = next;
    return {};
  }
  return ApiError::Conflict("patch retries exhausted for " + name);
}

ApiError ApiServer::finalize_delete_locked(std::shared_ptr<const ResourceInfo> res, const std::string& key) {
  commit_delete(res, key);
  return {};
}

ApiError ApiServer::r_delete(std::shared_ptr<const ResourceInfo> res, const std::string& ns_in, const std::string& name,
                             const DeleteOptions& o, Json* out) {
  if (take_fault("error", res->plural)) return ApiError::Internal("injected fault");
  std::string ns = res->namespaced ? ns_in : "";
  const std::string key = object_key(ns, name);
  Json cur;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& m = data_[res->key()];
    auto it = m.find(key);
    if (it == m.end()) return ApiError::NotFound(res->plural + (res->group.empty() ? "" : "." + res->group), name);
    cur = it->second;
  }
  if (!o.precondition_uid.empty() && o.precondition_uid != cur.str_at({"metadata", "uid"}))
    return ApiError::Conflict("Precondition failed: UID in precondition: " + o.precondition_uid);
  if (!o.precondition_rv.empty() && o.precondition_rv != cur.str_at({"metadata", "resourceVersion"}))
    return ApiError::Conflict("Precondition failed: ResourceVersion in precondition: " + o.precondition_rv);
  AdmissionAttrs a;
  a.operation = "DELETE";
  a.res = res;
  a.ns = ns;
  a.name = name;
  a.old_object = &cur;
  a.user = &o.user;
  a.dry_run = o.dry_run;
  ApiError err = run_admission(a, false);
  if (err) return err;
  if (o.dry_run) {
    if (out) *out = cur;
    return {};
  }
  std::string propagation = o.propagation;
  if (propagation.empty()) propagation = "Background";
  if (res->kind == "Namespace" && res->group.empty()) {
    std::lock_guard<std::mutex> g(mu_);
    auto& m = data_[res->key()];
    auto it = m.find(key);
    if (it == m.end()) return ApiError::NotFound("namespaces", name);
    Json next = it->second;
    if (!next.at_path({"metadata", "deletionTimestamp"}).is_string()) {
      next["metadata"]["deletionTimestamp"] = rfc3339_now();
      next["status"]["phase"] = "Terminating";
      commit_put(res, key, next, "MODIFIED");
    }
    if (out) *out = next;
    {
      std::lock_guard<std::mutex> g2(bg_mu_);
      bg_kick_ = true;
    }
    bg_cv_.notify_all();
    return {};
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& m = data_[res->key()];
    auto it = m.find(key);
    if (it == m.end()) return ApiError::NotFound(res->plural, name);
    Json next = it->second;
    Json& md = next["metadata"];
    bool already = md["deletionTimestamp"].is_string();
    if (propagation == "Foreground" || propagation == "Orphan") {
      const char* fin = propagation == "Foreground" ? "foregroundDeletion" : "orphan";
      bool has = false;
      for (const auto& f : md["finalizers"].as_array()) has = has || f.as_string() == fin;
      if (!has) md["finalizers"].push_back(fin);
    }
    int64_t grace = o.grace_seconds;
    bool graceful_pod = res->group.empty() && res->kind == "Pod" && next.at_path({"spec", "nodeName"}).is_string() &&
                        grace != 0 && next.at_path({"status", "phase"}).as_string() != "Succeeded" &&
                        next.at_path({"status", "phase"}).as_string() != "Failed";
    if (graceful_pod && grace < 0) grace = next.at_path({"spec", "terminationGracePeriodSeconds"}).as_int(30);
    if (!md["finalizers"].empty() || graceful_pod) {
      if (!already) {
        md["deletionTimestamp"] = rfc3339_now();
        md["deletionGracePeriodSeconds"] = graceful_pod ? grace : 0;
        commit_put(res, key, next, "MODIFIED");
      } else if (graceful_pod && grace < md["deletionGracePeriodSeconds"].as_int(30)) {
        md["deletionGracePeriodSeconds"] = grace;
        commit_put(res, key, next, "MODIFIED");
      }
      if (out) *out = next;
    } else {
      commit_delete(res, key);
      if (out) *out = cur;
    }
  }
  req_counter()->inc({"delete", res->plural, "200"});
  return {};
}

WatchPtr ApiServer::r_watch(std::shared_ptr<const ResourceInfo> res, const std::string& version, const std::string& ns,
                            const ListOptions& lo, ApiError* err) {
  auto w = std::make_shared<Watch>();
  w->res_ = res;
  w->res_key_ = res->key();
  w->ns_ = res->namespaced ? ns : "";
  w->version_ = version;
  std::string perr;
  if (!LabelSelector::parse(lo.label_selector, w->labels_, &perr) || !FieldSelector::parse(lo.field_selector, w->fields_, &perr)) {
    if (err) *err = ApiError::BadRequest(perr);
    return nullptr;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (lo.resource_version.empty() || lo.resource_version == "0") {
    auto rit = data_.find(res->key());
    if (rit != data_.end()) {
      for (const auto& kv : rit->second) {
        if (!w->ns_.empty() && !starts_with(kv.first, w->ns_ + "/")) continue;
        if (!w->labels_.matches(kv.second.at_path({"metadata", "labels"})) || !w->fields_.matches(kv.second)) continue;
        Json o = kv.second;
        convert_out(res, version, o);
        w->q_.push_back(Watch::Item{"ADDED", std::make_shared<const Json>(std::move(o)), rv_});
      }
    }
  } else {
    int64_t from = std::atoll(lo.resource_version.c_str());
    if (!log_.empty() && log_.front().rv > from + 1 && from < rv_) {
      // events between `from` and the oldest retained one are gone
      bool covered = false;
      for (const auto& e : log_)
        if (e.rv == from + 1) covered = true;
      if (!covered) {
        if (err) *err = ApiError{410, "Expired", "too old resource version: " + lo.resource_version + " (" + std::to_string(log_.front().rv) + ")"};
        return nullptr;
      }
    }
    for (const auto& e : log_) {
      if (e.res_key != w->res_key_ || e.rv <= from) continue;
      const Json& obj = *e.obj;
      if (!w->ns_.empty() && obj.str_at({"metadata", "namespace"}) != w->ns_) continue;
      if (!w->labels_.matches(obj.at_path({"metadata", "labels"})) || !w->fields_.matches(obj)) continue;
      Json o = obj;
      convert_out(res, version, o);
      w->q_.push_back(Watch::Item{e.type, std::make_shared<const Json>(std::move(o)), e.rv});
    }
  }
  watchers_.push_back(w);
  return w;
}

// ---- typed helpers -------------------------------------------------------------------------------
namespace {
std::string ver(const std::string& api_version) { return version_of(api_version); }
}  // namespace

ApiError ApiServer::create(Json& obj, const WriteOptions& o) {
  auto res = reg_.by_kind(obj["apiVersion"].as_string(), obj["kind"].as_string());
  if (!res) return ApiError::NotFound("kind", obj["apiVersion"].as_string() + "/" + obj["kind"].as_string());
  return r_create(res, ver(obj["apiVersion"].as_string()), obj.str_at({"metadata", "namespace"}), obj, o);
}
ApiError ApiServer::get(const std::string& api_version, const std::string& kind, const std::string& ns,
                        const std::string& name, Json& out) {
  auto res = reg_.by_kind(api_version, kind);
  if (!res) return ApiError::NotFound("kind", api_version + "/" + kind);
  return r_get(res, ver(api_version), ns, name, out);
}
ApiError ApiServer::list(const std::string& api_version, const std::string& kind, const std::string& ns,
                         const ListOptions& lo, Json& out) {
  auto res = reg_.by_kind(api_version, kind);
  if (!res) return ApiError::NotFound("kind", api_version + "/" + kind);
  return r_list(res, ver(api_version), ns, lo, out);
}
ApiError ApiServer::update(Json& obj, const WriteOptions& o) {
  auto res = reg_.by_kind(obj["apiVersion"].as_string(), obj["kind"].as_string());
  if (!res) return ApiError::NotFound("kind", obj["kind"].as_string());
  return r_update(res, ver(obj["apiVersion"].as_string()), obj.str_at({"metadata", "namespace"}),
                  obj.str_at({"metadata", "name"}), obj, o, "");
}
ApiError ApiServer::update_status(Json& obj, const WriteOptions& o) {
  auto res = reg_.by_kind(obj["apiVersion"].as_string(), obj["kind"].as_string());
  if (!res) return ApiError::NotFound("kind", obj["kind"].as_string());
  return r_update(res, ver(obj["apiVersion"].as_string()), obj.str_at({"metadata", "namespace"}),
                  obj.str_at({"metadata", "name"}), obj, o, res->has_status ? "status" : "");
}
ApiError ApiServer::patch(const std::string& api_version, const std::string& kind, const std::string& ns,
                          const std::string& name, const std::string& patch_type, const Json& p, Json& out,
                          const WriteOptions& o, const std::string& subresource) {
  auto res = reg_.by_kind(api_version, kind);
  if (!res) return ApiError::NotFound("kind", kind);
  return r_patch(res, ver(api_version), ns, name, patch_type, p, out, o, subresource);
}
ApiError ApiServer::remove(const std::string& api_version, const std::string& kind, const std::string& ns,
                           const std::string& name, const DeleteOptions& o) {
  auto res = reg_.by_kind(api_version, kind);
  if (!res) return ApiError::NotFound("kind", kind);
  return r_delete(res, ns, name, o);
}
WatchPtr ApiServer::watch(const std::string& api_version, const std::string& kind, const std::string& ns,
                          const ListOptions& lo, ApiError* err) {
  auto res = reg_.by_kind(api_version, kind);
  if (!res) {
    if (err) *err = ApiError::NotFound("kind", kind);
    return nullptr;
  }
  return r_watch(res, ver(api_version), ns, lo, err);
}

}  // namespace kf
