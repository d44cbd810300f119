// resources.cc — see resources.h.
#include "apiserver/resources.h"

#include <climits>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <regex>

#include "apiserver/schemas.h"
#include "core/util.h"

namespace kf {

bool ResourceInfo::serves(const std::string& v) const {
  for (const auto& x : versions)
    if (x == v) return true;
  return false;
}

namespace {
std::shared_ptr<ResourceInfo> R(const std::string& group, const std::vector<std::string>& versions,
                                const std::string& kind, const std::string& plural, bool namespaced,
                                bool status, std::vector<std::string> shorts = {}) {
  auto r = std::make_shared<ResourceInfo>();
  r->group = group;
  r->versions = versions;
  r->storage_version = versions.front();
  r->kind = kind;
  r->list_kind = kind + "List";
  r->plural = plural;
  r->singular = to_lower(kind);
  r->namespaced = namespaced;
  r->has_status = status;
  r->short_names = std::move(shorts);
  return r;
}
}  // namespace

ResourceRegistry::ResourceRegistry() {
  // core/v1
  add(R("", {"v1"}, "Namespace", "namespaces", false, true, {"ns"}));
  add(R("", {"v1"}, "Pod", "pods", true, true, {"po"}));
  add(R("", {"v1"}, "Service", "services", true, true, {"svc"}));
  add(R("", {"v1"}, "Endpoints", "endpoints", true, false, {"ep"}));
  add(R("", {"v1"}, "ConfigMap", "configmaps", true, false, {"cm"}));
  add(R("", {"v1"}, "Secret", "secrets", true, false));
  add(R("", {"v1"}, "ServiceAccount", "serviceaccounts", true, false, {"sa"}));
  add(R("", {"v1"}, "Event", "events", true, false, {"ev"}));
  add(R("", {"v1"}, "PersistentVolumeClaim", "persistentvolumeclaims", true, true, {"pvc"}));
  add(R("", {"v1"}, "PersistentVolume", "persistentvolumes", false, true, {"pv"}));
  add(R("", {"v1"}, "Node", "nodes", false, true, {"no"}));
  add(R("", {"v1"}, "ResourceQuota", "resourcequotas", true, true, {"quota"}));
  add(R("", {"v1"}, "LimitRange", "limitranges", true, false, {"limits"}));
  // apps/v1
  {
    auto sts = R("apps", {"v1"}, "StatefulSet", "statefulsets", true, true, {"sts"});
    sts->has_scale = true;
    add(sts);
    auto dep = R("apps", {"v1"}, "Deployment", "deployments", true, true, {"deploy"});
    dep->has_scale = true;
    add(dep);
    auto rs = R("apps", {"v1"}, "ReplicaSet", "replicasets", true, true, {"rs"});
    rs->has_scale = true;
    add(rs);
    add(R("apps", {"v1"}, "ControllerRevision", "controllerrevisions", true, false));
  }
  // rbac
  add(R("rbac.authorization.k8s.io", {"v1"}, "Role", "roles", true, false));
  add(R("rbac.authorization.k8s.io", {"v1"}, "RoleBinding", "rolebindings", true, false));
  add(R("rbac.authorization.k8s.io", {"v1"}, "ClusterRole", "clusterroles", false, false));
  add(R("rbac.authorization.k8s.io", {"v1"}, "ClusterRoleBinding", "clusterrolebindings", false, false));
  // networking / storage / coordination / admission / apiextensions
  add(R("networking.k8s.io", {"v1"}, "NetworkPolicy", "networkpolicies", true, false, {"netpol"}));
  add(R("networking.k8s.io", {"v1"}, "Ingress", "ingresses", true, true, {"ing"}));
  add(R("storage.k8s.io", {"v1"}, "StorageClass", "storageclasses", false, false, {"sc"}));
  add(R("coordination.k8s.io", {"v1"}, "Lease", "leases", true, false));
  add(R("admissionregistration.k8s.io", {"v1"}, "MutatingWebhookConfiguration", "mutatingwebhookconfigurations", false, false));
  add(R("admissionregistration.k8s.io", {"v1"}, "ValidatingWebhookConfiguration", "validatingwebhookconfigurations", false, false));
  add(R("apiextensions.k8s.io", {"v1"}, "CustomResourceDefinition", "customresourcedefinitions", false, true, {"crd", "crds"}));
  {
    auto sar = R("authorization.k8s.io", {"v1"}, "SubjectAccessReview", "subjectaccessreviews", false, true);
    sar->virtual_only = true;
    add(sar);
    auto ssar = R("authorization.k8s.io", {"v1"}, "SelfSubjectAccessReview", "selfsubjectaccessreviews", false, true);
    ssar->virtual_only = true;
    add(ssar);
    // bearer-token authentication as a service (the gateway's authn, SURVEY L5 / VERDICT r3 item 2)
    auto tr = R("authentication.k8s.io", {"v1"}, "TokenReview", "tokenreviews", false, true);
    tr->virtual_only = true;
    add(tr);
  }
}

void ResourceRegistry::add(std::shared_ptr<ResourceInfo> r) {
  std::lock_guard<std::mutex> g(mu_);
  by_key_[r->key()] = std::move(r);
}

std::shared_ptr<const ResourceInfo> ResourceRegistry::by_plural(const std::string& group, const std::string& plural) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = by_key_.find(group + "/" + plural);
  if (it != by_key_.end()) return it->second;
  // allow singular / short names (kubectl-style)
  for (const auto& kv : by_key_) {
    const auto& r = kv.second;
    if (r->group != group) continue;
    if (r->singular == plural) return r;
    for (const auto& s : r->short_names)
      if (s == plural) return r;
  }
  return nullptr;
}

std::shared_ptr<const ResourceInfo> ResourceRegistry::by_kind(const std::string& api_version, const std::string& kind) const {
  std::string group, version = api_version;
  size_t slash = api_version.find('/');
  if (slash != std::string::npos) {
    group = api_version.substr(0, slash);
    version = api_version.substr(slash + 1);
  }
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& kv : by_key_)
    if (kv.second->group == group && kv.second->kind == kind && kv.second->serves(version)) return kv.second;
  return nullptr;
}

std::shared_ptr<const ResourceInfo> ResourceRegistry::by_kind_any(const std::string& kind) const {
  std::lock_guard<std::mutex> g(mu_);
  std::string lk = to_lower(kind);
  for (const auto& kv : by_key_) {
    const auto& r = kv.second;
    if (to_lower(r->kind) == lk || r->plural == lk || r->singular == lk) return r;
    for (const auto& s : r->short_names)
      if (s == lk) return r;
  }
  return nullptr;
}

std::vector<std::shared_ptr<const ResourceInfo>> ResourceRegistry::all() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::shared_ptr<const ResourceInfo>> out;
  for (const auto& kv : by_key_) out.push_back(kv.second);
  return out;
}

std::string ResourceRegistry::add_crd(const Json& crd) {
  const Json& spec = crd["spec"];
  auto r = std::make_shared<ResourceInfo>();
  r->is_crd = true;
  r->group = spec["group"].as_string();
  r->kind = spec.at_path({"names", "kind"}).as_string();
  r->plural = spec.at_path({"names", "plural"}).as_string();
  r->singular = spec.at_path({"names", "singular"}).as_string_or(to_lower(r->kind));
  r->list_kind = spec.at_path({"names", "listKind"}).as_string_or(r->kind + "List");
  for (const auto& s : spec.at_path({"names", "shortNames"}).as_array()) r->short_names.push_back(s.as_string());
  for (const auto& s : spec.at_path({"names", "categories"}).as_array()) r->categories.push_back(s.as_string());
  r->namespaced = spec["scope"].as_string() != "Cluster";
  if (r->group.empty() || r->kind.empty() || r->plural.empty()) return "spec.group, spec.names.kind and spec.names.plural are required";
  int storage_count = 0;
  for (const auto& v : spec["versions"].as_array()) {
    if (!v["served"].as_bool(true)) continue;
    const std::string name = v["name"].as_string();
    r->versions.push_back(name);
    if (v["storage"].as_bool()) {
      r->storage_version = name;
      storage_count++;
    }
    if (v.at_path({"subresources", "status"}).is_object()) r->has_status = true;
    if (v.at_path({"subresources", "scale"}).is_object()) r->has_scale = true;
    if (v.at_path({"schema", "openAPIV3Schema"}).is_object()) r->schemas[name] = v.at_path({"schema", "openAPIV3Schema"});
  }
  if (r->versions.empty()) return "at least one served version is required";
  if (storage_count != 1) return "exactly one version must be the storage version";
  add(r);
  return "";
}

void ResourceRegistry::remove_crd(const Json& crd) {
  const Json& spec = crd["spec"];
  std::lock_guard<std::mutex> g(mu_);
  by_key_.erase(spec["group"].as_string() + "/" + spec.at_path({"names", "plural"}).as_string());
}

// ---------------------------------------------------------------------------------------------
namespace {
const char* json_type_name(const Json& v) {
  if (v.is_null()) return "null";
  if (v.is_bool()) return "boolean";
  if (v.is_int()) return "integer";
  if (v.is_number()) return "number";
  if (v.is_string()) return "string";
  if (v.is_array()) return "array";
  return "object";
}

// `pattern` as kube-apiserver evaluates it (ECMA-262 regex), compiled once per pattern; the
// Quantity pattern is checked with the Quantity parser itself
bool matches_pattern(const std::string& pattern, const std::string& s) {
  if (pattern == kQuantityPattern) return parse_quantity(s).has_value() && s == trim(s);
  static std::mutex mu;
  static std::map<std::string, std::shared_ptr<const std::regex>> cache;
  std::shared_ptr<const std::regex> re;
  {
    std::lock_guard<std::mutex> g(mu);
    auto& slot = cache[pattern];
    if (!slot) {
      try {
        slot = std::make_shared<const std::regex>(pattern, std::regex::ECMAScript);
      } catch (const std::regex_error&) {
        slot = std::make_shared<const std::regex>(".*");  // an invalid pattern never rejects
      }
    }
    re = slot;
  }
  return std::regex_search(s, *re);
}
}  // namespace

// OpenAPI v3 validation with kube-apiserver's messages ("<path> in body must be of type integer:
// \"string\"", "should match '<pattern>'", "Unsupported value", "Required value")
std::vector<std::string> validate_schema(const Json& schema, const Json& value, const std::string& path) {
  std::vector<std::string> errs;
  if (!schema.is_object()) return errs;
  const std::string here = path.empty() ? "<root>" : path;
  if (value.is_null() && schema["nullable"].as_bool()) return errs;
  auto type_error = [&](const std::string& want) {
    errs.push_back(here + ": Invalid value: \"" + json_type_name(value) + "\": " + here + " in body must be of type " + want +
                   ": \"" + json_type_name(value) + "\"");
  };
  const bool int_or_string = schema["x-kubernetes-int-or-string"].as_bool();
  const std::string& type = schema["type"].as_string();
  if (int_or_string) {
    if (!value.is_int() && !value.is_string()) {
      type_error("integer or string");
      return errs;
    }
  } else if (!type.empty()) {
    bool ok = true;
    if (type == "object") ok = value.is_object();
    else if (type == "array") ok = value.is_array();
    else if (type == "string") ok = value.is_string();
    else if (type == "integer") ok = value.is_int();
    else if (type == "number") ok = value.is_number();
    else if (type == "boolean") ok = value.is_bool();
    if (!ok) {
      type_error(type);
      return errs;
    }
  }
  if (value.is_int()) {
    const std::string& fmt = schema["format"].as_string();
    const int64_t v = value.as_int();
    if (fmt == "int32" && (v < INT32_MIN || v > INT32_MAX))
      errs.push_back(here + ": Invalid value: " + value.dump() + ": " + here + " in body must be of type int32: \"" + value.dump() + "\"");
  }
  if (value.is_string() && schema["pattern"].is_string() && !matches_pattern(schema["pattern"].as_string(), value.as_string()))
    errs.push_back(here + ": Invalid value: \"" + value.as_string() + "\": " + here + " in body should match '" +
                   schema["pattern"].as_string() + "'");
  if (schema.has("enum")) {
    bool found = false;
    std::vector<std::string> allowed;
    for (const auto& e : schema["enum"].as_array()) {
      found = found || e == value;
      allowed.push_back(e.dump());
    }
    if (!found) errs.push_back(here + ": Unsupported value: " + value.dump() + ": supported values: " + join(allowed, ", "));
  }
  if (value.is_number()) {
    if (schema.has("minimum") && value.as_double() < schema["minimum"].as_double())
      errs.push_back(here + ": Invalid value: " + value.dump() + ": " + here + " in body should be greater than or equal to " +
                     schema["minimum"].dump());
    if (schema.has("maximum") && value.as_double() > schema["maximum"].as_double())
      errs.push_back(here + ": Invalid value: " + value.dump() + ": " + here + " in body should be less than or equal to " +
                     schema["maximum"].dump());
  }
  if (value.is_object()) {
    for (const auto& req : schema["required"].as_array())
      if (!value.has(req.as_string())) errs.push_back((path.empty() ? req.as_string() : here + "." + req.as_string()) + ": Required value");
    const Json& props = schema["properties"];
    for (const auto& m : value.as_object()) {
      if (path.empty() && m.first == "metadata") continue;
      const Json* ps = props.find(m.first);
      std::string sub = path.empty() ? m.first : path + "." + m.first;
      const Json* sch = ps ? ps : (schema["additionalProperties"].is_object() ? &schema["additionalProperties"] : nullptr);
      if (!sch) continue;
      auto e = validate_schema(*sch, m.second, sub);
      errs.insert(errs.end(), e.begin(), e.end());
    }
  }
  if (value.is_array()) {
    if (schema.has("minItems") && static_cast<int64_t>(value.size()) < schema["minItems"].as_int())
      errs.push_back(here + ": Invalid value: " + std::to_string(value.size()) + ": " + here + " in body should have at least " +
                     std::to_string(schema["minItems"].as_int()) + " items");
    if (schema.has("maxItems") && static_cast<int64_t>(value.size()) > schema["maxItems"].as_int())
      errs.push_back(here + ": Too many: " + std::to_string(value.size()) + ": must have at most " +
                     std::to_string(schema["maxItems"].as_int()) + " items");
    if (schema["items"].is_object()) {
      for (size_t i = 0; i < value.size(); ++i) {
        auto e = validate_schema(schema["items"], value[i], path + "[" + std::to_string(i) + "]");
        errs.insert(errs.end(), e.begin(), e.end());
      }
    }
  }
  return errs;
}

// ---------------------------------------------------------------------------------------------
namespace {
Json crd(const std::string& group, const std::string& kind, const std::string& plural, const std::string& scope,
         const std::vector<std::pair<std::string, bool>>& versions, bool status, const Json& schema,
         std::vector<std::string> shorts = {}, std::vector<std::string> categories = {}) {
  Json vs = Json::array();
  for (const auto& v : versions) {
    Json ver{{"name", v.first}, {"served", true}, {"storage", v.second}};
    if (status) ver["subresources"] = Json{{"status", Json::object()}};
    if (schema.is_object()) ver["schema"] = Json{{"openAPIV3Schema", schema}};
    vs.push_back(ver);
  }
  Json names{{"kind", kind}, {"listKind", kind + "List"}, {"plural", plural}, {"singular", to_lower(kind)}};
  if (!shorts.empty()) {
    Json a = Json::array();
    for (auto& s : shorts) a.push_back(s);
    names["shortNames"] = a;
  }
  if (!categories.empty()) {
    Json a = Json::array();
    for (auto& s : categories) a.push_back(s);
    names["categories"] = a;
  }
  return Json{{"apiVersion", "apiextensions.k8s.io/v1"},
              {"kind", "CustomResourceDefinition"},
              {"metadata", Json{{"name", plural + "." + group}}},
              {"spec", Json{{"group", group}, {"names", names}, {"scope", scope}, {"versions", vs},
                            {"conversion", Json{{"strategy", "None"}}}}}};
}
}  // namespace

std::vector<Json> builtin_crds() {
  std::vector<Json> out;
  // Structural schemas (apiserver/schemas.cc): full core/v1 PodSpec under Notebook
  // spec.template.spec (all three versions, storage v1) and PVCViewer spec.podSpec, the PodDefault
  // merge fields, Profile owner / plugins / quota, Tensorboard logspath; unknown fields are pruned.
  out.push_back(crd("kubeflow.org", "Notebook", "notebooks", "Namespaced",
                    {{"v1", true}, {"v1alpha1", false}, {"v1beta1", false}}, true, notebook_schema(), {}, {"kubeflow"}));
  out.push_back(crd("kubeflow.org", "Profile", "profiles", "Cluster", {{"v1", true}, {"v1beta1", false}}, true, profile_schema()));
  out.push_back(crd("tensorboard.kubeflow.org", "Tensorboard", "tensorboards", "Namespaced", {{"v1alpha1", true}}, true,
                    tensorboard_schema()));
  out.push_back(crd("kubeflow.org", "PVCViewer", "pvcviewers", "Namespaced", {{"v1alpha1", true}}, true, pvcviewer_schema()));
  out.push_back(crd("kubeflow.org", "PodDefault", "poddefaults", "Namespaced", {{"v1alpha1", true}}, false, poddefault_schema()));
  // Istio (what the reconcilers own / create)
  out.push_back(crd("networking.istio.io", "VirtualService", "virtualservices", "Namespaced",
                    {{"v1alpha3", true}, {"v1beta1", false}, {"v1", false}}, true, Json(), {"vs"}));
  out.push_back(crd("networking.istio.io", "Gateway", "gateways", "Namespaced", {{"v1beta1", true}, {"v1alpha3", false}}, true, Json()));
  out.push_back(crd("security.istio.io", "AuthorizationPolicy", "authorizationpolicies", "Namespaced",
                    {{"v1beta1", true}, {"v1", false}}, true, Json()));
  // OpenShift kinds used by the platform-extension reconciler and webhook
  out.push_back(crd("route.openshift.io", "Route", "routes", "Namespaced", {{"v1", true}}, true, Json()));
  out.push_back(crd("image.openshift.io", "ImageStream", "imagestreams", "Namespaced", {{"v1", true}}, true, Json(), {"is"}));
  // app.k8s.io Application (dashboard reads the platform version from it)
  out.push_back(crd("app.k8s.io", "Application", "applications", "Namespaced", {{"v1beta1", true}}, true, Json()));
  return out;
}

const ResourceRegistry& builtin_registry() {
  static ResourceRegistry* r = [] {
    auto* reg = new ResourceRegistry();
    for (const auto& crd : builtin_crds()) reg->add_crd(crd);
    return reg;
  }();
  return *r;
}

}  // namespace kf
