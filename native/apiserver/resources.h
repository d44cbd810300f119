// resources.h — the API server's type registry: built-in Kubernetes resources plus the
// CustomResourceDefinitions of this framework (Notebook, Profile, Tensorboard, PVCViewer,
// PodDefault) and the third-party kinds the reconcilers own (Istio VirtualService /
// AuthorizationPolicy, OpenShift Route / ImageStream).
//
// CRDs are real `apiextensions.k8s.io/v1` objects: the built-in ones are generated here
// (equivalent of the reference's config/crd/bases/*.yaml) and created at bootstrap, and any CRD
// created later through the API registers a new resource dynamically. Multi-version CRDs use the
// "None" conversion strategy (apiVersion rewrite), which is what the reference configures for
// Notebook (notebook-controller/config/crd/patches/trivial_conversion_patch.yaml).
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

struct ResourceInfo {
  std::string group;  // "" for core
  std::vector<std::string> versions;
  std::string storage_version;
  std::string kind, list_kind, plural, singular;
  std::vector<std::string> short_names;
  std::vector<std::string> categories;
  bool namespaced = true;
  bool has_status = false;
  bool has_scale = false;
  bool virtual_only = false;  // e.g. SubjectAccessReview: create-only, never stored
  bool is_crd = false;
  // OpenAPI v3 schema per version (CRDs); null = no structural validation
  std::map<std::string, Json> schemas;

  std::string key() const { return group + "/" + plural; }
  std::string api_version(const std::string& v) const { return group.empty() ? v : group + "/" + v; }
  std::string storage_api_version() const { return api_version(storage_version); }
  bool serves(const std::string& v) const;
};

class ResourceRegistry {
 public:
  ResourceRegistry();
  std::shared_ptr<const ResourceInfo> by_plural(const std::string& group, const std::string& plural) const;
  std::shared_ptr<const ResourceInfo> by_kind(const std::string& api_version, const std::string& kind) const;
  std::shared_ptr<const ResourceInfo> by_kind_any(const std::string& kind) const;
  std::vector<std::shared_ptr<const ResourceInfo>> all() const;
  void add(std::shared_ptr<ResourceInfo> r);
  // Registers (or updates) a resource from a CustomResourceDefinition object.
  std::string add_crd(const Json& crd);
  void remove_crd(const Json& crd);

 private:
  mutable std::mutex mu_;
  std::map<std::string, std::shared_ptr<ResourceInfo>> by_key_;
};

// Built-in CRD objects of this framework (Notebook v1/v1beta1/v1alpha1, Profile v1/v1beta1,
// Tensorboard, PVCViewer, PodDefault) and the third-party kinds (Istio, OpenShift, app.k8s.io).
std::vector<Json> builtin_crds();
// Process-wide registry of the built-in kinds + built-in CRDs (for components that need
// ResourceInfo without an embedded API server, e.g. webhook self-registration).
const ResourceRegistry& builtin_registry();

// Minimal structural OpenAPI v3 validation (type, required, properties, items, minItems,
// maxItems, enum, minimum, maximum, pattern-free). Returns error strings (empty = valid).
std::vector<std::string> validate_schema(const Json& schema, const Json& value, const std::string& path = "");

}  // namespace kf
