// resources.h — container resource requirements with kube-apiserver's rules, and the ONE normalized
// GPU count that ResourceQuota admission, the scheduler and the device plugin all charge.
//
// kube-apiserver (pkg/apis/core/validation ValidateResourceRequirements) gives the reference its
// guarantees for free; kube-lite has to provide them itself:
//   * every quantity parses under resource.Quantity's grammar and is >= 0;
//   * extended resources (amd.com/gpu, amd.com/gpu-memory, any non-kubernetes.io domain) are
//     integers, cannot be overcommitted (requests == limits) and need a limit when requested;
//   * for cpu / memory requests <= limits.
// Pod defaulting (SetDefaults_Pod) copies each limit without a request into requests, so after
// admission `requests` is the single source of truth. The reference depends on this: the spawner
// sets limits only (crud-web-apps/jupyter/backend/apps/common/form.py:247-250) while tenant quotas are
// written on requests (profile-controller/config/samples/_v1beta1_profile.yaml:13).
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

// cpu, memory, ephemeral-storage, hugepages-*, storage and anything under kubernetes.io
bool is_native_resource(const std::string& name);
// fully-qualified, not in the kubernetes.io domain, not a quota "requests." key
bool is_extended_resource(const std::string& name);

// canonical rendering the API server uses in messages ("0.5" -> "500m", "2" -> "2")
std::string canonical_quantity(const Json& q);

// Errors in kube-apiserver's wording for one container's `resources` at `path`
// (e.g. "spec.containers[0].resources"). Two lists: unparsable quantities (the API server
// refuses those at decode time, 400 BadRequest) and field errors (422 Invalid).
struct ResourceErrors {
  std::vector<std::string> decode;
  std::vector<std::string> invalid;
  bool empty() const { return decode.empty() && invalid.empty(); }
};
void validate_resource_requirements(const Json& resources, const std::string& path, ResourceErrors& out);
// every container, init container and ephemeral container of a PodSpec at `path` ("spec" or
// "spec.template.spec")
void validate_pod_spec_resources(const Json& spec, const std::string& path, ResourceErrors& out);

// SetDefaults_Pod: each limit without a request becomes the request too
void default_requests_from_limits(Json& pod_spec);

// The amount of `resource` a container asks for: its request, else its limit (identical after
// admission for extended resources). nullopt when the value does not parse or is not a
// non-negative integer (the device plugin must fail on that, never allocate 0).
std::optional<int64_t> container_integer_request(const Json& container, const std::string& resource);

// Whole GPUs the device plugin allocates for a pod: sum over app containers, max with each
// non-sidecar init container (restartable sidecars add to the app sum, as in the Kubernetes
// sidecar KEP). nullopt on an unparsable / non-integer count.
std::optional<int64_t> pod_gpu_count(const Json& pod, const std::string& resource = "amd.com/gpu");

}  // namespace kf
