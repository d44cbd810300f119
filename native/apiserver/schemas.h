// schemas.h — structural OpenAPI v3 schemas for the kubeflow CRDs, built in C++ from one set of
// core/v1 type schemas (PodSpec, Container, Volume, Probe, ...), plus kube-apiserver's structural
// semantics over them: pruning of unknown fields, defaulting from `default`, and type / format /
// pattern / enum validation (ResourceRegistry CRDs use these; apiserver.cc applies them).
//
// Parity: the reference ships controller-gen output —
//   notebook-controller/config/crd/bases/kubeflow.org_notebooks.yaml     (PodSpec under spec.template.spec, 3 versions)
//   pvcviewer-controller/config/crd/bases/kubeflow.org_pvcviewers.yaml   (PodSpec under spec.podSpec)
//   admission-webhook/manifests/base/crd.yaml                            (PodDefault: env, volumes, sidecars, ...)
//   profile-controller/config/crd/bases/kubeflow.org_profiles.yaml
//   tensorboard-controller/config/crd/bases/tensorboard.kubeflow.org_tensorboards.yaml
// tests/test_crd_schemas.py checks that every property path of those files exists here with the
// same type. Descriptions are omitted (they are documentation, not behaviour).
#pragma once

#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

Json pod_spec_schema();  // core/v1 PodSpec
Json notebook_schema();
Json pvcviewer_schema();
Json poddefault_schema();
Json profile_schema();
Json tensorboard_schema();

// The resource.Quantity pattern controller-gen emits for every Quantity field
extern const char* const kQuantityPattern;

// kube-apiserver's pruning: drop every field the structural schema does not specify (unless under
// x-kubernetes-preserve-unknown-fields), recording each dropped path ("spec.foo",
// "spec.template.spec.containers[0].resourcez"). apiVersion / kind / metadata are kept at the root.
void prune_unknown_fields(const Json& schema, Json& value, std::vector<std::string>* pruned, const std::string& path = "");
// structural defaulting: fill `default` of absent properties of present objects
void apply_schema_defaults(const Json& schema, Json& value);

}  // namespace kf
