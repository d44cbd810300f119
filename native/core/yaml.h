// yaml.h — YAML (block/flow subset used by Kubernetes manifests) -> Json.
//
// Supported: block mappings and sequences (incl. "- key: v" items and compact nesting), plain /
// single- / double-quoted scalars, literal `|` and folded `>` block scalars (with -/+ chomping),
// flow sequences / mappings, comments, multi-document streams (`---`), int / float / bool / null
// resolution (YAML 1.2 core schema). Not supported: anchors/aliases, tags, complex keys.
#pragma once

#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

bool parse_yaml(const std::string& text, Json& out, std::string* err = nullptr);            // first document
bool parse_yaml_all(const std::string& text, std::vector<Json>& docs, std::string* err = nullptr);
std::string dump_yaml(const Json& v);

}  // namespace kf
