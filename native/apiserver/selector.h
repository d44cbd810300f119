// selector.h — Kubernetes label selectors (string and LabelSelector-object forms) and field
// selectors. Used by the API server (list/watch), the controllers (PodDefault matching, Service
// endpoints, RWO PVC scheduling) and the kubelet.
#pragma once

#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

struct Requirement {
  enum class Op { Eq, NotEq, In, NotIn, Exists, DoesNotExist, Gt, Lt } op = Op::Eq;
  std::string key;
  std::vector<std::string> values;
};

class LabelSelector {
 public:
  LabelSelector() = default;  // matches everything
  static bool parse(const std::string& s, LabelSelector& out, std::string* err = nullptr);
  // metav1.LabelSelector {matchLabels, matchExpressions}. A null/absent selector object
  // matches nothing when `null_matches_nothing` (PodDefault semantics), else everything.
  static LabelSelector from_json(const Json& sel, bool null_matches_nothing = false);
  bool matches(const Json& labels) const;
  bool empty() const { return reqs_.empty() && !nothing_; }
  std::string str() const;

 private:
  std::vector<Requirement> reqs_;
  bool nothing_ = false;
};

class FieldSelector {
 public:
  static bool parse(const std::string& s, FieldSelector& out, std::string* err = nullptr);
  bool matches(const Json& obj) const;
  bool empty() const { return terms_.empty(); }

 private:
  struct Term {
    std::vector<std::string> path;
    std::string value;
    bool neq = false;
  };
  std::vector<Term> terms_;
};

// Node-affinity style matchExpressions over a label map (In/NotIn/Exists/DoesNotExist/Gt/Lt).
bool match_node_selector_term(const Json& term, const Json& node);

}  // namespace kf
