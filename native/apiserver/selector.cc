// selector.cc — see selector.h.
#include "apiserver/selector.h"

#include <cstdlib>

#include "core/util.h"

namespace kf {

namespace {
bool req_matches(const Requirement& r, const Json& labels) {
  const Json* v = labels.find(r.key);
  switch (r.op) {
    case Requirement::Op::Exists: return v != nullptr;
    case Requirement::Op::DoesNotExist: return v == nullptr;
    case Requirement::Op::Eq:
    case Requirement::Op::In:
      if (!v) return false;
      for (const auto& x : r.values)
        if (v->as_string() == x) return true;
      return false;
    case Requirement::Op::NotEq:
    case Requirement::Op::NotIn:
      if (!v) return true;
      for (const auto& x : r.values)
        if (v->as_string() == x) return false;
      return true;
    case Requirement::Op::Gt:
    case Requirement::Op::Lt: {
      if (!v || r.values.empty()) return false;
      double a = std::strtod(v->as_string().c_str(), nullptr), b = std::strtod(r.values[0].c_str(), nullptr);
      return r.op == Requirement::Op::Gt ? a > b : a < b;
    }
  }
  return false;
}
}  // namespace

bool LabelSelector::parse(const std::string& s_in, LabelSelector& out, std::string* err) {
  out = LabelSelector();
  std::string s = trim(s_in);
  if (s.empty()) return true;
  // split on commas that are not inside parentheses
  std::vector<std::string> terms;
  std::string cur;
  int depth = 0;
  for (char c : s) {
    if (c == '(') depth++;
    if (c == ')') depth--;
    if (c == ',' && depth == 0) {
      terms.push_back(trim(cur));
      cur.clear();
    } else {
      cur += c;
    }
  }
  terms.push_back(trim(cur));
  for (auto& t : terms) {
    if (t.empty()) continue;
    Requirement r;
    auto set_values = [&](const std::string& body) {
      for (auto& v : split(body, ',')) r.values.push_back(trim(v));
    };
    size_t p;
    if (t[0] == '!') {
      r.op = Requirement::Op::DoesNotExist;
      r.key = trim(t.substr(1));
    } else if ((p = t.find(" notin ")) != std::string::npos) {
      r.op = Requirement::Op::NotIn;
      r.key = trim(t.substr(0, p));
      std::string rest = trim(t.substr(p + 7));
      if (rest.size() < 2 || rest.front() != '(' || rest.back() != ')') goto bad;
      set_values(rest.substr(1, rest.size() - 2));
    } else if ((p = t.find(" in ")) != std::string::npos) {
      r.op = Requirement::Op::In;
      r.key = trim(t.substr(0, p));
      std::string rest = trim(t.substr(p + 4));
      if (rest.size() < 2 || rest.front() != '(' || rest.back() != ')') goto bad;
      set_values(rest.substr(1, rest.size() - 2));
    } else if ((p = t.find("!=")) != std::string::npos) {
      r.op = Requirement::Op::NotEq;
      r.key = trim(t.substr(0, p));
      r.values.push_back(trim(t.substr(p + 2)));
    } else if ((p = t.find("==")) != std::string::npos) {
      r.op = Requirement::Op::Eq;
      r.key = trim(t.substr(0, p));
      r.values.push_back(trim(t.substr(p + 2)));
    } else if ((p = t.find('=')) != std::string::npos) {
      r.op = Requirement::Op::Eq;
      r.key = trim(t.substr(0, p));
      r.values.push_back(trim(t.substr(p + 1)));
    } else if ((p = t.find('>')) != std::string::npos) {
      r.op = Requirement::Op::Gt;
      r.key = trim(t.substr(0, p));
      r.values.push_back(trim(t.substr(p + 1)));
    } else if ((p = t.find('<')) != std::string::npos) {
      r.op = Requirement::Op::Lt;
      r.key = trim(t.substr(0, p));
      r.values.push_back(trim(t.substr(p + 1)));
    } else {
      r.op = Requirement::Op::Exists;
      r.key = t;
    }
    if (r.key.empty()) goto bad;
    out.reqs_.push_back(std::move(r));
    continue;
  bad:
    if (err) *err = "invalid label selector term: " + t;
    return false;
  }
  return true;
}

LabelSelector LabelSelector::from_json(const Json& sel, bool null_matches_nothing) {
  LabelSelector out;
  if (!sel.is_object()) {
    out.nothing_ = null_matches_nothing;
    return out;
  }
  for (const auto& m : sel["matchLabels"].as_object()) {
    Requirement r;
    r.op = Requirement::Op::Eq;
    r.key = m.first;
    r.values.push_back(m.second.as_string());
    out.reqs_.push_back(r);
  }
  for (const auto& e : sel["matchExpressions"].as_array()) {
    Requirement r;
    r.key = e["key"].as_string();
    const std::string& op = e["operator"].as_string();
    if (op == "In") r.op = Requirement::Op::In;
    else if (op == "NotIn") r.op = Requirement::Op::NotIn;
    else if (op == "Exists") r.op = Requirement::Op::Exists;
    else if (op == "DoesNotExist") r.op = Requirement::Op::DoesNotExist;
    else continue;
    for (const auto& v : e["values"].as_array()) r.values.push_back(v.as_string());
    out.reqs_.push_back(r);
  }
  return out;
}

bool LabelSelector::matches(const Json& labels) const {
  if (nothing_) return false;
  for (const auto& r : reqs_)
    if (!req_matches(r, labels)) return false;
  return true;
}

std::string LabelSelector::str() const {
  std::vector<std::string> parts;
  for (const auto& r : reqs_) {
    switch (r.op) {
      case Requirement::Op::Eq: parts.push_back(r.key + "=" + (r.values.empty() ? "" : r.values[0])); break;
      case Requirement::Op::NotEq: parts.push_back(r.key + "!=" + (r.values.empty() ? "" : r.values[0])); break;
      case Requirement::Op::In: parts.push_back(r.key + " in (" + join(r.values, ",") + ")"); break;
      case Requirement::Op::NotIn: parts.push_back(r.key + " notin (" + join(r.values, ",") + ")"); break;
      case Requirement::Op::Exists: parts.push_back(r.key); break;
      case Requirement::Op::DoesNotExist: parts.push_back("!" + r.key); break;
      case Requirement::Op::Gt: parts.push_back(r.key + ">" + r.values[0]); break;
      case Requirement::Op::Lt: parts.push_back(r.key + "<" + r.values[0]); break;
    }
  }
  return join(parts, ",");
}

bool FieldSelector::parse(const std::string& s, FieldSelector& out, std::string* err) {
  out = FieldSelector();
  for (auto& t : split(s, ',', true)) {
    Term term;
    size_t p = t.find("!=");
    std::string k, v;
    if (p != std::string::npos) {
      term.neq = true;
      k = t.substr(0, p);
      v = t.substr(p + 2);
    } else if ((p = t.find("==")) != std::string::npos) {
      k = t.substr(0, p);
      v = t.substr(p + 2);
    } else if ((p = t.find('=')) != std::string::npos) {
      k = t.substr(0, p);
      v = t.substr(p + 1);
    } else {
      if (err) *err = "invalid field selector: " + t;
      return false;
    }
    term.path = split(trim(k), '.', true);
    term.value = trim(v);
    out.terms_.push_back(std::move(term));
  }
  return true;
}

bool FieldSelector::matches(const Json& obj) const {
  for (const auto& t : terms_) {
    const Json& v = obj.at_path(t.path);
    std::string sv;
    if (v.is_string()) sv = v.as_string();
    else if (v.is_bool()) sv = v.as_bool() ? "true" : "false";
    else if (v.is_number()) sv = v.dump();
    bool eq = sv == t.value;
    if (t.neq ? eq : !eq) return false;
  }
  return true;
}

bool match_node_selector_term(const Json& term, const Json& node) {
  const Json& labels = node.at_path({"metadata", "labels"});
  for (const auto& e : term["matchExpressions"].as_array()) {
    Requirement r;
    r.key = e["key"].as_string();
    const std::string& op = e["operator"].as_string();
    if (op == "In") r.op = Requirement::Op::In;
    else if (op == "NotIn") r.op = Requirement::Op::NotIn;
    else if (op == "Exists") r.op = Requirement::Op::Exists;
    else if (op == "DoesNotExist") r.op = Requirement::Op::DoesNotExist;
    else if (op == "Gt") r.op = Requirement::Op::Gt;
    else if (op == "Lt") r.op = Requirement::Op::Lt;
    else return false;
    for (const auto& v : e["values"].as_array()) r.values.push_back(v.as_string());
    if (!req_matches(r, labels)) return false;
  }
  for (const auto& e : term["matchFields"].as_array()) {
    const std::string& key = e["key"].as_string();
    std::string val = key == "metadata.name" ? node.str_at({"metadata", "name"}) : "";
    bool in = false;
    for (const auto& v : e["values"].as_array()) in = in || v.as_string() == val;
    if ((e["operator"].as_string() == "In") != in) return false;
  }
  return true;
}

}  // namespace kf
