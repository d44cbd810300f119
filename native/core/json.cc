// json.cc — see json.h.
#include "core/json.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace kf {

namespace {
const Json kNull;
const std::string kEmptyStr;
const Json::Array kEmptyArr;
const Json::Object kEmptyObj;

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}
  Json parse_document() {
    ws();
    Json v = value(0);
    ws();
    if (p_ != s_.size()) fail("trailing characters");
    return v;
  }

 private:
  [[noreturn]] void fail(const char* what) {
    throw JsonError(std::string("json: ") + what + " at offset " + std::to_string(p_));
  }
  void ws() {
    while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\n' || s_[p_] == '\t' || s_[p_] == '\r')) ++p_;
  }
  bool lit(const char* w) {
    size_t n = std::strlen(w);
    if (s_.compare(p_, n, w) == 0) {
      p_ += n;
      return true;
    }
    return false;
  }
  Json value(int depth) {
    if (depth > 512) fail("nesting too deep");
    if (p_ >= s_.size()) fail("unexpected end");
    char c = s_[p_];
    if (c == '{') return object(depth);
    if (c == '[') return array(depth);
    if (c == '"') return Json(string());
    if (c == 't') {
      if (lit("true")) return Json(true);
      fail("bad literal");
    }
    if (c == 'f') {
      if (lit("false")) return Json(false);
      fail("bad literal");
    }
    if (c == 'n') {
      if (lit("null")) return Json();
      fail("bad literal");
    }
    return number();
  }
  Json object(int depth) {
    ++p_;
    Json::Object o;
    ws();
    if (p_ < s_.size() && s_[p_] == '}') {
      ++p_;
      return Json(std::move(o));
    }
    for (;;) {
      ws();
      if (p_ >= s_.size() || s_[p_] != '"') fail("expected key");
      std::string k = string();
      ws();
      if (p_ >= s_.size() || s_[p_] != ':') fail("expected ':'");
      ++p_;
      ws();
      Json v = value(depth + 1);
      bool replaced = false;
      for (auto& m : o)
        if (m.first == k) {
          m.second = std::move(v);
          replaced = true;
          break;
        }
      if (!replaced) o.emplace_back(std::move(k), std::move(v));
      ws();
      if (p_ >= s_.size()) fail("unterminated object");
      if (s_[p_] == ',') {
        ++p_;
        continue;
      }
      if (s_[p_] == '}') {
        ++p_;
        break;
      }
      fail("expected ',' or '}'");
    }
    return Json(std::move(o));
  }
  Json array(int depth) {
    ++p_;
    Json::Array a;
    ws();
    if (p_ < s_.size() && s_[p_] == ']') {
      ++p_;
      return Json(std::move(a));
    }
    for (;;) {
      ws();
      a.push_back(value(depth + 1));
      ws();
      if (p_ >= s_.size()) fail("unterminated array");
      if (s_[p_] == ',') {
        ++p_;
        continue;
      }
      if (s_[p_] == ']') {
        ++p_;
        break;
      }
      fail("expected ',' or ']'");
    }
    return Json(std::move(a));
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += static_cast<char>(cp);
    } else if (cp < 0x800) {
      out += static_cast<char>(0xC0 | (cp >> 6));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += static_cast<char>(0xE0 | (cp >> 12));
      out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    } else {
      out += static_cast<char>(0xF0 | (cp >> 18));
      out += static_cast<char>(0x80 | ((cp >> 12) & 0x3F));
      out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (p_ + 4 > s_.size()) fail("bad \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = s_[p_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string string() {
    ++p_;
    std::string out;
    for (;;) {
      if (p_ >= s_.size()) fail("unterminated string");
      char c = s_[p_++];
      if (c == '"') break;
      if (c != '\\') {
        out += c;
        continue;
      }
      if (p_ >= s_.size()) fail("bad escape");
      char e = s_[p_++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF && p_ + 1 < s_.size() && s_[p_] == '\\' && s_[p_ + 1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Json number() {
    size_t start = p_;
    bool is_float = false;
    if (s_[p_] == '-') ++p_;
    while (p_ < s_.size()) {
      char c = s_[p_];
      if (c >= '0' && c <= '9') {
        ++p_;
      } else if (c == '.' || c == 'e' || c == 'E' || c == '+' || (c == '-' && p_ > start)) {
        is_float = true;
        ++p_;
      } else {
        break;
      }
    }
    if (p_ == start) fail("unexpected character");
    std::string tok = s_.substr(start, p_ - start);
    if (!is_float) {
      errno = 0;
      char* end = nullptr;
      long long v = std::strtoll(tok.c_str(), &end, 10);
      if (errno == 0 && end && *end == 0) return Json(v);
    }
    char* end = nullptr;
    double d = std::strtod(tok.c_str(), &end);
    if (!end || *end != 0) fail("bad number");
    return Json(d);
  }
  const std::string& s_;
  size_t p_ = 0;
};

void dump_string(std::string& out, const std::string& s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += static_cast<char>(c);
        }
    }
  }
  out += '"';
}
}  // namespace

Json Json::parse(const std::string& text) { return Parser(text).parse_document(); }

bool Json::try_parse(const std::string& text, Json& out, std::string* err) {
  try {
    out = parse(text);
    return true;
  } catch (const JsonError& e) {
    if (err) *err = e.what();
    return false;
  }
}

int64_t Json::as_int(int64_t def) const {
  if (t_ == Type::Int) return i_;
  if (t_ == Type::Double) return static_cast<int64_t>(d_);
  return def;
}
double Json::as_double(double def) const {
  if (t_ == Type::Double) return d_;
  if (t_ == Type::Int) return static_cast<double>(i_);
  return def;
}
Json::Json(const Json& o)
    : t_(o.t_), b_(o.b_), i_(o.i_), d_(o.d_), s_(o.s_),
      a_(o.a_ ? std::make_unique<Array>(*o.a_) : nullptr),
      o_(o.o_ ? std::make_unique<Object>(*o.o_) : nullptr) {}
Json::Json(Json&& o) noexcept
    : t_(o.t_), b_(o.b_), i_(o.i_), d_(o.d_), s_(std::move(o.s_)), a_(std::move(o.a_)), o_(std::move(o.o_)) {
  o.t_ = Type::Null;
}
void Json::swap(Json& o) noexcept {
  std::swap(t_, o.t_);
  std::swap(b_, o.b_);
  std::swap(i_, o.i_);
  std::swap(d_, o.d_);
  s_.swap(o.s_);
  a_.swap(o.a_);
  o_.swap(o.o_);
}
// copy/move into a temporary first: `x = x["child"]` (source inside the target) stays valid
Json& Json::operator=(const Json& o) {
  if (this != &o) {
    Json tmp(o);
    swap(tmp);
  }
  return *this;
}
Json& Json::operator=(Json&& o) noexcept {
  if (this != &o) {
    Json tmp(std::move(o));
    swap(tmp);
  }
  return *this;
}

const std::string& Json::as_string() const { return t_ == Type::String ? s_ : kEmptyStr; }
const Json::Array& Json::as_array() const { return t_ == Type::Array ? *a_ : kEmptyArr; }
Json::Array& Json::mut_array() {
  if (t_ != Type::Array) {
    *this = Json(Array{});
  }
  return *a_;
}
const Json::Object& Json::as_object() const { return t_ == Type::Object ? *o_ : kEmptyObj; }
Json::Object& Json::mut_object() {
  if (t_ != Type::Object) *this = Json(Object{});
  return *o_;
}

Json& Json::operator[](const std::string& key) {
  if (t_ != Type::Object) *this = Json(Object{});
  for (auto& m : *o_)
    if (m.first == key) return m.second;
  o_->emplace_back(key, Json());
  return o_->back().second;
}
const Json& Json::get(const std::string& key) const {
  const Json* p = find(key);
  return p ? *p : kNull;
}
const Json* Json::find(const std::string& key) const {
  if (t_ != Type::Object) return nullptr;
  for (auto& m : *o_)
    if (m.first == key) return &m.second;
  return nullptr;
}
Json* Json::find(const std::string& key) {
  if (t_ != Type::Object) return nullptr;
  for (auto& m : *o_)
    if (m.first == key) return &m.second;
  return nullptr;
}
bool Json::erase(const std::string& key) {
  if (t_ != Type::Object) return false;
  for (auto it = o_->begin(); it != o_->end(); ++it)
    if (it->first == key) {
      o_->erase(it);
      return true;
    }
  return false;
}
Json& Json::operator[](size_t i) {
  if (t_ != Type::Array || i >= a_->size()) throw JsonError("json: array index out of range");
  return (*a_)[i];
}
const Json& Json::operator[](size_t i) const {
  if (t_ != Type::Array || i >= a_->size()) return kNull;
  return (*a_)[i];
}
void Json::push_back(Json v) {
  if (t_ != Type::Array) *this = Json(Array{});
  a_->push_back(std::move(v));
}
size_t Json::size() const {
  if (t_ == Type::Array) return a_->size();
  if (t_ == Type::Object) return o_->size();
  return 0;
}

const Json& Json::at_path(std::initializer_list<const char*> path) const {
  const Json* cur = this;
  for (const char* k : path) {
    cur = cur->find(k);
    if (!cur) return kNull;
  }
  return *cur;
}
const Json& Json::at_path(const std::vector<std::string>& path) const {
  const Json* cur = this;
  for (const auto& k : path) {
    if (cur->is_array()) {
      char* end = nullptr;
      long idx = std::strtol(k.c_str(), &end, 10);
      if (!end || *end || idx < 0 || static_cast<size_t>(idx) >= cur->a_->size()) return kNull;
      cur = &(*cur->a_)[idx];
      continue;
    }
    cur = cur->find(k);
    if (!cur) return kNull;
  }
  return *cur;
}
Json& Json::mut_path(std::initializer_list<const char*> path) {
  Json* cur = this;
  for (const char* k : path) {
    if (!cur->is_object()) *cur = Json(Object{});
    cur = &(*cur)[k];
  }
  return *cur;
}
std::string Json::str_at(std::initializer_list<const char*> path, const std::string& def) const {
  const Json& v = at_path(path);
  return v.is_string() ? v.s_ : def;
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  auto nl = [&](int d) {
    if (indent < 0) return;
    out += '\n';
    out.append(static_cast<size_t>(indent * d), ' ');
  };
  switch (t_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: out += std::to_string(i_); break;
    case Type::Double: {
      if (!std::isfinite(d_)) {
        out += "null";
        break;
      }
      char buf[32];
      std::snprintf(buf, sizeof buf, "%.17g", d_);
      // shortest round-trip-ish representation
      char buf2[32];
      for (int prec = 1; prec <= 17; ++prec) {
        std::snprintf(buf2, sizeof buf2, "%.*g", prec, d_);
        if (std::strtod(buf2, nullptr) == d_) {
          std::memcpy(buf, buf2, sizeof buf);
          break;
        }
      }
      out += buf;
      if (!std::strpbrk(buf, ".eEn")) out += ".0";
      break;
    }
    case Type::String: dump_string(out, s_); break;
    case Type::Array: {
      out += '[';
      for (size_t i = 0; i < a_->size(); ++i) {
        if (i) out += ',';
        nl(depth + 1);
        (*a_)[i].dump_to(out, indent, depth + 1);
      }
      if (!a_->empty()) nl(depth);
      out += ']';
      break;
    }
    case Type::Object: {
      out += '{';
      for (size_t i = 0; i < o_->size(); ++i) {
        if (i) out += ',';
        nl(depth + 1);
        dump_string(out, (*o_)[i].first);
        out += indent >= 0 ? ": " : ":";
        (*o_)[i].second.dump_to(out, indent, depth + 1);
      }
      if (!o_->empty()) nl(depth);
      out += '}';
      break;
    }
  }
}

std::string Json::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

bool Json::operator==(const Json& o) const {
  if (is_number() && o.is_number()) {
    if (t_ == Type::Int && o.t_ == Type::Int) return i_ == o.i_;
    return as_double() == o.as_double();
  }
  if (t_ != o.t_) return false;
  switch (t_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::String: return s_ == o.s_;
    case Type::Array: return *a_ == *o.a_;
    case Type::Object: {
      if (o_->size() != o.o_->size()) return false;
      for (const auto& m : *o_) {
        const Json* v = o.find(m.first);
        if (!v || !(*v == m.second)) return false;
      }
      return true;
    }
    default: return false;
  }
}

std::string json_quote(const std::string& s) {
  std::string out;
  dump_string(out, s);
  return out;
}

std::string json_pointer_escape(const std::string& s) {
  std::string out;
  for (char c : s) {
    if (c == '~') out += "~0";
    else if (c == '/') out += "~1";
    else out += c;
  }
  return out;
}

// ---------------------------------------------------------------------------------------------
Json merge_patch(const Json& target, const Json& patch) {
  if (!patch.is_object()) return patch;
  Json result = target.is_object() ? target : Json::object();
  for (const auto& m : patch.as_object()) {
    if (m.second.is_null()) {
      result.erase(m.first);
    } else {
      result[m.first] = merge_patch(result.get(m.first), m.second);
    }
  }
  return result;
}

Json diff_merge_patch(const Json& from, const Json& to) {
  if (!from.is_object() || !to.is_object()) return to;
  Json patch = Json::object();
  for (const auto& m : from.as_object()) {
    if (!to.has(m.first)) patch[m.first] = Json();
  }
  for (const auto& m : to.as_object()) {
    const Json* f = from.find(m.first);
    if (!f) {
      patch[m.first] = m.second;
    } else if (*f != m.second) {
      if (f->is_object() && m.second.is_object()) patch[m.first] = diff_merge_patch(*f, m.second);
      else patch[m.first] = m.second;
    }
  }
  return patch;
}

namespace {
std::vector<std::string> split_pointer(const std::string& ptr) {
  std::vector<std::string> out;
  if (ptr.empty()) return out;
  if (ptr[0] != '/') throw JsonError("json patch: path must start with '/': " + ptr);
  size_t i = 1;
  std::string cur;
  for (; i <= ptr.size(); ++i) {
    if (i == ptr.size() || ptr[i] == '/') {
      out.push_back(cur);
      cur.clear();
      continue;
    }
    if (ptr[i] == '~' && i + 1 < ptr.size()) {
      cur += ptr[i + 1] == '1' ? '/' : '~';
      ++i;
    } else {
      cur += ptr[i];
    }
  }
  return out;
}

Json* resolve_parent(Json& root, const std::vector<std::string>& toks, bool create) {
  Json* cur = &root;
  for (size_t i = 0; i + 1 < toks.size(); ++i) {
    const std::string& t = toks[i];
    if (cur->is_array()) {
      size_t idx = static_cast<size_t>(std::strtoul(t.c_str(), nullptr, 10));
      if (idx >= cur->size()) throw JsonError("json patch: index out of range: " + t);
      cur = &(*cur)[idx];
    } else if (cur->is_object()) {
      Json* n = cur->find(t);
      if (!n) {
        if (!create) throw JsonError("json patch: missing path segment: " + t);
        n = &(*cur)[t];
        *n = Json::object();
      }
      cur = n;
    } else {
      throw JsonError("json patch: cannot traverse scalar at " + t);
    }
  }
  return cur;
}

Json get_ptr(const Json& root, const std::vector<std::string>& toks) {
  const Json* cur = &root;
  for (const auto& t : toks) {
    if (cur->is_array()) {
      size_t idx = static_cast<size_t>(std::strtoul(t.c_str(), nullptr, 10));
      if (idx >= cur->size()) throw JsonError("json patch: index out of range");
      cur = &(*cur)[idx];
    } else {
      cur = cur->find(t);
      if (!cur) throw JsonError("json patch: path not found");
    }
  }
  return *cur;
}

void remove_ptr(Json& root, const std::vector<std::string>& toks) {
  if (toks.empty()) throw JsonError("json patch: cannot remove root");
  Json* parent = resolve_parent(root, toks, false);
  const std::string& last = toks.back();
  if (parent->is_array()) {
    size_t idx = static_cast<size_t>(std::strtoul(last.c_str(), nullptr, 10));
    auto& arr = parent->mut_array();
    if (idx >= arr.size()) throw JsonError("json patch: remove index out of range");
    arr.erase(arr.begin() + static_cast<long>(idx));
  } else {
    if (!parent->erase(last)) throw JsonError("json patch: remove of missing key " + last);
  }
}

void add_ptr(Json& root, const std::vector<std::string>& toks, Json value, bool replace) {
  if (toks.empty()) {
    root = std::move(value);
    return;
  }
  Json* parent = resolve_parent(root, toks, false);
  const std::string& last = toks.back();
  if (parent->is_array()) {
    auto& arr = parent->mut_array();
    if (last == "-") {
      if (replace) throw JsonError("json patch: replace with '-'");
      arr.push_back(std::move(value));
      return;
    }
    size_t idx = static_cast<size_t>(std::strtoul(last.c_str(), nullptr, 10));
    if (replace) {
      if (idx >= arr.size()) throw JsonError("json patch: replace index out of range");
      arr[idx] = std::move(value);
    } else {
      if (idx > arr.size()) throw JsonError("json patch: add index out of range");
      arr.insert(arr.begin() + static_cast<long>(idx), std::move(value));
    }
  } else if (parent->is_object()) {
    // kube-apiserver's json-patch (evanphx/json-patch v4) lets `replace` create a missing object
    // member; the reference CI relies on it to set the webhook's absent caBundle
    // (odh_notebook_controller_integration_test.yaml:207-212). Array indices stay strict.
    (*parent)[last] = std::move(value);
  } else {
    throw JsonError("json patch: parent is not a container");
  }
}

void diff_into(const Json& from, const Json& to, const std::string& path, Json& ops) {
  if (from == to) return;
  if (from.is_object() && to.is_object()) {
    for (const auto& m : from.as_object())
      if (!to.has(m.first))
        ops.push_back(Json{{"op", "remove"}, {"path", path + "/" + json_pointer_escape(m.first)}});
    for (const auto& m : to.as_object()) {
      const Json* f = from.find(m.first);
      std::string p = path + "/" + json_pointer_escape(m.first);
      if (!f) ops.push_back(Json{{"op", "add"}, {"path", p}, {"value", m.second}});
      else diff_into(*f, m.second, p, ops);
    }
    return;
  }
  if (from.is_array() && to.is_array() && from.size() == to.size()) {
    for (size_t i = 0; i < from.size(); ++i) diff_into(from[i], to[i], path + "/" + std::to_string(i), ops);
    return;
  }
  if (from.is_array() && to.is_array() && to.size() > from.size()) {
    bool prefix = true;
    for (size_t i = 0; i < from.size() && prefix; ++i) prefix = from[i] == to[i];
    if (prefix) {
      for (size_t i = from.size(); i < to.size(); ++i)
        ops.push_back(Json{{"op", "add"}, {"path", path + "/-"}, {"value", to[i]}});
      return;
    }
  }
  if (path.empty()) {
    ops.push_back(Json{{"op", "replace"}, {"path", ""}, {"value", to}});
  } else {
    ops.push_back(Json{{"op", "replace"}, {"path", path}, {"value", to}});
  }
}
}  // namespace

Json apply_json_patch(const Json& target, const Json& ops) {
  if (!ops.is_array()) throw JsonError("json patch: document must be an array");
  Json doc = target;
  for (const auto& op : ops.as_array()) {
    const std::string& kind = op["op"].as_string();
    auto toks = split_pointer(op["path"].as_string());
    if (kind == "add") {
      add_ptr(doc, toks, op["value"], false);
    } else if (kind == "replace") {
      add_ptr(doc, toks, op["value"], true);
    } else if (kind == "remove") {
      remove_ptr(doc, toks);
    } else if (kind == "test") {
      if (get_ptr(doc, toks) != op["value"]) throw JsonError("json patch: test failed at " + op["path"].as_string());
    } else if (kind == "move" || kind == "copy") {
      auto from = split_pointer(op["from"].as_string());
      Json v = get_ptr(doc, from);
      if (kind == "move") remove_ptr(doc, from);
      add_ptr(doc, toks, std::move(v), false);
    } else {
      throw JsonError("json patch: unknown op " + kind);
    }
  }
  return doc;
}

Json diff_json_patch(const Json& from, const Json& to) {
  Json ops = Json::array();
  diff_into(from, to, "", ops);
  return ops;
}

// ---------------------------------------------------------------------------------------------
namespace {
const char* merge_key_for(const std::string& field) {
  static const std::map<std::string, const char*> keys = {
      {"containers", "name"},     {"initContainers", "name"}, {"ephemeralContainers", "name"},
      {"volumes", "name"},        {"env", "name"},            {"imagePullSecrets", "name"},
      {"volumeMounts", "mountPath"}, {"volumeDevices", "devicePath"}, {"ports", "containerPort"},
      {"hostAliases", "ip"},      {"conditions", "type"},     {"finalizers", ""},
      {"ownerReferences", "uid"}, {"envFrom", ""},            {"subjects", ""},
  };
  auto it = keys.find(field);
  return it == keys.end() ? nullptr : it->second;
}
}  // namespace

Json strategic_merge_patch(const Json& target, const Json& patch, const std::string& field) {
  if (patch.is_array()) {
    const char* key = merge_key_for(field);
    if (!key || !*key || !target.is_array()) {
      if (key && !*key && target.is_array()) {
        // primitive set-merge list (e.g. finalizers): union preserving order
        Json out = target;
        for (const auto& v : patch.as_array()) {
          bool found = false;
          for (const auto& e : out.as_array()) found = found || e == v;
          if (!found) out.push_back(v);
        }
        return out;
      }
      return patch;
    }
    Json out = target;
    for (const auto& item : patch.as_array()) {
      // Service ports merge by "port" (container ports by "containerPort", the table's key)
      const char* k = key;
      if (field == "ports" && item.is_object() && !item.has(k) && item.has("port")) k = "port";
      if (!item.is_object() || !item.has(k)) {
        out.push_back(item);
        continue;
      }
      const Json& kv = item[k];
      bool del = item["$patch"].as_string() == "delete";
      auto& arr = out.mut_array();
      bool merged = false;
      for (size_t i = 0; i < arr.size(); ++i) {
        if (arr[i][k] == kv) {
          if (del) {
            arr.erase(arr.begin() + static_cast<long>(i));
          } else {
            arr[i] = strategic_merge_patch(arr[i], item, "");
          }
          merged = true;
          break;
        }
      }
      if (!merged && !del) out.push_back(item);
    }
    return out;
  }
  if (!patch.is_object()) return patch;
  if (patch["$patch"].as_string() == "replace") {
    Json p = patch;
    p.erase("$patch");
    return p;
  }
  Json result = target.is_object() ? target : Json::object();
  for (const auto& m : patch.as_object()) {
    if (m.first == "$patch" || m.first == "$retainKeys") continue;
    if (m.second.is_null()) {
      result.erase(m.first);
    } else if (m.second.is_object() && m.second["$patch"].as_string() == "delete") {
      result.erase(m.first);
    } else {
      result[m.first] = strategic_merge_patch(result.get(m.first), m.second, m.first);
    }
  }
  if (patch.has("$retainKeys")) {
    Json kept = Json::object();
    for (const auto& k : patch["$retainKeys"].as_array())
      if (result.has(k.as_string())) kept[k.as_string()] = result[k.as_string()];
    result = kept;
  }
  return result;
}

void prune_nulls(Json& v) {
  if (v.is_object()) {
    auto& o = v.mut_object();
    for (auto it = o.begin(); it != o.end();) {
      if (it->second.is_null()) {
        it = o.erase(it);
      } else {
        prune_nulls(it->second);
        ++it;
      }
    }
  } else if (v.is_array()) {
    for (auto& e : v.mut_array()) prune_nulls(e);
  }
}

}  // namespace kf
