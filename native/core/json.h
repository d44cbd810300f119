// json.h — self-contained JSON DOM, parser, serializer and patch algebra for the control plane.
//
// Kubernetes objects are schemaless JSON on the wire; the control plane keeps them as this DOM.
// Objects preserve insertion order (stable, diff-friendly output). Value semantics throughout:
// copying a Json deep-copies it, so a controller's working copy can never alias the cache.
//
// Patch support (used by the API server and the admission webhooks):
//   * RFC 7386 JSON merge patch           (merge_patch)
//   * RFC 6902 JSON patch apply / create  (apply_json_patch, diff_json_patch)
//   * strategic-merge subset with the Kubernetes list merge keys (strategic_merge_patch)
#pragma once

#include <cstdint>
#include <deque>
#include <initializer_list>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace kf {

class JsonError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Json {
 public:
  enum class Type : uint8_t { Null, Bool, Int, Double, String, Array, Object };
  // std::deque: appending a member/element never invalidates references to existing children,
  // so `Json& md = obj["metadata"]; obj["status"] = ...; md["x"] = 1;` is safe.
  using Array = std::deque<Json>;
  using Member = std::pair<std::string, Json>;
  using Object = std::deque<Member>;

  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : t_(Type::Bool), b_(b) {}
  Json(int v) : t_(Type::Int), i_(v) {}
  Json(long v) : t_(Type::Int), i_(v) {}
  Json(long long v) : t_(Type::Int), i_(v) {}
  Json(unsigned v) : t_(Type::Int), i_(v) {}
  Json(unsigned long v) : t_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(unsigned long long v) : t_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(double v) : t_(Type::Double), d_(v) {}
  Json(const char* s) : t_(Type::String), s_(s) {}
  Json(std::string s) : t_(Type::String), s_(std::move(s)) {}
  Json(Array a) : t_(Type::Array), a_(std::make_unique<Array>(std::move(a))) {}
  Json(Object o) : t_(Type::Object), o_(std::make_unique<Object>(std::move(o))) {}
  Json(std::initializer_list<Member> init) : t_(Type::Object), o_(std::make_unique<Object>(init)) {}
  Json(const Json& o);
  Json(Json&& o) noexcept;
  Json& operator=(const Json& o);
  Json& operator=(Json&& o) noexcept;
  ~Json() = default;
  void swap(Json& o) noexcept;

  static Json object() { return Json(Object{}); }
  static Json array() { return Json(Array{}); }
  static Json array(std::initializer_list<Json> init) { return Json(Array(init)); }
  static Json parse(const std::string& text);             // throws JsonError
  static bool try_parse(const std::string& text, Json& out, std::string* err = nullptr);

  Type type() const { return t_; }
  bool is_null() const { return t_ == Type::Null; }
  bool is_bool() const { return t_ == Type::Bool; }
  bool is_int() const { return t_ == Type::Int; }
  bool is_number() const { return t_ == Type::Int || t_ == Type::Double; }
  bool is_string() const { return t_ == Type::String; }
  bool is_array() const { return t_ == Type::Array; }
  bool is_object() const { return t_ == Type::Object; }

  // Lenient accessors: return the default when the type does not match.
  bool as_bool(bool def = false) const { return t_ == Type::Bool ? b_ : def; }
  int64_t as_int(int64_t def = 0) const;
  double as_double(double def = 0.0) const;
  const std::string& as_string() const;  // "" if not a string
  std::string as_string_or(const std::string& def) const { return is_string() ? s_ : def; }
  const Array& as_array() const;         // empty if not an array
  Array& mut_array();                    // converts to array if null
  const Object& as_object() const;       // empty if not an object
  Object& mut_object();                  // converts to object if null

  // Object access. operator[] on a non-const Null converts it to an Object.
  Json& operator[](const std::string& key);
  Json& operator[](const char* key) { return (*this)[std::string(key)]; }
  const Json& operator[](const std::string& key) const { return get(key); }
  const Json& operator[](const char* key) const { return get(std::string(key)); }
  const Json& get(const std::string& key) const;  // Null sentinel if missing
  const Json* find(const std::string& key) const;
  Json* find(const std::string& key);
  bool has(const std::string& key) const { return find(key) != nullptr; }
  bool erase(const std::string& key);
  void set(const std::string& key, Json v) { (*this)[key] = std::move(v); }

  // Array access.
  Json& operator[](size_t i);
  const Json& operator[](size_t i) const;
  Json& operator[](int i) { return (*this)[static_cast<size_t>(i)]; }
  const Json& operator[](int i) const { return (*this)[static_cast<size_t>(i)]; }
  void push_back(Json v);
  size_t size() const;
  bool empty() const { return size() == 0; }

  // Dotted/segmented path helpers ("metadata.annotations" style, no escaping).
  const Json& at_path(std::initializer_list<const char*> path) const;
  const Json& at_path(const std::vector<std::string>& path) const;
  Json& mut_path(std::initializer_list<const char*> path);  // creates objects on the way
  std::string str_at(std::initializer_list<const char*> path, const std::string& def = "") const;

  std::string dump(int indent = -1) const;
  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

 private:
  void dump_to(std::string& out, int indent, int depth) const;
  Type t_ = Type::Null;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0.0;
  std::string s_;
  // Containers live behind a pointer, present iff t_ is Array / Object: a scalar node allocates
  // nothing, and a deep copy costs one container per array/object instead of two (allocating)
  // empty std::deques per node — the copy is on every informer / watch / admission path.
  std::unique_ptr<Array> a_;
  std::unique_ptr<Object> o_;
};

// RFC 7386: null values delete, objects merge recursively, everything else replaces.
Json merge_patch(const Json& target, const Json& patch);
// Drops null-valued object members recursively (typed Kubernetes decoding and CRD pruning treat
// an explicit null like an absent field); array elements are kept but recursed into.
void prune_nulls(Json& v);
// RFC 7396-style diff producing a merge patch that turns `from` into `to`.
Json diff_merge_patch(const Json& from, const Json& to);
// RFC 6902 apply. Throws JsonError on a failed `test` or invalid path.
Json apply_json_patch(const Json& target, const Json& ops);
// RFC 6902 create: minimal-ish op list that turns `from` into `to` (arrays replaced wholesale
// when lengths differ; element-wise when equal length).
Json diff_json_patch(const Json& from, const Json& to);
// Kubernetes strategic merge patch subset: lists of named maps merge by their merge key
// (containers/initContainers/volumes/env/imagePullSecrets by "name", volumeMounts by
// "mountPath", ports by "containerPort", tolerations/args/command replace), `$patch: delete`
// and `$retainKeys` are honoured for map entries; anything else behaves as a merge patch.
Json strategic_merge_patch(const Json& target, const Json& patch, const std::string& field = "");

std::string json_pointer_escape(const std::string& s);
std::string json_quote(const std::string& s);

}  // namespace kf
