// resources.cc — see resources.h.
#include "core/resources.h"

#include <cmath>

#include "core/util.h"

namespace kf {

namespace {
const char* kQuantityRe = "quantities must match the regular expression '^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$'";

bool starts(const std::string& s, const char* p) { return s.rfind(p, 0) == 0; }

std::optional<double> quantity_of(const Json& q) {
  if (q.is_number()) return q.as_double();
  if (!q.is_string()) return std::nullopt;
  const std::string& s = q.as_string();
  if (s != trim(s)) return std::nullopt;  // resource.ParseQuantity takes no surrounding whitespace
  return parse_quantity(s);
}

std::string field_invalid(const std::string& path, const std::string& value, const std::string& msg) {
  return path + ": Invalid value: \"" + value + "\": " + msg;
}
}  // namespace

bool is_native_resource(const std::string& name) {
  if (name.find('/') == std::string::npos)
    return name == "cpu" || name == "memory" || name == "ephemeral-storage" || name == "storage" || name == "pods" ||
           starts(name, "hugepages-");
  const std::string domain = name.substr(0, name.find('/'));
  return domain == "kubernetes.io" || ends_with(domain, ".kubernetes.io");
}

bool is_extended_resource(const std::string& name) {
  return name.find('/') != std::string::npos && !is_native_resource(name) && !starts(name, "requests.");
}

std::string canonical_quantity(const Json& q) {
  if (!q.is_string() && !q.is_number()) return q.dump();
  const std::string raw = q.is_string() ? q.as_string() : q.dump();
  auto v = quantity_of(q);
  if (!v) return raw;
  // whole numbers keep their spelling ("2Gi" stays "2Gi"); plain fractions print in milli units
  // like resource.Quantity's DecimalSI canonical form ("0.5" -> "500m", "1.5" -> "1500m")
  if (raw.find('.') != std::string::npos && raw.find_first_of("eEinumkKMGTP") == std::string::npos) {
    const double milli = *v * 1000.0;
    if (std::fabs(milli - std::round(milli)) < 1e-6) {
      if (std::fabs(*v - std::round(*v)) < 1e-9) return std::to_string(static_cast<int64_t>(std::llround(*v)));
      return std::to_string(static_cast<int64_t>(std::llround(milli))) + "m";
    }
  }
  return raw;
}

void validate_resource_requirements(const Json& resources, const std::string& path, ResourceErrors& out) {
  if (resources.is_null()) return;
  if (!resources.is_object()) {
    out.decode.push_back(path + ": expected an object");
    return;
  }
  const Json& lim = resources["limits"];
  const Json& req = resources["requests"];
  for (const char* part : {"limits", "requests"}) {
    const Json& m = resources[part];
    if (m.is_null()) continue;
    if (!m.is_object()) {
      out.decode.push_back(path + "." + part + ": expected a map of resource name to quantity");
      return;
    }
    for (const auto& kv : m.as_object())
      if (!quantity_of(kv.second)) {
        out.decode.push_back(std::string(kQuantityRe) + " (" + path + "." + part + "[" + kv.first + "]: \"" +
                             (kv.second.is_string() ? kv.second.as_string() : kv.second.dump()) + "\")");
      }
  }
  if (!out.decode.empty()) return;
  // ValidateResourceQuantityValue: non-negative; integer for extended resources
  auto check_value = [&](const std::string& fld, const std::string& name, const Json& q) {
    const double v = *quantity_of(q);
    if (v < 0) out.invalid.push_back(field_invalid(fld, canonical_quantity(q), "must be greater than or equal to 0"));
    if (is_extended_resource(name) && std::fabs(v - std::round(v)) > 1e-9)
      out.invalid.push_back(field_invalid(fld, canonical_quantity(q), "must be an integer"));
    if (name.find('/') == std::string::npos && !is_native_resource(name))
      out.invalid.push_back(path + "[" + name + "]: Invalid value: \"" + name + "\": must be a standard resource for containers");
  };
  for (const auto& kv : lim.as_object()) check_value(path + ".limits[" + kv.first + "]", kv.first, kv.second);
  for (const auto& kv : req.as_object()) {
    check_value(path + ".requests[" + kv.first + "]", kv.first, kv.second);
    const bool overcommit = !is_extended_resource(kv.first) && !starts(kv.first, "hugepages-");
    if (!lim.has(kv.first)) {
      if (!overcommit)
        out.invalid.push_back(path + ".limits: Required value: Limit must be set for non overcommitable resources");
      continue;
    }
    const double r = *quantity_of(kv.second), l = *quantity_of(lim[kv.first]);
    if (!overcommit && std::fabs(r - l) > 1e-9)
      out.invalid.push_back(field_invalid(path + ".requests", canonical_quantity(kv.second),
                                          "must be equal to " + kv.first + " limit of " + canonical_quantity(lim[kv.first])));
    else if (r > l + 1e-12)
      out.invalid.push_back(field_invalid(path + ".requests", canonical_quantity(kv.second),
                                          "must be less than or equal to " + kv.first + " limit of " +
                                              canonical_quantity(lim[kv.first])));
  }
}

void validate_pod_spec_resources(const Json& spec, const std::string& path, ResourceErrors& out) {
  for (const char* list : {"containers", "initContainers", "ephemeralContainers"}) {
    const auto& cs = spec[list].as_array();
    for (size_t i = 0; i < cs.size(); ++i)
      validate_resource_requirements(cs[i]["resources"], path + "." + list + "[" + std::to_string(i) + "].resources", out);
  }
}

void default_requests_from_limits(Json& pod_spec) {
  for (const char* list : {"containers", "initContainers"}) {
    Json* cs = pod_spec.find(list);
    if (!cs || !cs->is_array()) continue;
    for (auto& c : cs->mut_array()) {
      Json* res = c.find("resources");
      if (!res || !res->is_object()) continue;
      const Json& lim = (*res)["limits"];
      if (!lim.is_object() || lim.empty()) continue;
      Json& req = (*res)["requests"];
      if (!req.is_object()) req = Json::object();
      for (const auto& kv : lim.as_object())
        if (!req.has(kv.first)) req[kv.first] = kv.second;
    }
  }
}

std::optional<int64_t> container_integer_request(const Json& c, const std::string& resource) {
  const Json* q = &c.at_path({"resources", "requests", resource});
  if (q->is_null()) q = &c.at_path({"resources", "limits", resource});
  if (q->is_null()) return 0;
  auto v = quantity_of(*q);
  if (!v || *v < 0 || std::fabs(*v - std::round(*v)) > 1e-9) return std::nullopt;
  return static_cast<int64_t>(std::llround(*v));
}

std::optional<int64_t> pod_gpu_count(const Json& pod, const std::string& resource) {
  int64_t app = 0, init_max = 0;
  const Json& spec = pod["spec"];
  for (const auto& c : spec["initContainers"].as_array()) {
    auto n = container_integer_request(c, resource);
    if (!n) return std::nullopt;
    if (c["restartPolicy"].as_string() == "Always") app += *n;  // sidecars run beside the app
    else init_max = std::max(init_max, *n);
  }
  for (const auto& c : spec["containers"].as_array()) {
    auto n = container_integer_request(c, resource);
    if (!n) return std::nullopt;
    app += *n;
  }
  return std::max(app, init_max);
}

}  // namespace kf
