// registry.h — name -> pure function table behind libkfcore_capi.so (see capi.cc).
#pragma once

#include <functional>
#include <map>
#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

struct CapiRegistry {
  using Fn = std::function<Json(const Json& args)>;
  std::map<std::string, Fn> fns;
  void add(const std::string& name, Fn f) { fns[name] = std::move(f); }
  static CapiRegistry& global();
};

// Other translation units (odh, tensorboard, pvcviewer, kfam) append their registrations here.
std::vector<std::function<void(CapiRegistry&)>>& capi_extensions();

}  // namespace kf
