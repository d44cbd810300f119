// poddefault.cc — N18 PodDefault mutation (see admission.h; reference admission-webhook/main.go:72-704).
#include <set>

#include "admission/admission.h"
#include "apiserver/selector.h"
#include "controllers/common.h"
#include "core/resources.h"
#include "core/util.h"

namespace kf {

namespace {
constexpr const char* kAnnotationPrefix = "poddefault.admission.kubeflow.org";
constexpr const char* kIstioProxy = "istio-proxy";

std::string pd_name(const Json& pd) { return pd.str_at({"metadata", "name"}); }

// Generic "merge list by key, identical duplicates allowed, different -> conflict" (mergeEnv,
// mergeVolumes, mergeTolerations, mergeImagePullSecrets, mergeContainers).
Json merge_list(const Json& orig, const std::vector<Json>& pds, const std::vector<const char*>& field, const char* key,
                const char* what, std::vector<std::string>& errs) {
  std::map<std::string, Json> seen;
  Json merged = orig.is_array() ? orig : Json::array();
  for (const auto& v : orig.as_array()) seen[v[key].as_string()] = v;
  for (const auto& pd : pds) {
    const Json* list = &pd["spec"];
    for (const char* f : field) list = &(*list)[f];
    for (const auto& v : list->as_array()) {
      const std::string k = v[key].as_string();
      auto it = seen.find(k);
      if (it == seen.end()) {
        seen[k] = v;
        merged.push_back(v);
      } else if (it->second != v) {
        errs.push_back(std::string("merging ") + what + " for " + pd_name(pd) + " has a conflict on " + k + ": " + v.dump() +
                       " does not match " + it->second.dump());
      }
    }
  }
  return merged;
}

Json merge_volume_mounts(const Json& orig, const std::vector<Json>& pds, std::vector<std::string>& errs) {
  std::map<std::string, Json> by_name, by_path;
  Json merged = orig.is_array() ? orig : Json::array();
  for (const auto& v : orig.as_array()) {
    by_name[v["name"].as_string()] = v;
    by_path[v["mountPath"].as_string()] = v;
  }
  for (const auto& pd : pds) {
    for (const auto& v : pd.at_path({"spec", "volumeMounts"}).as_array()) {
      auto it = by_name.find(v["name"].as_string());
      if (it == by_name.end()) {
        by_name[v["name"].as_string()] = v;
        merged.push_back(v);
      } else if (it->second != v) {
        errs.push_back("merging volume mounts for " + pd_name(pd) + " has a conflict on " + v["name"].as_string());
      }
      auto pt = by_path.find(v["mountPath"].as_string());
      if (pt == by_path.end()) {
        by_path[v["mountPath"].as_string()] = v;
      } else if (pt->second != v) {
        errs.push_back("merging volume mounts for " + pd_name(pd) + " has a conflict on mount path " + v["mountPath"].as_string());
      }
    }
  }
  return merged;
}
}  // namespace

std::vector<Json> filter_pod_defaults(const std::vector<Json>& list, const Json& pod) {
  std::vector<Json> out;
  for (const auto& pd : list) {
    LabelSelector sel = LabelSelector::from_json(pd.at_path({"spec", "selector"}), false);
    if (!sel.matches(pod.at_path({"metadata", "labels"}))) continue;
    if (pd.str_at({"metadata", "namespace"}) != pod.str_at({"metadata", "namespace"})) continue;
    out.push_back(pd);
  }
  return out;
}

bool merge_map(const Json& existing, const std::vector<Json>& defaults, Json& out, std::string* err) {
  out = existing.is_object() ? existing : Json::object();
  std::vector<std::string> errs;
  for (const auto& def : defaults)
    for (const auto& m : def.as_object()) {
      const Json* ov = out.find(m.first);
      if (!ov) out[m.first] = m.second;
      else if (*ov != m.second) errs.push_back("merging has conflict on " + m.first + ": " + m.second.dump() + " does not match " + ov->dump());
    }
  if (err) *err = join(errs, "; ");
  return errs.empty();
}

std::string safe_to_apply_pod_defaults(const Json& pod, const std::vector<Json>& pds) {
  std::vector<std::string> errs;
  const Json& spec = pod["spec"];
  merge_list(spec["volumes"], pds, {"volumes"}, "name", "volumes", errs);
  merge_list(spec["tolerations"], pds, {"tolerations"}, "key", "tolerations", errs);
  merge_list(spec["imagePullSecrets"], pds, {"imagePullSecrets"}, "name", "imagePullSecret", errs);
  for (const auto& c : spec["containers"].as_array()) {
    merge_list(c["env"], pds, {"env"}, "name", "env", errs);
    merge_volume_mounts(c["volumeMounts"], pds, errs);
  }
  std::vector<Json> anns, labels;
  for (const auto& pd : pds) {
    anns.push_back(pd.at_path({"spec", "annotations"}));
    labels.push_back(pd.at_path({"spec", "labels"}));
  }
  Json tmp;
  std::string e;
  if (!merge_map(pod.at_path({"metadata", "annotations"}), anns, tmp, &e)) errs.push_back(e);
  if (!merge_map(pod.at_path({"metadata", "labels"}), labels, tmp, &e)) errs.push_back(e);
  merge_list(spec["initContainers"], pds, {"initContainers"}, "name", "containers", errs);
  merge_list(spec["containers"], pds, {"sidecars"}, "name", "containers", errs);
  return join(errs, "; ");
}

void set_command_and_args(Json& c, const std::vector<Json>& pds) {
  if (static_cast<const Json&>(c)["name"].as_string() == kIstioProxy) return;  // const read: no autovivify
  for (const auto& pd : pds) {
    if (!c.has("command") && pd.at_path({"spec", "command"}).is_array()) c["command"] = pd.at_path({"spec", "command"});
    if (!c.has("args") && pd.at_path({"spec", "args"}).is_array()) c["args"] = pd.at_path({"spec", "args"});
  }
}

void apply_pod_defaults(Json& pod, const std::vector<Json>& pds) {
  if (pds.empty()) return;
  std::vector<std::string> ignored;
  Json& spec = pod["spec"];
  Json vols = merge_list(spec["volumes"], pds, {"volumes"}, "name", "volumes", ignored);
  if (!vols.empty()) spec["volumes"] = vols;
  Json tols = merge_list(spec["tolerations"], pds, {"tolerations"}, "key", "tolerations", ignored);
  if (!tols.empty()) spec["tolerations"] = tols;
  Json ips = merge_list(spec["imagePullSecrets"], pds, {"imagePullSecrets"}, "name", "imagePullSecret", ignored);
  if (!ips.empty()) spec["imagePullSecrets"] = ips;
  std::vector<Json> anns, labels;
  for (const auto& pd : pds) {
    anns.push_back(pd.at_path({"spec", "annotations"}));
    labels.push_back(pd.at_path({"spec", "labels"}));
    if (pd.at_path({"spec", "automountServiceAccountToken"}).is_bool())
      spec["automountServiceAccountToken"] = pd.at_path({"spec", "automountServiceAccountToken"});
    if (!pd.at_path({"spec", "serviceAccountName"}).as_string().empty())
      spec["serviceAccountName"] = pd.at_path({"spec", "serviceAccountName"});
  }
  Json merged;
  merge_map(pod.at_path({"metadata", "annotations"}), anns, merged, nullptr);
  pod["metadata"]["annotations"] = merged;
  merge_map(pod.at_path({"metadata", "labels"}), labels, merged, nullptr);
  pod["metadata"]["labels"] = merged;
  for (auto& c : spec["containers"].mut_array()) {
    Json env = merge_list(c["env"], pds, {"env"}, "name", "env", ignored);
    if (!env.empty()) c["env"] = env;
    Json vm = merge_volume_mounts(c["volumeMounts"], pds, ignored);
    if (!vm.empty()) c["volumeMounts"] = vm;
    Json ef = c["envFrom"].is_array() ? c["envFrom"] : Json::array();
    for (const auto& pd : pds)
      for (const auto& x : pd.at_path({"spec", "envFrom"}).as_array()) ef.push_back(x);
    if (!ef.empty()) c["envFrom"] = ef;
    set_command_and_args(c, pds);
  }
  Json ics = merge_list(spec["initContainers"], pds, {"initContainers"}, "name", "containers", ignored);
  if (!ics.empty()) spec["initContainers"] = ics;
  Json cs = merge_list(spec["containers"], pds, {"sidecars"}, "name", "containers", ignored);
  if (!cs.empty()) spec["containers"] = cs;
  for (const auto& pd : pds)
    pod["metadata"]["annotations"][std::string(kAnnotationPrefix) + "/poddefault-" + pd_name(pd)] =
        pd.str_at({"metadata", "resourceVersion"});
  prune_nulls(pod);  // the merge helpers read through operator[] on the mutable pod
}

AdmissionFn make_poddefault_plugin(std::shared_ptr<Client> c, PodDefaultOptions o) {
  return [c, o](AdmissionAttrs& a) -> ApiError {
    if (a.operation != "CREATE" || a.res->kind != "Pod" || !a.res->group.empty() || !a.object) return {};
    Json& pod = *a.object;
    if (annotation(pod, std::string(kAnnotationPrefix) + "/exclude") == "true") return {};
    if (has_annotation(pod, "kubernetes.io/config.mirror")) return {};
    if (!o.namespace_selector.empty()) {
      Json ns;
      if (c->get("v1", "Namespace", "", a.ns, ns)) return {};
      LabelSelector sel;
      LabelSelector::parse(o.namespace_selector, sel);
      if (!sel.matches(ns.at_path({"metadata", "labels"}))) return {};
    }
    Json list;
    ApiError e = c->list("kubeflow.org/v1alpha1", "PodDefault", a.ns, ListOptions(), list);
    if (e) return ApiError{500, "InternalError", "error fetching poddefaults: " + e.message};
    std::vector<Json> all(list["items"].as_array().begin(), list["items"].as_array().end());
    if (all.empty()) return {};
    if (pod.str_at({"metadata", "namespace"}).empty()) pod["metadata"]["namespace"] = a.ns;
    auto matching = filter_pod_defaults(all, pod);
    if (matching.empty()) return {};
    std::string conflict = safe_to_apply_pod_defaults(pod, matching);
    if (!conflict.empty()) {
      std::vector<std::string> names;
      for (auto& pd : matching) names.push_back(pd_name(pd));
      return ApiError{403, "Forbidden", "conflict occurred while applying poddefaults: " + join(names, ",") + " on pod: " +
                                            pod.str_at({"metadata", "name"}) + " err: " + conflict};
    }
    apply_pod_defaults(pod, matching);
    return {};
  };
}

// ---- GPU readiness init container (CS6) -------------------------------------------------------
AdmissionFn make_gpu_readiness_plugin(GpuReadinessOptions o) {
  return [o](AdmissionAttrs& a) -> ApiError {
    if (a.operation != "CREATE" || a.res->kind != "Pod" || !a.res->group.empty() || !a.object) return {};
    Json& pod = *a.object;
    if (o.only_notebooks && label(pod, "notebook-name").empty()) return {};
    if (annotation(pod, "kfamd.io/gpu-readiness-op") == "false") return {};
    int64_t gpus = 0;
    for (const auto& c : pod.at_path({"spec", "containers"}).as_array())
      gpus += container_integer_request(c, GPU_RESOURCE).value_or(0);  // invalid counts: rejected by validation
    if (gpus <= 0) return {};
    for (const auto& ic : pod.at_path({"spec", "initContainers"}).as_array())
      if (ic["name"].as_string() == "gpu-readiness") return {};
    Json args = Json::array();
    for (const auto& s : o.args) args.push_back(s);
    // kfamd.io/gpu-readiness-args: extra op flags, e.g. "--min-tflops 1200" (fail a notebook whose
    // GPU underperforms) or "--inject-fault gemm" (fault-injection drills)
    for (const auto& s : split(annotation(pod, "kfamd.io/gpu-readiness-args"), ' ', true)) args.push_back(s);
    std::string mode = annotation(pod, "kfamd.io/gpu-readiness-mode");
    if (mode.empty()) mode = o.mode;
    if (const char* m = std::getenv("KFAMD_GPU_READINESS_MODE"); m && *m && annotation(pod, "kfamd.io/gpu-readiness-mode").empty())
      mode = m;
    const bool sidecar = mode != "init";
    Json env = Json::array();
    Json ic{{"name", "gpu-readiness"},
            {"image", o.image},
            {"command", Json::array({"kfamd-readiness"})},
            {"terminationMessagePolicy", "FallbackToLogsOnError"}};
    if (sidecar) {
      // native sidecar: started before the notebook container, not waited for; the pod is Ready
      // when the server AND /readyz (the op's verdict, published before its GPU teardown) are
      Json sargs = Json::array({"--sidecar", "--port", std::to_string(o.port)});
      for (const auto& x : args.as_array()) sargs.push_back(x);
      ic["args"] = sargs;
      ic["restartPolicy"] = "Always";
      ic["ports"] = Json::array({Json{{"name", "kfamd-ready"}, {"containerPort", o.port}}});
      ic["readinessProbe"] = Json{{"httpGet", Json{{"path", "/readyz"}, {"port", o.port}}},
                                  {"periodSeconds", 10}, {"failureThreshold", 1}};
      // the notebook container holds the GPUs; the sidecar checks THOSE devices (no second
      // allocation: requests of restartable init containers would add to the pod's)
      env.push_back(Json{{"name", "KFAMD_SHARE_POD_GPUS"}, {"value", "true"}});
    } else {
      ic["args"] = args;
      ic["resources"] = Json{{"limits", Json{{GPU_RESOURCE, std::to_string(gpus)}}}};
    }
    // kfamd.io/gpu-readiness-profile: "true" -> the op runs itself under rocprofv3 and reports the
    // per-kernel stats with its result (Notebook status.gpuReadiness.rocprof_top)
    if (annotation(pod, "kfamd.io/gpu-readiness-profile") == "true")
      env.push_back(Json{{"name", "KFAMD_READINESS_PROFILE"}, {"value", "1"}});
    if (env.size()) ic["env"] = env;
    Json& ics = pod["spec"]["initContainers"];
    Json out = Json::array({ic});
    for (const auto& x : ics.as_array()) out.push_back(x);
    ics = out;
    return {};
  };
}

}  // namespace kf
