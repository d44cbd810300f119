// capi.cc — libkfcore_capi.so: a C ABI over the control plane's pure functions.
//
// One entry point, `kf_call(name, args_json)`, dispatches to the reconcilers' pure helpers
// (StatefulSet/Service/VirtualService generation, notebook status, culling decisions, profile
// label merge / IAM trust-policy edits, PodDefault merge, quota accounting, xGMI placement,
// selectors, patches, schema validation, ...). The Python test-suite drives the reference's
// table-driven unit cases through it (tests/test_unit_*.py), and the web apps reuse the same
// native code instead of re-implementing it in Python.
//
// Result: malloc'd JSON {"ok": true, "result": ...} | {"ok": false, "error": "..."}; release it
// with kf_free().
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <string>

#include "admission/admission.h"
#include "apiserver/resources.h"
#include "apiserver/schemas.h"
#include "apiserver/selector.h"
#include "capi/registry.h"
#include "controllers/common.h"
#include "controllers/notebook.h"
#include "controllers/profile.h"
#include "controllers/tensorboard.h"
#include "core/yaml.h"
#include "kfam/kfam.h"
#include "controllers/odh.h"
#include "core/util.h"
#include "gpu/smi.h"
#include "gpu/topology.h"
#include "node/authz.h"
#include "node/netpol.h"

namespace kf {
namespace {

NotebookOptions nb_opts(const Json& o) {
  NotebookOptions r;
  if (o["use_istio"].is_bool()) r.use_istio = o["use_istio"].as_bool();
  if (o["istio_gateway"].is_string()) r.istio_gateway = o["istio_gateway"].as_string();
  if (o["istio_host"].is_string()) r.istio_host = o["istio_host"].as_string();
  if (o["cluster_domain"].is_string()) r.cluster_domain = o["cluster_domain"].as_string();
  if (o["add_fsgroup"].is_bool()) r.add_fsgroup = o["add_fsgroup"].as_bool();
  return r;
}

std::vector<Json> vec(const Json& a) { return std::vector<Json>(a.as_array().begin(), a.as_array().end()); }

GpuTopology topo_from(const Json& a) {
  return GpuTopology::synthetic(static_cast<int>(a["gpus"].as_int(8)), static_cast<int>(a["numa_nodes"].as_int(2)));
}

Json placement_json(const Placement& p) {
  Json d = Json::array(), r = Json::array();
  for (int x : p.devices) d.push_back(x);
  for (int x : p.ring) r.push_back(x);
  return Json{{"devices", d}, {"ring", r}, {"numa_node", p.numa_node}, {"reason", p.reason}};
}

void register_core(CapiRegistry& R) {
  R.add("parse_quantity", [](const Json& a) -> Json {
    auto v = parse_quantity(a["q"].as_string());
    return v ? Json(*v) : Json();
  });
  R.add("label_selector_matches", [](const Json& a) -> Json {
    LabelSelector sel;
    if (a["selector"].is_string()) {
      std::string err;
      if (!LabelSelector::parse(a["selector"].as_string(), sel, &err)) throw std::runtime_error(err);
    } else {
      sel = LabelSelector::from_json(a["selector"], a["null_matches_nothing"].as_bool());
    }
    return sel.matches(a["labels"]);
  });
  R.add("field_selector_matches", [](const Json& a) -> Json {
    FieldSelector sel;
    std::string err;
    if (!FieldSelector::parse(a["selector"].as_string(), sel, &err)) throw std::runtime_error(err);
    return sel.matches(a["object"]);
  });
  R.add("merge_patch", [](const Json& a) -> Json { return merge_patch(a["target"], a["patch"]); });
  // the gateway's policy enforcement point (node/authz.cc): path normalization, request-line
  // encoding and AuthorizationPolicy evaluation
  R.add("authz_normalize_path", [](const Json& a) -> Json { return normalize_authz_path(a["path"].as_string()); });
  R.add("authz_encode_path", [](const Json& a) -> Json { return encode_request_path(a["path"].as_string()); });
  R.add("authz_evaluate", [](const Json& a) -> Json {
    AuthzRequest r;
    const Json& q = a["request"];
    r.principal = q["principal"].as_string();
    r.source_namespace = q["source_namespace"].as_string();
    r.source_ip = r.remote_ip = q["ip"].as_string();
    r.method = q["method"].as_string_or("GET");
    r.path = q["path"].as_string();
    r.host = q["host"].as_string();
    r.port = static_cast<int>(q["port"].as_int(80));
    for (const auto& kv : q["headers"].as_object()) r.headers[to_lower(kv.first)] = kv.second.as_string();
    std::map<std::string, std::string> labels;
    for (const auto& kv : a["labels"].as_object()) labels[kv.first] = kv.second.as_string();
    const AuthzDecision d = evaluate_authz(vec(a["policies"]), r, a["namespace"].as_string(), labels,
                                           a["root_namespace"].as_string_or("istio-system"));
    return Json{{"allowed", d.allowed}, {"policy", d.policy}, {"reason", d.reason}};
  });
  R.add("diff_merge_patch", [](const Json& a) -> Json { return diff_merge_patch(a["from"], a["to"]); });
  R.add("apply_json_patch", [](const Json& a) -> Json { return apply_json_patch(a["target"], a["ops"]); });
  R.add("diff_json_patch", [](const Json& a) -> Json { return diff_json_patch(a["from"], a["to"]); });
  R.add("strategic_merge_patch", [](const Json& a) -> Json { return strategic_merge_patch(a["target"], a["patch"]); });
  R.add("validate_schema", [](const Json& a) -> Json {
    Json out = Json::array();
    for (const auto& e : validate_schema(a["schema"], a["value"])) out.push_back(e);
    return out;
  });
  R.add("parse_yaml_all", [](const Json& a) -> Json {
    std::vector<Json> docs;
    std::string err;
    if (!parse_yaml_all(a["text"].as_string(), docs, &err)) throw std::runtime_error(err);
    Json out = Json::array();
    for (auto& d : docs) out.push_back(d);
    return out;
  });
  R.add("dump_yaml", [](const Json& a) -> Json { return dump_yaml(a["value"]); });
  R.add("evaluate_netpol", [](const Json& a) -> Json {
    std::vector<Json> pols(a["policies"].as_array().begin(), a["policies"].as_array().end());
    auto strmap = [](const Json& j) {
      std::map<std::string, std::string> m;
      for (const auto& kv : j.as_object()) m[kv.first] = kv.second.as_string();
      return m;
    };
    NetpolSource src;
    const Json& s = a["source"];
    src.pod = s["pod"].as_bool();
    src.ns = s["ns"].as_string();
    src.pod_labels = strmap(s["pod_labels"]);
    src.ns_labels = strmap(s["ns_labels"]);
    src.ip = s["ip"].as_string();
    const NetpolDecision d = evaluate_netpol(pols, a["namespace"].as_string(), strmap(a["pod_labels"]),
                                             static_cast<int>(a["port"].as_int()), a["port_name"].as_string(),
                                             a["protocol"].as_string_or("TCP"), src);
    return Json{{"allowed", d.allowed}, {"isolated", d.isolated}, {"policy", d.policy}, {"reason", d.reason}};
  });
  R.add("prune_unknown_fields", [](const Json& a) -> Json {
    Json v = a["value"];
    std::vector<std::string> pruned;
    prune_unknown_fields(a["schema"], v, &pruned);
    apply_schema_defaults(a["schema"], v);
    Json p = Json::array();
    for (const auto& x : pruned) p.push_back(x);
    return Json{{"value", v}, {"pruned", p}};
  });
  R.add("builtin_crds", [](const Json&) -> Json {
    Json out = Json::array();
    for (const auto& c : builtin_crds()) out.push_back(c);
    return out;
  });
}

void register_notebook(CapiRegistry& R) {
  R.add("generate_statefulset", [](const Json& a) -> Json { return generate_statefulset(a["notebook"], nb_opts(a["options"])); });
  R.add("generate_service", [](const Json& a) -> Json { return generate_service(a["notebook"]); });
  R.add("generate_virtual_service", [](const Json& a) -> Json { return generate_virtual_service(a["notebook"], nb_opts(a["options"])); });
  R.add("virtual_service_name", [](const Json& a) -> Json { return virtual_service_name(a["name"].as_string(), a["namespace"].as_string()); });
  R.add("create_notebook_status", [](const Json& a) -> Json { return create_notebook_status(a["notebook"], a["statefulset"], a["pod"]); });
  R.add("pod_cond_to_notebook_cond", [](const Json& a) -> Json { return pod_cond_to_notebook_cond(a["condition"]); });
  R.add("copy_statefulset_fields", [](const Json& a) -> Json {
    Json to = a["to"];
    bool changed = copy_statefulset_fields(a["from"], to);
    return Json{{"changed", changed}, {"to", to}};
  });
  R.add("copy_service_fields", [](const Json& a) -> Json {
    Json to = a["to"];
    bool changed = copy_service_fields(a["from"], to);
    return Json{{"changed", changed}, {"to", to}};
  });
  R.add("stop_annotation_is_set", [](const Json& a) -> Json { return stop_annotation_is_set(a["object"]); });
  R.add("set_stop_annotation", [](const Json& a) -> Json {
    Json nb = a["object"];
    set_stop_annotation(nb, nullptr);
    return nb;
  });
  R.add("all_kernels_are_idle", [](const Json& a) -> Json { return all_kernels_are_idle(a["kernels"]); });
  R.add("notebook_recent_time", [](const Json& a) -> Json {
    std::vector<std::string> t;
    for (const auto& x : a["times"].as_array()) t.push_back(x.as_string());
    return notebook_recent_time(t);
  });
  R.add("update_timestamp_from_kernels_activity", [](const Json& a) -> Json {
    Json ann = a["annotations"].is_object() ? a["annotations"] : Json::object();
    bool ch = update_timestamp_from_kernels_activity(ann, a["kernels"]);
    return Json{{"changed", ch}, {"annotations", ann}};
  });
  R.add("update_timestamp_from_terminals_activity", [](const Json& a) -> Json {
    Json ann = a["annotations"].is_object() ? a["annotations"] : Json::object();
    bool ch = update_timestamp_from_terminals_activity(ann, a["terminals"]);
    return Json{{"changed", ch}, {"annotations", ann}};
  });
  R.add("notebook_is_idle", [](const Json& a) -> Json {
    return notebook_is_idle(a["notebook"], a["cull_idle_minutes"].as_int(1440), a["now_ms"].as_int(now_unix_ms()));
  });
  R.add("culling_check_period_has_passed", [](const Json& a) -> Json {
    return culling_check_period_has_passed(a["notebook"], a["period_s"].as_double(), a["now_ms"].as_int(now_unix_ms()));
  });
}

void register_profile(CapiRegistry& R) {
  R.add("set_namespace_labels", [](const Json& a) -> Json {
    Json ns = a["namespace"];
    std::map<std::string, std::string> l;
    for (const auto& m : a["labels"].as_object()) l[m.first] = m.second.as_string();
    set_namespace_labels(ns, l);
    return ns;
  });
  R.add("parse_flat_yaml_map", [](const Json& a) -> Json {
    bool ok = true;
    Json m = Json::object();
    for (const auto& kv : parse_flat_yaml_map(a["text"].as_string(), &ok)) m[kv.first] = kv.second;
    return Json{{"ok", ok}, {"map", m}};
  });
  R.add("get_issuer_url_from_provider_arn", [](const Json& a) -> Json { return get_issuer_url_from_provider_arn(a["arn"].as_string()); });
  R.add("get_iam_role_name_from_iam_role_arn", [](const Json& a) -> Json { return get_iam_role_name_from_iam_role_arn(a["arn"].as_string()); });
  R.add("add_service_account_in_assume_role_policy", [](const Json& a) -> Json {
    std::string out;
    bool exists = false;
    bool ch = add_service_account_in_assume_role_policy(a["doc"].as_string(), a["namespace"].as_string(), a["sa"].as_string(), out, &exists);
    return Json{{"changed", ch}, {"exists", exists}, {"doc", out}};
  });
  R.add("remove_service_account_in_assume_role_policy", [](const Json& a) -> Json {
    std::string out;
    bool ch = remove_service_account_in_assume_role_policy(a["doc"].as_string(), a["namespace"].as_string(), a["sa"].as_string(), out);
    return Json{{"changed", ch}, {"doc", out}};
  });
  R.add("gcp_project_id", [](const Json& a) -> Json { return gcp_project_id(a["sa"].as_string()); });
  R.add("gcp_add_binding", [](const Json& a) -> Json {
    Json p = a["policy"];
    gcp_add_binding(p, a["member"].as_string());
    return p;
  });
  R.add("gcp_revoke_binding", [](const Json& a) -> Json {
    Json p = a["policy"];
    gcp_revoke_binding(p, a["member"].as_string());
    return p;
  });
  R.add("authorization_policy_spec", [](const Json& a) -> Json {
    ProfileOptions o;
    if (a["userid_header"].is_string()) o.userid_header = a["userid_header"].as_string();
    if (a["userid_prefix"].is_string()) o.userid_prefix = a["userid_prefix"].as_string();
    return authorization_policy_spec(a["profile"], o);
  });
}

void register_admission(CapiRegistry& R) {
  R.add("merge_map", [](const Json& a) -> Json {
    Json out;
    std::string err;
    bool ok = merge_map(a["existing"], vec(a["defaults"]), out, &err);
    return Json{{"ok", ok}, {"out", out}, {"error", err}};
  });
  R.add("filter_pod_defaults", [](const Json& a) -> Json {
    Json out = Json::array();
    for (const auto& p : filter_pod_defaults(vec(a["poddefaults"]), a["pod"])) out.push_back(p);
    return out;
  });
  R.add("safe_to_apply_pod_defaults", [](const Json& a) -> Json { return safe_to_apply_pod_defaults(a["pod"], vec(a["poddefaults"])); });
  R.add("apply_pod_defaults", [](const Json& a) -> Json {
    Json pod = a["pod"];
    apply_pod_defaults(pod, vec(a["poddefaults"]));
    return pod;
  });
  R.add("set_command_and_args", [](const Json& a) -> Json {
    Json c = a["container"];
    set_command_and_args(c, vec(a["poddefaults"]));
    return c;
  });
  R.add("pod_quota_usage", [](const Json& a) -> Json {
    Json out = Json::object();
    for (const auto& kv : pod_quota_usage(a["pod"], a["hbm_gib_per_gpu"].as_int(288))) out[kv.first] = kv.second;
    return out;
  });
  R.add("gpu_readiness_mutate", [](const Json& a) -> Json {
    auto fn = make_gpu_readiness_plugin();
    Json pod = a["pod"];
    AdmissionAttrs at;
    at.operation = "CREATE";
    auto res = std::make_shared<ResourceInfo>();
    res->kind = "Pod";
    at.res = res;
    at.object = &pod;
    ApiError e = fn(at);
    if (e) throw std::runtime_error(e.message);
    return pod;
  });
}

void register_tensorboard(CapiRegistry& R) {
  R.add("tb_paths", [](const Json& a) -> Json {
    const std::string p = a["path"].as_string();
    return Json{{"cloud", tb_is_cloud_path(p)}, {"gcs", tb_is_gcs_path(p)}, {"pvc", tb_is_pvc_path(p)},
                {"pvc_name", tb_extract_pvc_name(p)}, {"pvc_subpath", tb_extract_pvc_subpath(p)}};
  });
  R.add("tb_generate_deployment", [](const Json& a) -> Json {
    return tb_generate_deployment(a["tensorboard"], a["image"].as_string(), preferred_node_affinity(a["node"].as_string()));
  });
  R.add("tb_generate_service", [](const Json& a) -> Json { return tb_generate_service(a["tensorboard"]); });
  R.add("tb_generate_virtual_service", [](const Json& a) -> Json {
    return tb_generate_virtual_service(a["tensorboard"], a["gateway"].as_string(), a["host"].as_string());
  });
  R.add("tb_copy_deployment_fields", [](const Json& a) -> Json {
    Json to = a["to"];
    bool ch = tb_copy_deployment_fields(a["from"], to);
    return Json{{"changed", ch}, {"to", to}};
  });
  R.add("tb_status", [](const Json& a) -> Json { return tb_status(a["tensorboard"], a["deployment"]); });
  R.add("pvcviewer_default", [](const Json& a) -> Json { return pvcviewer_default(a["viewer"], a["default_pod_spec"]); });
  R.add("pvcviewer_validate", [](const Json& a) -> Json { return pvcviewer_validate(a["viewer"]); });
  R.add("pvcviewer_generate_deployment", [](const Json& a) -> Json {
    return pvcviewer_generate_deployment(a["viewer"], preferred_node_affinity(a["node"].as_string()));
  });
  R.add("pvcviewer_generate_service", [](const Json& a) -> Json { return pvcviewer_generate_service(a["viewer"]); });
  R.add("pvcviewer_generate_virtual_service", [](const Json& a) -> Json {
    return pvcviewer_generate_virtual_service(a["viewer"], a["gateway"].as_string());
  });
  R.add("pvcviewer_rwo_node", [](const Json& a) -> Json { return pvcviewer_rwo_node(a["pvc"], vec(a["pods"])); });
}

void register_kfam(CapiRegistry& R) {
  R.add("kfam_binding_name", [](const Json& a) -> Json { return kfam_binding_name(a["binding"]); });
  R.add("kfam_role_map", [](const Json& a) -> Json { return kfam_role_map(a["role"].as_string()); });
  R.add("kfam_authorization_policy_spec", [](const Json& a) -> Json {
    return kfam_authorization_policy_spec(a["binding"], a["userid_header"].as_string(), a["userid_prefix"].as_string());
  });
}

void register_odh(CapiRegistry& R) {
  R.add("odh_flags", [](const Json& a) -> Json {
    const Json& nb = a["notebook"];
    return Json{{"oauth", odh_oauth_enabled(nb)}, {"mesh", odh_service_mesh_enabled(nb)}, {"lock", odh_lock_enabled(nb)}};
  });
  R.add("odh_inject_oauth_proxy", [](const Json& a) -> Json {
    Json nb = a["notebook"];
    odh_inject_oauth_proxy(nb, a["image"].as_string());
    return nb;
  });
  R.add("odh_inject_cert_config", [](const Json& a) -> Json {
    Json nb = a["notebook"];
    odh_inject_cert_config(nb, a["configmap"].as_string());
    return nb;
  });
  R.add("odh_unset_cert_config", [](const Json& a) -> Json {
    Json nb = a["notebook"];
    bool ch = odh_unset_cert_config(nb);
    return Json{{"changed", ch}, {"notebook", nb}};
  });
  R.add("odh_set_image_from_imagestreams", [](const Json& a) -> Json {
    Json nb = a["notebook"];
    std::string err = odh_set_image_from_imagestreams(nb, vec(a["imagestreams"]));
    return Json{{"error", err}, {"notebook", nb}};
  });
  R.add("json_first_difference", [](const Json& a) -> Json { return json_first_difference(a["a"], a["b"], a["type"].as_string()); });
  R.add("pem_certificate_valid", [](const Json& a) -> Json { return pem_certificate_valid(a["pem"].as_string()); });
  R.add("odh_objects", [](const Json& a) -> Json {
    const Json& nb = a["notebook"];
    return Json{{"network_policy", odh_network_policy(nb, a["controller_namespace"].as_string())},
                {"oauth_network_policy", odh_oauth_network_policy(nb)},
                {"route", odh_route(nb)},
                {"oauth_route", odh_oauth_route(nb)},
                {"service_account", odh_service_account(nb)},
                {"oauth_service", odh_oauth_service(nb)},
                {"oauth_secret", odh_oauth_secret(nb)}};
  });
}

void register_gpu(CapiRegistry& R) {
  R.add("cpulist_roundtrip", [](const Json& a) -> Json {
    auto v = parse_cpulist(a["s"].as_string());
    Json arr = Json::array();
    for (int c : v) arr.push_back(c);
    return Json{{"cpus", arr}, {"formatted", format_cpulist(v)}};
  });
  R.add("topology_synthetic", [](const Json& a) -> Json { return topo_from(a).to_json(); });
  R.add("topology_discover", [](const Json& a) -> Json {
    if (a["sysfs_root"].is_string()) {
      GpuTopology t = GpuTopology::discover(SysfsRoots::under(a["sysfs_root"].as_string()));
      Json j = t.to_json();
      j["describe"] = t.describe();
      Json lc = Json::array();
      for (int c : t.local_cpus({0})) lc.push_back(c);
      j["localCpusDevice0"] = lc;
      return j;
    }
    return a["root"].is_string() ? GpuTopology::discover(a["root"].as_string()).to_json() : GpuTopology::discover().to_json();
  });
  R.add("gpu_choose", [](const Json& a) -> Json {
    GpuTopology t = topo_from(a);
    std::set<int> free;
    if (a["free"].is_array()) {
      for (const auto& x : a["free"].as_array()) free.insert(static_cast<int>(x.as_int()));
    } else {
      for (int i = 0; i < t.size(); ++i) free.insert(i);
    }
    Placement p;
    if (!GpuAllocator::choose(t, free, static_cast<int>(a["n"].as_int()), p)) return Json();
    return placement_json(p);
  });
  R.add("gpu_allocate_sequence", [](const Json& a) -> Json {
    // [{"owner": "...", "n": 2} | {"release": "..."}] -> placements, exercising the allocator state
    GpuAllocator alloc(topo_from(a));
    Json out = Json::array();
    for (const auto& op : a["ops"].as_array()) {
      if (op["release"].is_string()) {
        alloc.release(op["release"].as_string());
        out.push_back(Json{{"released", op["release"]}, {"free", alloc.free_count()}});
        continue;
      }
      Placement p;
      bool ok = alloc.allocate(op["owner"].as_string(), static_cast<int>(op["n"].as_int()), p);
      Json r = ok ? placement_json(p) : Json::object();
      r["ok"] = ok;
      r["free"] = alloc.free_count();
      out.push_back(r);
    }
    return out;
  });
  R.add("gpu_env_for", [](const Json& a) -> Json {
    GpuTopology t = topo_from(a);
    Placement p;
    for (const auto& x : a["devices"].as_array()) p.devices.push_back(static_cast<int>(x.as_int()));
    p.ring = GpuAllocator::ring_order(t, p.devices);
    return gpu_env_for(p, t, p.devices.size() > 1);
  });
  // one AMD SMI telemetry sample (what the kubelet's collectors export), matched to the KFD topology
  R.add("smi_sample", [](const Json&) -> Json {
    Json devs = Json::array();
    for (const auto& t : AmdSmi::instance().sample()) {
      Json rd = Json::array(), wr = Json::array();
      for (int l = 0; l < t.xgmi_links; ++l) {
        rd.push_back(t.xgmi_read_bytes[l]);
        wr.push_back(t.xgmi_write_bytes[l]);
      }
      devs.push_back(Json{{"bdf", t.bdf}, {"gfx_activity", t.gfx_activity}, {"umc_activity", t.umc_activity},
                          {"power_w", t.power_w}, {"temp_hotspot_c", t.temp_hotspot_c}, {"temp_mem_c", t.temp_mem_c},
                          {"gfxclk_mhz", t.gfxclk_mhz}, {"energy_j", t.energy_j}, {"xgmi_read_bytes", rd},
                          {"xgmi_write_bytes", wr}, {"accumulation_counter", static_cast<double>(t.accumulation_counter)},
                          {"ppt_residency_acc", static_cast<double>(t.ppt_residency_acc)},
                          {"thermal_residency_acc", static_cast<double>(t.thermal_residency_acc)}});
    }
    Json buses = Json::array();
    for (const auto& g : GpuTopology::discover().gpus) buses.push_back(g.pci_bus);
    return Json{{"available", AmdSmi::instance().available()}, {"error", AmdSmi::instance().error()},
                {"devices", devs}, {"topology_buses", buses}};
  });
}

}  // namespace

CapiRegistry& CapiRegistry::global() {
  static CapiRegistry* r = [] {
    auto* reg = new CapiRegistry();
    register_core(*reg);
    register_notebook(*reg);
    register_profile(*reg);
    register_admission(*reg);
    register_gpu(*reg);
    register_tensorboard(*reg);
    register_kfam(*reg);
    register_odh(*reg);
    for (auto& ext : capi_extensions()) ext(*reg);
    return reg;
  }();
  return *r;
}

std::vector<std::function<void(CapiRegistry&)>>& capi_extensions() {
  static std::vector<std::function<void(CapiRegistry&)>> v;
  return v;
}

}  // namespace kf

extern "C" {

char* kf_call(const char* name, const char* args_json) {
  kf::Json out;
  try {
    kf::Json args;
    std::string perr;
    if (args_json && *args_json && !kf::Json::try_parse(args_json, args, &perr)) throw std::runtime_error("bad args json: " + perr);
    auto& R = kf::CapiRegistry::global();
    auto it = R.fns.find(name ? name : "");
    if (it == R.fns.end()) throw std::runtime_error(std::string("unknown function: ") + (name ? name : ""));
    out = kf::Json{{"ok", true}, {"result", it->second(args)}};
  } catch (const std::exception& e) {
    out = kf::Json{{"ok", false}, {"error", e.what()}};
  }
  const std::string s = out.dump();
  char* buf = static_cast<char*>(std::malloc(s.size() + 1));
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return buf;
}

void kf_free(char* p) { std::free(p); }

char* kf_functions() {
  kf::Json names = kf::Json::array();
  for (const auto& kv : kf::CapiRegistry::global().fns) names.push_back(kv.first);
  const std::string s = names.dump();
  char* buf = static_cast<char*>(std::malloc(s.size() + 1));
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return buf;
}

}  // extern "C"
