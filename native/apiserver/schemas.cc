// schemas.cc — see schemas.h.
#include "apiserver/schemas.h"

#include <utility>

#include "core/util.h"

namespace kf {

const char* const kQuantityPattern =
    "^(\\+|-)?(([0-9]+(\\.[0-9]*)?)|(\\.[0-9]+))(([KMGTPE]i)|[numkMGTPE]|([eE](\\+|-)?(([0-9]+(\\.[0-9]*)?)|(\\.[0-9]+))))?$";

namespace {
using Props = std::vector<std::pair<std::string, Json>>;

Json T(const char* t) { return Json{{"type", t}}; }
Json str() { return T("string"); }
Json boolean() { return T("boolean"); }
Json i32() { return Json{{"type", "integer"}, {"format", "int32"}}; }
Json i64() { return Json{{"type", "integer"}, {"format", "int64"}}; }
Json date_time() { return Json{{"type", "string"}, {"format", "date-time"}}; }
Json int_or_string() {
  return Json{{"anyOf", Json::array({T("integer"), T("string")})}, {"x-kubernetes-int-or-string", true}};
}
Json quantity() {
  Json q = int_or_string();
  q["pattern"] = kQuantityPattern;
  return q;
}
Json arr(Json item) { return Json{{"type", "array"}, {"items", std::move(item)}}; }
Json str_arr() { return arr(str()); }
Json atomic_list(Json a) {
  a["x-kubernetes-list-type"] = "atomic";
  return a;
}
Json list_map(Json a, std::vector<std::string> keys) {
  Json k = Json::array();
  for (auto& x : keys) k.push_back(x);
  a["x-kubernetes-list-map-keys"] = k;
  a["x-kubernetes-list-type"] = "map";
  return a;
}
Json obj(const Props& props, const std::vector<std::string>& required = {}) {
  Json p = Json::object();
  for (const auto& kv : props) p[kv.first] = kv.second;
  Json s{{"type", "object"}, {"properties", p}};
  if (!required.empty()) {
    Json r = Json::array();
    for (const auto& x : required) r.push_back(x);
    s["required"] = r;
  }
  return s;
}
Json atomic(Json s) {
  s["x-kubernetes-map-type"] = "atomic";
  return s;
}
Json map_of(Json v) { return Json{{"type", "object"}, {"additionalProperties", std::move(v)}}; }
Json free_object() { return Json{{"type", "object"}, {"x-kubernetes-preserve-unknown-fields", true}}; }
Json with_default(Json s, Json d) {
  s["default"] = std::move(d);
  return s;
}

// ---- shared core/v1 pieces -------------------------------------------------------------------
Json local_object_ref() { return atomic(obj({{"name", str()}})); }
Json label_selector() {
  Json req = obj({{"key", str()}, {"operator", str()}, {"values", atomic_list(str_arr())}}, {"key", "operator"});
  return atomic(obj({{"matchExpressions", atomic_list(arr(req))}, {"matchLabels", map_of(str())}}));
}
Json key_selector() { return atomic(obj({{"key", str()}, {"name", str()}, {"optional", boolean()}}, {"key"})); }
Json field_ref() { return atomic(obj({{"apiVersion", str()}, {"fieldPath", str()}}, {"fieldPath"})); }
Json resource_field_ref() {
  return atomic(obj({{"containerName", str()}, {"divisor", quantity()}, {"resource", str()}}, {"resource"}));
}
Json env_var() {
  return obj({{"name", str()},
              {"value", str()},
              {"valueFrom", obj({{"configMapKeyRef", key_selector()},
                                 {"fieldRef", field_ref()},
                                 {"resourceFieldRef", resource_field_ref()},
                                 {"secretKeyRef", key_selector()}})}},
             {"name"});
}
Json env_from() {
  Json ref = atomic(obj({{"name", str()}, {"optional", boolean()}}));
  return obj({{"configMapRef", ref}, {"prefix", str()}, {"secretRef", ref}});
}
Json http_get() {
  Json header = obj({{"name", str()}, {"value", str()}}, {"name", "value"});
  return obj({{"host", str()}, {"httpHeaders", atomic_list(arr(header))}, {"path", str()}, {"port", int_or_string()},
              {"scheme", str()}},
             {"port"});
}
Json exec_action() { return obj({{"command", atomic_list(str_arr())}}); }
Json tcp_socket() { return obj({{"host", str()}, {"port", int_or_string()}}, {"port"}); }
Json lifecycle_handler() {
  return obj({{"exec", exec_action()},
              {"httpGet", http_get()},
              {"sleep", obj({{"seconds", i64()}}, {"seconds"})},
              {"tcpSocket", tcp_socket()}});
}
Json probe() {
  return obj({{"exec", exec_action()},
              {"failureThreshold", i32()},
              {"grpc", obj({{"port", i32()}, {"service", with_default(str(), "")}}, {"port"})},
              {"httpGet", http_get()},
              {"initialDelaySeconds", i32()},
              {"periodSeconds", i32()},
              {"successThreshold", i32()},
              {"tcpSocket", tcp_socket()},
              {"terminationGracePeriodSeconds", i64()},
              {"timeoutSeconds", i32()}});
}
Json resource_requirements() {
  Json claim = obj({{"name", str()}, {"request", str()}}, {"name"});
  return obj({{"claims", list_map(arr(claim), {"name"})}, {"limits", map_of(quantity())}, {"requests", map_of(quantity())}});
}
Json se_linux_options() { return obj({{"level", str()}, {"role", str()}, {"type", str()}, {"user", str()}}); }
Json profile_ref() { return obj({{"localhostProfile", str()}, {"type", str()}}, {"type"}); }
Json windows_options() {
  return obj({{"gmsaCredentialSpec", str()}, {"gmsaCredentialSpecName", str()}, {"hostProcess", boolean()},
              {"runAsUserName", str()}});
}
Json security_context() {
  return obj({{"allowPrivilegeEscalation", boolean()},
              {"appArmorProfile", profile_ref()},
              {"capabilities", obj({{"add", atomic_list(str_arr())}, {"drop", atomic_list(str_arr())}})},
              {"privileged", boolean()},
              {"procMount", str()},
              {"readOnlyRootFilesystem", boolean()},
              {"runAsGroup", i64()},
              {"runAsNonRoot", boolean()},
              {"runAsUser", i64()},
              {"seLinuxOptions", se_linux_options()},
              {"seccompProfile", profile_ref()},
              {"windowsOptions", windows_options()}});
}
Json volume_mount() {
  return obj({{"mountPath", str()}, {"mountPropagation", str()}, {"name", str()}, {"readOnly", boolean()},
              {"recursiveReadOnly", str()}, {"subPath", str()}, {"subPathExpr", str()}},
             {"mountPath", "name"});
}
Json container_port() {
  return obj({{"containerPort", i32()}, {"hostIP", str()}, {"hostPort", i32()}, {"name", str()},
              {"protocol", with_default(str(), "TCP")}},
             {"containerPort"});
}

// Container / EphemeralContainer (ephemeral adds targetContainerName)
Json container(bool ephemeral) {
  Props p = {{"args", atomic_list(str_arr())},
             {"command", atomic_list(str_arr())},
             {"env", list_map(arr(env_var()), {"name"})},
             {"envFrom", atomic_list(arr(env_from()))},
             {"image", str()},
             {"imagePullPolicy", str()},
             {"lifecycle", obj({{"postStart", lifecycle_handler()}, {"preStop", lifecycle_handler()}})},
             {"livenessProbe", probe()},
             {"name", str()},
             {"ports", list_map(arr(container_port()), {"containerPort", "protocol"})},
             {"readinessProbe", probe()},
             {"resizePolicy", atomic_list(arr(obj({{"resourceName", str()}, {"restartPolicy", str()}},
                                                  {"resourceName", "restartPolicy"})))},
             {"resources", resource_requirements()},
             {"restartPolicy", str()},
             {"securityContext", security_context()},
             {"startupProbe", probe()},
             {"stdin", boolean()},
             {"stdinOnce", boolean()},
             {"terminationMessagePath", str()},
             {"terminationMessagePolicy", str()},
             {"tty", boolean()},
             {"volumeDevices", list_map(arr(obj({{"devicePath", str()}, {"name", str()}}, {"devicePath", "name"})), {"devicePath"})},
             {"volumeMounts", list_map(arr(volume_mount()), {"mountPath"})},
             {"workingDir", str()}};
  if (ephemeral) p.push_back({"targetContainerName", str()});
  return obj(p, {"name"});
}

Json node_selector_term() {
  Json req = obj({{"key", str()}, {"operator", str()}, {"values", atomic_list(str_arr())}}, {"key", "operator"});
  return atomic(obj({{"matchExpressions", atomic_list(arr(req))}, {"matchFields", atomic_list(arr(req))}}));
}
Json pod_affinity_term() {
  return obj({{"labelSelector", label_selector()},
              {"matchLabelKeys", atomic_list(str_arr())},
              {"mismatchLabelKeys", atomic_list(str_arr())},
              {"namespaceSelector", label_selector()},
              {"namespaces", atomic_list(str_arr())},
              {"topologyKey", str()}},
             {"topologyKey"});
}
Json pod_affinity() {
  Json weighted = obj({{"podAffinityTerm", pod_affinity_term()}, {"weight", i32()}}, {"podAffinityTerm", "weight"});
  return obj({{"preferredDuringSchedulingIgnoredDuringExecution", atomic_list(arr(weighted))},
              {"requiredDuringSchedulingIgnoredDuringExecution", atomic_list(arr(pod_affinity_term()))}});
}
Json affinity() {
  Json pref = obj({{"preference", node_selector_term()}, {"weight", i32()}}, {"preference", "weight"});
  Json node = obj({{"preferredDuringSchedulingIgnoredDuringExecution", atomic_list(arr(pref))},
                   {"requiredDuringSchedulingIgnoredDuringExecution",
                    atomic(obj({{"nodeSelectorTerms", atomic_list(arr(node_selector_term()))}}, {"nodeSelectorTerms"}))}});
  return obj({{"nodeAffinity", node}, {"podAffinity", pod_affinity()}, {"podAntiAffinity", pod_affinity()}});
}
Json toleration() {
  return obj({{"effect", str()}, {"key", str()}, {"operator", str()}, {"tolerationSeconds", i64()}, {"value", str()}});
}
Json pod_security_context() {
  return obj({{"appArmorProfile", profile_ref()},
              {"fsGroup", i64()},
              {"fsGroupChangePolicy", str()},
              {"runAsGroup", i64()},
              {"runAsNonRoot", boolean()},
              {"runAsUser", i64()},
              {"seLinuxOptions", se_linux_options()},
              {"seccompProfile", profile_ref()},
              {"supplementalGroups", atomic_list(arr(i64()))},
              {"supplementalGroupsPolicy", str()},
              {"sysctls", atomic_list(arr(obj({{"name", str()}, {"value", str()}}, {"name", "value"})))},
              {"windowsOptions", windows_options()}});
}
Json key_to_path() { return obj({{"key", str()}, {"mode", i32()}, {"path", str()}}, {"key", "path"}); }
Json downward_file() {
  return obj({{"fieldRef", field_ref()}, {"mode", i32()}, {"path", str()}, {"resourceFieldRef", resource_field_ref()}},
             {"path"});
}
Json pvc_spec() {
  Json tref = atomic(obj({{"apiGroup", str()}, {"kind", str()}, {"name", str()}}, {"kind", "name"}));
  return obj({{"accessModes", atomic_list(str_arr())},
              {"dataSource", tref},
              {"dataSourceRef", obj({{"apiGroup", str()}, {"kind", str()}, {"name", str()}, {"namespace", str()}},
                                    {"kind", "name"})},
              {"resources", obj({{"limits", map_of(quantity())}, {"requests", map_of(quantity())}})},
              {"selector", label_selector()},
              {"storageClassName", str()},
              {"volumeAttributesClassName", str()},
              {"volumeMode", str()},
              {"volumeName", str()}});
}
// every volume source of core/v1 Volume, the legacy in-tree plugins included (they are still API)
Json volume() {
  const Json ref = local_object_ref();
  const Json fs = str(), ro = boolean();
  Props p = {
      {"awsElasticBlockStore", obj({{"fsType", fs}, {"partition", i32()}, {"readOnly", ro}, {"volumeID", str()}}, {"volumeID"})},
      {"azureDisk", obj({{"cachingMode", str()}, {"diskName", str()}, {"diskURI", str()}, {"fsType", with_default(str(), "ext4")},
                         {"kind", str()}, {"readOnly", with_default(boolean(), false)}},
                        {"diskName", "diskURI"})},
      {"azureFile", obj({{"readOnly", ro}, {"secretName", str()}, {"shareName", str()}}, {"secretName", "shareName"})},
      {"cephfs", obj({{"monitors", atomic_list(str_arr())}, {"path", str()}, {"readOnly", ro}, {"secretFile", str()},
                      {"secretRef", ref}, {"user", str()}},
                     {"monitors"})},
      {"cinder", obj({{"fsType", fs}, {"readOnly", ro}, {"secretRef", ref}, {"volumeID", str()}}, {"volumeID"})},
      {"configMap", atomic(obj({{"defaultMode", i32()}, {"items", atomic_list(arr(key_to_path()))}, {"name", str()},
                                {"optional", boolean()}}))},
      {"csi", obj({{"driver", str()}, {"fsType", fs}, {"nodePublishSecretRef", ref}, {"readOnly", ro},
                   {"volumeAttributes", map_of(str())}},
                  {"driver"})},
      {"downwardAPI", obj({{"defaultMode", i32()}, {"items", atomic_list(arr(downward_file()))}})},
      {"emptyDir", obj({{"medium", str()}, {"sizeLimit", quantity()}})},
      {"ephemeral", obj({{"volumeClaimTemplate", obj({{"metadata", T("object")}, {"spec", pvc_spec()}}, {"spec"})}})},
      {"fc", obj({{"fsType", fs}, {"lun", i32()}, {"readOnly", ro}, {"targetWWNs", atomic_list(str_arr())},
                  {"wwids", atomic_list(str_arr())}})},
      {"flexVolume", obj({{"driver", str()}, {"fsType", fs}, {"options", map_of(str())}, {"readOnly", ro}, {"secretRef", ref}},
                         {"driver"})},
      {"flocker", obj({{"datasetName", str()}, {"datasetUUID", str()}})},
      {"gcePersistentDisk", obj({{"fsType", fs}, {"partition", i32()}, {"pdName", str()}, {"readOnly", ro}}, {"pdName"})},
      {"gitRepo", obj({{"directory", str()}, {"repository", str()}, {"revision", str()}}, {"repository"})},
      {"glusterfs", obj({{"endpoints", str()}, {"path", str()}, {"readOnly", ro}}, {"endpoints", "path"})},
      {"hostPath", obj({{"path", str()}, {"type", str()}}, {"path"})},
      {"image", obj({{"pullPolicy", str()}, {"reference", str()}})},
      {"iscsi", obj({{"chapAuthDiscovery", boolean()}, {"chapAuthSession", boolean()}, {"fsType", fs},
                     {"initiatorName", str()}, {"iqn", str()}, {"iscsiInterface", with_default(str(), "default")},
                     {"lun", i32()}, {"portals", atomic_list(str_arr())}, {"readOnly", ro}, {"secretRef", ref},
                     {"targetPortal", str()}},
                    {"iqn", "lun", "targetPortal"})},
      {"name", str()},
      {"nfs", obj({{"path", str()}, {"readOnly", ro}, {"server", str()}}, {"path", "server"})},
      {"persistentVolumeClaim", obj({{"claimName", str()}, {"readOnly", ro}}, {"claimName"})},
      {"photonPersistentDisk", obj({{"fsType", fs}, {"pdID", str()}}, {"pdID"})},
      {"portworxVolume", obj({{"fsType", fs}, {"readOnly", ro}, {"volumeID", str()}}, {"volumeID"})},
      {"projected",
       obj({{"defaultMode", i32()},
            {"sources",
             atomic_list(arr(obj({{"clusterTrustBundle", obj({{"labelSelector", label_selector()}, {"name", str()},
                                                              {"optional", boolean()}, {"path", str()}, {"signerName", str()}},
                                                             {"path"})},
                                  {"configMap", atomic(obj({{"items", atomic_list(arr(key_to_path()))}, {"name", str()},
                                                            {"optional", boolean()}}))},
                                  {"downwardAPI", obj({{"items", atomic_list(arr(downward_file()))}})},
                                  {"secret", atomic(obj({{"items", atomic_list(arr(key_to_path()))}, {"name", str()},
                                                         {"optional", boolean()}}))},
                                  {"serviceAccountToken",
                                   obj({{"audience", str()}, {"expirationSeconds", i64()}, {"path", str()}}, {"path"})}})))}})},
      {"quobyte", obj({{"group", str()}, {"readOnly", ro}, {"registry", str()}, {"tenant", str()}, {"user", str()},
                       {"volume", str()}},
                      {"registry", "volume"})},
      {"rbd", obj({{"fsType", fs}, {"image", str()}, {"keyring", with_default(str(), "/etc/ceph/keyring")},
                   {"monitors", atomic_list(str_arr())}, {"pool", with_default(str(), "rbd")}, {"readOnly", ro},
                   {"secretRef", ref}, {"user", with_default(str(), "admin")}},
                  {"image", "monitors"})},
      {"scaleIO", obj({{"fsType", with_default(str(), "xfs")}, {"gateway", str()}, {"protectionDomain", str()},
                       {"readOnly", ro}, {"secretRef", ref}, {"sslEnabled", boolean()},
                       {"storageMode", with_default(str(), "ThinProvisioned")}, {"storagePool", str()}, {"system", str()},
                       {"volumeName", str()}},
                      {"gateway", "secretRef", "system"})},
      {"secret", obj({{"defaultMode", i32()}, {"items", atomic_list(arr(key_to_path()))}, {"optional", boolean()},
                      {"secretName", str()}})},
      {"storageos", obj({{"fsType", fs}, {"readOnly", ro}, {"secretRef", ref}, {"volumeName", str()},
                         {"volumeNamespace", str()}})},
      {"vsphereVolume", obj({{"fsType", fs}, {"storagePolicyID", str()}, {"storagePolicyName", str()}, {"volumePath", str()}},
                            {"volumePath"})}};
  return obj(p, {"name"});
}

Json status_condition(const Props& extra, const std::vector<std::string>& required) {
  Props p = {{"message", str()}, {"reason", str()}, {"status", str()}, {"type", str()}};
  for (const auto& e : extra) p.push_back(e);
  return obj(p, required);
}

Json root(Json spec, Json status) {
  Props p = {{"apiVersion", str()}, {"kind", str()}, {"metadata", T("object")}, {"spec", std::move(spec)}};
  if (!status.is_null()) p.push_back({"status", std::move(status)});
  return obj(p);
}
}  // namespace

Json pod_spec_schema() {
  Json c = container(false);
  Json containers = list_map(arr(c), {"name"});
  return obj(
      {{"activeDeadlineSeconds", i64()},
       {"affinity", affinity()},
       {"automountServiceAccountToken", boolean()},
       {"containers", containers},
       {"dnsConfig", obj({{"nameservers", atomic_list(str_arr())},
                          {"options", atomic_list(arr(obj({{"name", str()}, {"value", str()}})))},
                          {"searches", atomic_list(str_arr())}})},
       {"dnsPolicy", str()},
       {"enableServiceLinks", boolean()},
       {"ephemeralContainers", list_map(arr(container(true)), {"name"})},
       {"hostAliases", list_map(arr(obj({{"hostnames", atomic_list(str_arr())}, {"ip", str()}}, {"ip"})), {"ip"})},
       {"hostIPC", boolean()},
       {"hostNetwork", boolean()},
       {"hostPID", boolean()},
       {"hostUsers", boolean()},
       {"hostname", str()},
       {"imagePullSecrets", list_map(arr(local_object_ref()), {"name"})},
       {"initContainers", list_map(arr(c), {"name"})},
       {"nodeName", str()},
       {"nodeSelector", atomic(map_of(str()))},
       {"os", obj({{"name", str()}}, {"name"})},
       {"overhead", map_of(quantity())},
       {"preemptionPolicy", str()},
       {"priority", i32()},
       {"priorityClassName", str()},
       {"readinessGates", atomic_list(arr(obj({{"conditionType", str()}}, {"conditionType"})))},
       {"resourceClaims",
        list_map(arr(obj({{"name", str()},
                          {"resourceClaimName", str()},
                          {"resourceClaimTemplateName", str()},
                          {"source", obj({{"resourceClaimName", str()}, {"resourceClaimTemplateName", str()}})}},
                         {"name"})),
                 {"name"})},
       {"resources", obj({{"claims", list_map(arr(obj({{"name", str()}, {"request", str()}}, {"name"})), {"name"})},
                          {"limits", map_of(quantity())},
                          {"requests", map_of(quantity())}})},
       {"restartPolicy", str()},
       {"runtimeClassName", str()},
       {"schedulerName", str()},
       {"schedulingGates", list_map(arr(obj({{"name", str()}}, {"name"})), {"name"})},
       {"securityContext", pod_security_context()},
       {"serviceAccount", str()},
       {"serviceAccountName", str()},
       {"setHostnameAsFQDN", boolean()},
       {"shareProcessNamespace", boolean()},
       {"subdomain", str()},
       {"terminationGracePeriodSeconds", i64()},
       {"tolerations", atomic_list(arr(toleration()))},
       {"topologySpreadConstraints",
        list_map(arr(obj({{"labelSelector", label_selector()},
                          {"matchLabelKeys", atomic_list(str_arr())},
                          {"maxSkew", i32()},
                          {"minDomains", i32()},
                          {"nodeAffinityPolicy", str()},
                          {"nodeTaintsPolicy", str()},
                          {"topologyKey", str()},
                          {"whenUnsatisfiable", str()}},
                         {"maxSkew", "topologyKey", "whenUnsatisfiable"})),
                 {"topologyKey", "whenUnsatisfiable"})},
       {"volumes", list_map(arr(volume()), {"name"})}},
      {"containers"});
}

Json notebook_schema() {
  // validation_patches.yaml: containers minItems 1, container name + image required
  Json ps = pod_spec_schema();
  Json& cs = ps["properties"]["containers"];
  cs["minItems"] = 1;
  cs["items"]["required"] = Json::array({"name", "image"});
  // template.metadata (labels / annotations for the pod) is an embedded ObjectMeta: kept whole
  Json spec = obj({{"template", obj({{"metadata", free_object()}, {"spec", ps}})}});
  Json cstate = obj({{"running", obj({{"startedAt", date_time()}})},
                     {"terminated", obj({{"containerID", str()}, {"exitCode", i32()}, {"finishedAt", date_time()},
                                         {"message", str()}, {"reason", str()}, {"signal", i32()}, {"startedAt", date_time()}},
                                        {"exitCode"})},
                     {"waiting", obj({{"message", str()}, {"reason", str()}})}});
  Json status = obj({{"conditions", arr(status_condition({{"lastProbeTime", date_time()}, {"lastTransitionTime", date_time()}},
                                                         {"status", "type"}))},
                     {"containerState", cstate},
                     {"readyReplicas", i32()},
                     // MI355X additions: devices held by the pod and the in-pod readiness op's report
                     {"gpus", str()},
                     {"gpuReadiness", free_object()}},
                    {"conditions", "containerState", "readyReplicas"});
  return root(spec, status);
}

Json pvcviewer_schema() {
  Json spec = obj({{"networking", obj({{"basePrefix", str()}, {"rewrite", str()}, {"targetPort", int_or_string()},
                                       {"timeout", str()}})},
                   {"podSpec", pod_spec_schema()},
                   {"pvc", str()},
                   {"rwoScheduling", with_default(boolean(), false)}},
                  {"pvc", "rwoScheduling"});
  Json status = obj({{"conditions", arr(status_condition({{"lastTransitionTime", date_time()}, {"lastUpdateTime", date_time()}},
                                                         {"status", "type"}))},
                     {"ready", with_default(boolean(), false)},
                     {"url", str()}},
                    {"ready"});
  return root(spec, status);
}

Json poddefault_schema() {
  Json spec = obj({{"annotations", map_of(str())},
                   {"args", atomic_list(str_arr())},
                   {"automountServiceAccountToken", boolean()},
                   {"command", atomic_list(str_arr())},
                   {"desc", str()},
                   {"env", arr(env_var())},
                   {"envFrom", arr(env_from())},
                   {"imagePullSecrets", arr(local_object_ref())},
                   {"initContainers", arr(container(false))},
                   {"labels", map_of(str())},
                   {"selector", label_selector()},
                   {"serviceAccountName", str()},
                   {"sidecars", arr(container(false))},
                   {"tolerations", arr(toleration())},
                   {"volumeMounts", arr(volume_mount())},
                   {"volumes", arr(volume())}},
                  {"selector"});
  return root(spec, T("object"));
}

Json profile_schema() {
  Json spec = obj(
      {{"owner", atomic(obj({{"apiGroup", str()}, {"kind", str()}, {"name", str()}, {"namespace", str()}}, {"kind", "name"}))},
       {"plugins", arr(obj({{"apiVersion", str()}, {"kind", str()}, {"spec", free_object()}}))},
       {"resourceQuotaSpec",
        obj({{"hard", map_of(quantity())},
             {"scopeSelector",
              atomic(obj({{"matchExpressions",
                           atomic_list(arr(obj({{"operator", str()}, {"scopeName", str()}, {"values", atomic_list(str_arr())}},
                                               {"operator", "scopeName"})))}}))},
             {"scopes", atomic_list(str_arr())}})}});
  Json status = obj({{"conditions", arr(obj({{"message", str()}, {"status", str()}, {"type", str()}}))}});
  return root(spec, status);
}

Json tensorboard_schema() {
  Json spec = obj({{"logspath", str()}}, {"logspath"});
  Json status = obj({{"conditions", arr(obj({{"deploymentState", str()}, {"lastProbeTime", date_time()}}, {"deploymentState"}))},
                     {"readyReplicas", i32()}},
                    {"conditions", "readyReplicas"});
  return root(spec, status);
}

// ---- structural semantics ---------------------------------------------------------------------
void prune_unknown_fields(const Json& schema, Json& value, std::vector<std::string>* pruned, const std::string& path) {
  if (!schema.is_object()) return;
  if (value.is_array()) {
    const Json& items = schema["items"];
    if (!items.is_object()) return;
    size_t i = 0;
    for (auto& v : value.mut_array()) prune_unknown_fields(items, v, pruned, path + "[" + std::to_string(i++) + "]");
    return;
  }
  if (!value.is_object()) return;
  const bool preserve = schema["x-kubernetes-preserve-unknown-fields"].as_bool();
  const Json& props = schema["properties"];
  const Json& addl = schema["additionalProperties"];
  std::vector<std::string> drop;
  for (auto& m : value.mut_object()) {
    const std::string sub = path.empty() ? m.first : path + "." + m.first;
    if (path.empty() && (m.first == "apiVersion" || m.first == "kind" || m.first == "metadata")) continue;
    if (const Json* ps = props.find(m.first)) {
      prune_unknown_fields(*ps, m.second, pruned, sub);
    } else if (addl.is_object()) {
      prune_unknown_fields(addl, m.second, pruned, sub);
    } else if (!preserve && !addl.as_bool()) {
      drop.push_back(m.first);
      if (pruned) pruned->push_back(sub);
    }
  }
  for (const auto& k : drop) value.erase(k);
}

void apply_schema_defaults(const Json& schema, Json& value) {
  if (!schema.is_object()) return;
  if (value.is_array()) {
    if (schema["items"].is_object())
      for (auto& v : value.mut_array()) apply_schema_defaults(schema["items"], v);
    return;
  }
  if (!value.is_object()) return;
  for (const auto& p : schema["properties"].as_object()) {
    if (!value.has(p.first)) {
      if (p.second.has("default")) value[p.first] = p.second["default"];
      continue;
    }
    apply_schema_defaults(p.second, value[p.first]);
  }
  if (schema["additionalProperties"].is_object())
    for (auto& m : value.mut_object()) apply_schema_defaults(schema["additionalProperties"], m.second);
}

}  // namespace kf
