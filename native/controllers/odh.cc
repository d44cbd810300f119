// odh.cc — N8 OpenshiftNotebookReconciler + N9 ODH NotebookWebhook (see odh.h).
#include "controllers/odh.h"

#include <openssl/bio.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/x509.h>

#include <algorithm>
#include <cctype>

#include "controllers/common.h"
#include "core/util.h"

namespace kf {

// ---- annotation predicates ------------------------------------------------------------------------
bool odh_bool_annotation(const Json& obj, const std::string& key) {
  const std::string v = annotation(obj, key);
  return v == "1" || v == "t" || v == "T" || v == "true" || v == "TRUE" || v == "True";
}
bool odh_oauth_enabled(const Json& nb) { return odh_bool_annotation(nb, ODH_ANNOTATION_INJECT_OAUTH); }
bool odh_service_mesh_enabled(const Json& nb) { return odh_bool_annotation(nb, ODH_ANNOTATION_SERVICE_MESH); }
bool odh_lock_enabled(const Json& nb) { return annotation(nb, STOP_ANNOTATION) == ODH_LOCK_VALUE; }

void odh_inject_lock(Json& nb) { set_annotation(nb, STOP_ANNOTATION, ODH_LOCK_VALUE); }

namespace {
// replace the element whose name matches, else append
void upsert_named(Json& list, const Json& item) {
  if (!list.is_array()) list = Json::array();
  for (auto& e : list.mut_array())
    if (e["name"] == item["name"]) {
      e = item;
      return;
    }
  list.push_back(item);
}

Json probe_oauth(int initial_delay) {
  return Json{{"httpGet", Json{{"path", "/oauth/healthz"}, {"port", "oauth-proxy"}, {"scheme", "HTTPS"}}},
              {"initialDelaySeconds", initial_delay},
              {"timeoutSeconds", 1},
              {"periodSeconds", 5},
              {"successThreshold", 1},
              {"failureThreshold", 3}};
}

const char* kCertMountPath = "/etc/pki/tls/custom-certs/ca-bundle.crt";
const std::vector<std::string> kCertEnv = {"GIT_SSL_CAINFO", "PIPELINES_SSL_SA_CERTS", "PIP_CERT", "REQUESTS_CA_BUNDLE",
                                           "SSL_CERT_FILE"};

std::string go_field(const std::string& k) {
  if (k.empty()) return k;
  std::string s = k;
  s[0] = static_cast<char>(std::toupper(static_cast<unsigned char>(s[0])));
  return s;
}
std::string go_value(const Json& v) {
  if (v.is_null()) return "<nil>";
  if (v.is_string()) return v.as_string();
  return v.dump();
}
bool first_diff(const Json& a, const Json& b, std::string path, std::string& out) {
  if (a == b) return false;
  if (a.is_object() && b.is_object()) {
    std::vector<std::string> keys;
    for (const auto& kv : a.as_object()) keys.push_back(kv.first);
    for (const auto& kv : b.as_object())
      if (!a.has(kv.first)) keys.push_back(kv.first);
    for (const auto& k : keys) {
      const Json* x = a.find(k);
      const Json* y = b.find(k);
      static const Json null;
      if (first_diff(x ? *x : null, y ? *y : null, path + "." + go_field(k), out)) return true;
    }
    return false;
  }
  if (a.is_array() && b.is_array() && a.size() == b.size()) {
    for (size_t i = 0; i < a.size(); ++i)
      if (first_diff(a[i], b[i], path + "[" + std::to_string(i) + "]", out)) return true;
    return false;
  }
  out = path + ": " + go_value(a) + " != " + go_value(b);
  return true;
}
}  // namespace

std::string json_first_difference(const Json& a, const Json& b, const std::string& root_type) {
  std::string out;
  first_diff(a, b, "{" + root_type + "}", out);
  return out;
}

void odh_inject_oauth_proxy(Json& nb, const std::string& image) {
  const std::string name = nb.str_at({"metadata", "name"});
  Json args = Json::array({"--provider=openshift", "--https-address=:8443", "--http-address=", "--openshift-service-account=" + name,
                           "--cookie-secret-file=/etc/oauth/config/cookie_secret", "--cookie-expire=24h0m0s",
                           "--tls-cert=/etc/tls/private/tls.crt", "--tls-key=/etc/tls/private/tls.key",
                           "--upstream=http://localhost:8888",
                           "--upstream-ca=/var/run/secrets/kubernetes.io/serviceaccount/ca.crt", "--email-domain=*",
                           "--skip-provider-button",
                           "--openshift-sar={\"verb\":\"get\",\"resource\":\"notebooks\",\"resourceAPIGroup\":\"kubeflow.org\","
                           "\"resourceName\":\"" +
                               name + "\",\"namespace\":\"$(NAMESPACE)\"}"});
  const std::string logout = annotation(nb, ODH_ANNOTATION_LOGOUT_URL);
  if (!logout.empty()) args.push_back("--logout-url=" + logout);
  Json res{{"cpu", "100m"}, {"memory", "64Mi"}};
  Json proxy{{"name", "oauth-proxy"},
             {"image", image},
             {"imagePullPolicy", "Always"},
             {"env", Json::array({Json{{"name", "NAMESPACE"}, {"valueFrom", Json{{"fieldRef", Json{{"fieldPath", "metadata.namespace"}}}}}}})},
             {"args", args},
             {"ports", Json::array({Json{{"name", "oauth-proxy"}, {"containerPort", 8443}, {"protocol", "TCP"}}})},
             {"livenessProbe", probe_oauth(30)},
             {"readinessProbe", probe_oauth(5)},
             {"resources", Json{{"requests", res}, {"limits", res}}},
             {"volumeMounts", Json::array({Json{{"name", "oauth-config"}, {"mountPath", "/etc/oauth/config"}},
                                           Json{{"name", "tls-certificates"}, {"mountPath", "/etc/tls/private"}}})}};
  Json& spec = nb["spec"]["template"]["spec"];
  upsert_named(spec["containers"], proxy);
  upsert_named(spec["volumes"], Json{{"name", "oauth-config"}, {"secret", Json{{"secretName", name + "-oauth-config"}, {"defaultMode", 420}}}});
  upsert_named(spec["volumes"], Json{{"name", "tls-certificates"}, {"secret", Json{{"secretName", name + "-tls"}, {"defaultMode", 420}}}});
  spec["serviceAccountName"] = name;
}

void odh_inject_cert_config(Json& nb, const std::string& cm) {
  const std::string name = nb.str_at({"metadata", "name"});
  Json& spec = nb["spec"]["template"]["spec"];
  upsert_named(spec["volumes"], Json{{"name", "trusted-ca"},
                                     {"configMap", Json{{"name", cm},
                                                        {"optional", true},
                                                        {"items", Json::array({Json{{"key", "ca-bundle.crt"}, {"path", "ca-bundle.crt"}}})}}}});
  for (auto& c : spec["containers"].mut_array()) {
    if (static_cast<const Json&>(c)["name"].as_string() != name) continue;
    // add the env vars that are missing (an existing var keeps its value, as in the reference)
    for (const auto& key : kCertEnv) {
      bool exists = false;
      for (const auto& e : static_cast<const Json&>(c)["env"].as_array()) exists = exists || e["name"].as_string() == key;
      if (!exists) c["env"].push_back(Json{{"name", key}, {"value", kCertMountPath}});
    }
    upsert_named(c["volumeMounts"], Json{{"name", "trusted-ca"}, {"readOnly", true}, {"mountPath", kCertMountPath}, {"subPath", "ca-bundle.crt"}});
    break;
  }
}

std::string odh_set_image_from_imagestreams(Json& nb, const std::vector<Json>& streams) {
  const std::string sel = annotation(nb, ODH_ANNOTATION_IMAGE_SELECTION);
  if (!has_annotation(nb, ODH_ANNOTATION_IMAGE_SELECTION)) return "";
  const std::string name = nb.str_at({"metadata", "name"});
  for (auto& c : nb["spec"]["template"]["spec"]["containers"].mut_array()) {
    if (static_cast<const Json&>(c)["name"].as_string() != name) continue;
    if (contains(static_cast<const Json&>(c)["image"].as_string(), "image-registry.openshift-image-registry.svc:5000")) return "";
    auto parts = split(sel, ':');
    if (parts.size() != 2) return "invalid image selection format";
    for (const auto& is : streams) {
      if (is.str_at({"metadata", "name"}) != parts[0]) continue;
      for (const auto& tag : is.at_path({"status", "tags"}).as_array()) {
        if (tag["tag"].as_string() != parts[1]) continue;
        std::vector<Json> items(tag["items"].as_array().begin(), tag["items"].as_array().end());
        if (items.empty()) continue;
        std::sort(items.begin(), items.end(),
                  [](const Json& x, const Json& y) { return x["created"].as_string() > y["created"].as_string(); });
        c["image"] = items[0]["dockerImageReference"];
        for (auto& e : c["env"].mut_array())
          if (static_cast<const Json&>(e)["name"].as_string() == "JUPYTER_IMAGE") {
            e["value"] = sel;
            break;
          }
        return "";
      }
    }
    KF_ERROR("odh-notebook-webhook", "Imagestream not found in main controller namespace",
             Json{{"imageSelected", parts[0]}, {"tag", parts[1]}});
    return "";
  }
  KF_ERROR("odh-notebook-webhook", "No container found matching the notebook name", Json{{"notebookName", name}});
  return "";
}

AdmissionFn make_odh_notebook_webhook(std::shared_ptr<Client> c, OdhOptions o) {
  return [c, o](AdmissionAttrs& a) -> ApiError {
    if (!a.object || a.res->kind != "Notebook" || a.res->group != "kubeflow.org") return {};
    if (a.operation != "CREATE" && a.operation != "UPDATE") return {};
    Json& nb = *a.object;
    const Json incoming = nb;
    const std::string ns = a.ns.empty() ? nb.str_at({"metadata", "namespace"}) : a.ns;
    if (a.operation == "CREATE") odh_inject_lock(nb);
    // image from the ImageStream selection
    Json streams;
    std::vector<Json> list;
    if (!c->list("image.openshift.io/v1", "ImageStream", o.controller_namespace, ListOptions(), streams))
      list.assign(streams["items"].as_array().begin(), streams["items"].as_array().end());
    std::string ierr = odh_set_image_from_imagestreams(nb, list);
    if (!ierr.empty()) return ApiError::Internal(ierr);
    // trusted CA bundle
    Json odh_cm;
    if (!c->get("v1", "ConfigMap", ns, "odh-trusted-ca-bundle", odh_cm)) {
      Json wb;
      bool have = !c->get("v1", "ConfigMap", ns, "workbench-trusted-ca-bundle", wb);
      if (!have) {
        Json cm{{"apiVersion", "v1"},
                {"kind", "ConfigMap"},
                {"metadata", Json{{"name", "workbench-trusted-ca-bundle"}, {"namespace", ns},
                                  {"labels", Json{{"opendatahub.io/managed-by", "workbenches"}}}}},
                {"data", Json{{"ca-bundle.crt", odh_cm.at_path({"data", "ca-bundle.crt"}).as_string()}}}};
        const ApiError ce = c->create(cm);
        have = !ce || ce.code == 409;  // the reconciler may have created it meanwhile
      }
      if (have) odh_inject_cert_config(nb, "workbench-trusted-ca-bundle");
    }
    if (odh_oauth_enabled(nb)) {
      if (odh_service_mesh_enabled(nb))
        return ApiError::Forbidden(std::string("admission webhook \"notebooks.opendatahub.io\" denied the request: Cannot have both ") +
                                   ODH_ANNOTATION_SERVICE_MESH + " and " + ODH_ANNOTATION_INJECT_OAUTH + " set to true. Pick one.");
      odh_inject_oauth_proxy(nb, o.oauth_proxy_image);
    }
    // maybeRestartRunningNotebook
    std::string pending;
    if (a.operation == "UPDATE" && a.old_object && !has_annotation(nb, STOP_ANNOTATION) &&
        !has_annotation(nb, ANNOTATION_NOTEBOOK_RESTART)) {
      const Json& old_spec = a.old_object->at_path({"spec", "template", "spec"});
      const Json& upd_spec = incoming.at_path({"spec", "template", "spec"});
      const Json& mut_spec = nb.at_path({"spec", "template", "spec"});
      if (old_spec == upd_spec && old_spec != mut_spec) {
        pending = json_first_difference(mut_spec, upd_spec, "v1.PodSpec");
        if (pending.empty()) pending = "failed to compute the reason for why there is a pending restart";
        nb["spec"]["template"]["spec"] = upd_spec;
      }
    }
    if (!pending.empty()) set_annotation(nb, ODH_ANNOTATION_UPDATE_PENDING, pending);
    else if (nb.at_path({"metadata", "annotations"}).is_object()) nb["metadata"]["annotations"].erase(ODH_ANNOTATION_UPDATE_PENDING);
    return {};
  };
}

// ---- PEM / DER validation (pem.Decode + x509.ParseCertificate structure) -------------------------
// notebook_controller.go:301-307: pem.Decode of the first block, which must be a CERTIFICATE, then
// x509.ParseCertificate of its DER — here OpenSSL's PEM reader + X.509 decoder (the whole
// tbsCertificate is parsed, not only the outer framing)
bool pem_certificate_valid(const std::string& pem) {
  const size_t b = pem.find("-----BEGIN ");
  if (b == std::string::npos || pem.compare(b, 27, "-----BEGIN CERTIFICATE-----") != 0) return false;
  BIO* bio = BIO_new_mem_buf(pem.data() + b, static_cast<int>(pem.size() - b));
  if (!bio) return false;
  X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
  BIO_free(bio);
  ERR_clear_error();
  if (!x) return false;
  X509_free(x);
  return true;
}

// ---- generated objects ----------------------------------------------------------------------------
namespace {
Json nb_labels(const Json& nb) { return Json{{"notebook-name", nb.str_at({"metadata", "name"})}}; }
Json meta(const Json& nb, const std::string& name) {
  return Json{{"name", name}, {"namespace", nb.str_at({"metadata", "namespace"})}, {"labels", nb_labels(nb)}};
}
}  // namespace

Json odh_network_policy(const Json& nb, const std::string& controller_ns) {
  const std::string name = nb.str_at({"metadata", "name"});
  Json m{{"name", name + "-ctrl-np"}, {"namespace", nb.str_at({"metadata", "namespace"})}};
  return Json{{"apiVersion", "networking.k8s.io/v1"},
              {"kind", "NetworkPolicy"},
              {"metadata", m},
              {"spec", Json{{"podSelector", Json{{"matchLabels", nb_labels(nb)}}},
                            {"ingress", Json::array({Json{{"ports", Json::array({Json{{"protocol", "TCP"}, {"port", 8888}}})},
                                                          {"from", Json::array({Json{{"namespaceSelector",
                                                                                      Json{{"matchLabels", Json{{"kubernetes.io/metadata.name", controller_ns}}}}}}})}}})},
                            {"policyTypes", Json::array({"Ingress"})}}}};
}

Json odh_oauth_network_policy(const Json& nb) {
  const std::string name = nb.str_at({"metadata", "name"});
  Json m{{"name", name + "-oauth-np"}, {"namespace", nb.str_at({"metadata", "namespace"})}};
  return Json{{"apiVersion", "networking.k8s.io/v1"},
              {"kind", "NetworkPolicy"},
              {"metadata", m},
              {"spec", Json{{"podSelector", Json{{"matchLabels", nb_labels(nb)}}},
                            {"ingress", Json::array({Json{{"ports", Json::array({Json{{"protocol", "TCP"}, {"port", 8443}}})}}})},
                            {"policyTypes", Json::array({"Ingress"})}}}};
}

Json odh_route(const Json& nb) {
  const std::string name = nb.str_at({"metadata", "name"});
  return Json{{"apiVersion", "route.openshift.io/v1"},
              {"kind", "Route"},
              {"metadata", meta(nb, name)},
              {"spec", Json{{"to", Json{{"kind", "Service"}, {"name", name}, {"weight", 100}}},
                            {"port", Json{{"targetPort", "http-" + name}}},
                            {"tls", Json{{"termination", "edge"}, {"insecureEdgeTerminationPolicy", "Redirect"}}},
                            {"wildcardPolicy", "None"}}}};
}

Json odh_oauth_route(const Json& nb) {
  Json r = odh_route(nb);
  r["spec"]["to"]["name"] = nb.str_at({"metadata", "name"}) + "-tls";
  r["spec"]["port"]["targetPort"] = "oauth-proxy";
  r["spec"]["tls"]["termination"] = "reencrypt";
  return r;
}

Json odh_service_account(const Json& nb) {
  const std::string name = nb.str_at({"metadata", "name"});
  Json m = meta(nb, name);
  m["annotations"] = Json{{"serviceaccounts.openshift.io/oauth-redirectreference.first",
                           "{\"kind\":\"OAuthRedirectReference\",\"apiVersion\":\"v1\",\"reference\":{\"kind\":\"Route\",\"name\":\"" + name +
                               "\"}}"}};
  return Json{{"apiVersion", "v1"}, {"kind", "ServiceAccount"}, {"metadata", m}};
}

Json odh_oauth_service(const Json& nb) {
  const std::string name = nb.str_at({"metadata", "name"});
  Json m = meta(nb, name + "-tls");
  m["annotations"] = Json{{"service.beta.openshift.io/serving-cert-secret-name", name + "-tls"}};
  return Json{{"apiVersion", "v1"},
              {"kind", "Service"},
              {"metadata", m},
              {"spec", Json{{"ports", Json::array({Json{{"name", "oauth-proxy"}, {"port", 443}, {"targetPort", "oauth-proxy"}, {"protocol", "TCP"}}})},
                            {"selector", Json{{"statefulset", name}}}}}};
}

Json odh_oauth_secret(const Json& nb) {
  // cookie secret: base64(base64(16 random bytes)) like NewNotebookOAuthSecret
  std::string seed;
  const std::string hex = secure_random_hex(16);
  for (size_t i = 0; i + 1 < hex.size(); i += 2) seed += static_cast<char>(std::stoi(hex.substr(i, 2), nullptr, 16));
  return Json{{"apiVersion", "v1"},
              {"kind", "Secret"},
              {"metadata", meta(nb, nb.str_at({"metadata", "name"}) + "-oauth-config")},
              {"stringData", Json{{"cookie_secret", base64_encode(base64_encode(seed))}}}};
}

Json odh_role_binding(const Json& nb, const std::string& name, const std::string& kind, const std::string& role) {
  return Json{{"apiVersion", "rbac.authorization.k8s.io/v1"},
              {"kind", "RoleBinding"},
              {"metadata", meta(nb, name)},
              {"subjects", Json::array({Json{{"kind", "ServiceAccount"}, {"name", nb.str_at({"metadata", "name"})},
                                             {"namespace", nb.str_at({"metadata", "namespace"})}}})},
              {"roleRef", Json{{"kind", kind}, {"name", role}, {"apiGroup", "rbac.authorization.k8s.io"}}}};
}

bool odh_unset_cert_config(Json& nb) {
  const std::string name = nb.str_at({"metadata", "name"});
  bool changed = false;
  Json& spec = nb["spec"]["template"]["spec"];
  for (auto& c : spec["containers"].mut_array()) {
    if (static_cast<const Json&>(c)["name"].as_string() != name) continue;
    Json env = Json::array(), mounts = Json::array();
    for (const auto& e : static_cast<const Json&>(c)["env"].as_array())
      if (std::find(kCertEnv.begin(), kCertEnv.end(), e["name"].as_string()) == kCertEnv.end()) env.push_back(e);
    for (const auto& m : static_cast<const Json&>(c)["volumeMounts"].as_array())
      if (m["name"].as_string() != "trusted-ca") mounts.push_back(m);
    if (c.has("env")) c["env"] = env;
    if (c.has("volumeMounts")) c["volumeMounts"] = mounts;
    changed = true;  // the reference marks the spec changed whenever the image container exists
    break;
  }
  Json vols = Json::array();
  bool removed = false;
  for (const auto& v : static_cast<const Json&>(spec)["volumes"].as_array()) {
    if (!removed && v.at_path({"configMap", "name"}).as_string() == "workbench-trusted-ca-bundle") {
      removed = changed = true;
      continue;
    }
    vols.push_back(v);
  }
  if (removed) spec["volumes"] = vols;
  return changed;
}

// ---- reconciler -------------------------------------------------------------------------------------
ApiError OdhNotebookReconciler::reconcile_cert_configmap(const Json& nb, bool* skipped) {
  *skipped = false;
  const std::string ns = nb.str_at({"metadata", "namespace"});
  std::vector<std::string> pool;
  const std::vector<std::pair<std::string, std::vector<std::string>>> cms = {
      {"odh-trusted-ca-bundle", {"ca-bundle.crt", "odh-ca-bundle.crt"}}, {"kube-root-ca.crt", {"ca.crt"}}};
  for (const auto& cm_files : cms) {
    Json cm;
    ApiError e = c_->get("v1", "ConfigMap", ns, cm_files.first, cm);
    if (e) {
      if (e.code == 404 && cm_files.first == "odh-trusted-ca-bundle") {
        *skipped = true;
        return {};
      }
      continue;
    }
    for (const auto& file : cm_files.second) {
      const Json* v = cm["data"].find(file);
      const std::string data = v ? trim(v->as_string()) : "";
      if (!v || (file == "ca-bundle.crt" && data.empty())) return {};  // (reference quirk: any missing key stops here)
      if (data.empty()) continue;
      if (pem_certificate_valid(data)) pool.push_back(data);
      else KF_INFO("odh-notebook-controller", "Invalid certificate format", Json{{"configMap", cm_files.first}, {"certFile", file}});
    }
  }
  if (pool.empty()) return {};
  Json desired{{"apiVersion", "v1"},
               {"kind", "ConfigMap"},
               {"metadata", Json{{"name", "workbench-trusted-ca-bundle"}, {"namespace", ns},
                                 {"labels", Json{{"opendatahub.io/managed-by", "workbenches"}}}}},
               {"data", Json{{"ca-bundle.crt", join(pool, "\n")}}}};
  Json found;
  ApiError e = c_->get("v1", "ConfigMap", ns, "workbench-trusted-ca-bundle", found);
  if (e.code == 404) {
    ApiError ce = c_->create(desired);
    if (ce && ce.code != 409) return ce;
  } else if (!e && found["data"] != desired["data"]) {
    found["data"] = desired["data"];
    return c_->update(found);
  }
  return {};
}

ApiError OdhNotebookReconciler::reconcile_simple(const Json& desired, bool compare_spec) {
  Json found;
  const std::string av = desired["apiVersion"].as_string(), kind = desired["kind"].as_string();
  const std::string ns = desired.str_at({"metadata", "namespace"}), name = desired.str_at({"metadata", "name"});
  ApiError e = c_->get(av, kind, ns, name, found);
  if (e.code == 404) {
    Json d = desired;
    ApiError ce = c_->create(d);
    return ce.code == 409 ? ApiError{} : ce;
  }
  if (e || !compare_spec) return e;
  auto norm = [](Json s) {
    if (s.is_object()) s.erase("host");  // the router fills spec.host (CompareNotebookRoutes)
    return s;
  };
  if (found.at_path({"metadata", "labels"}) == desired.at_path({"metadata", "labels"}) && norm(found["spec"]) == norm(desired["spec"]))
    return {};
  return c_->update_with_retry(av, kind, ns, name, [&](Json& o) {
    const Json host = o.at_path({"spec", "host"});
    o["spec"] = desired["spec"];
    if (host.is_string()) o["spec"]["host"] = host;
    o["metadata"]["labels"] = desired.at_path({"metadata", "labels"});
    return true;
  });
}

Result OdhNotebookReconciler::remove_lock(const Json& nb, std::string* err) {
  const std::string ns = nb.str_at({"metadata", "namespace"}), name = nb.str_at({"metadata", "name"});
  const std::string key = ns + "/" + name;
  if (odh_oauth_enabled(nb) && !odh_service_mesh_enabled(nb)) {
    // wait (by requeue) for the OAuth service account's image pull secret: 1s, 5s, then give up
    Json sa;
    const bool ready = !c_->get("v1", "ServiceAccount", ns, name, sa) && !sa["imagePullSecrets"].empty();
    if (!ready) {
      std::lock_guard<std::mutex> g(lock_mu_);
      int& n = lock_attempts_[key];
      if (n < 2) {
        const double delay = n == 0 ? 1.0 : 5.0;
        ++n;
        Result r;
        r.requeue_after = delay;
        return r;
      }
    }
  }
  {
    std::lock_guard<std::mutex> g(lock_mu_);
    lock_attempts_.erase(key);
  }
  Json out;
  ApiError e = c_->patch("kubeflow.org/v1", "Notebook", ns, name, "merge",
                         Json{{"metadata", Json{{"annotations", Json{{STOP_ANNOTATION, Json()}}}}}}, out);
  if (e && e.code != 404) *err = e.message;
  return {};
}

Result OdhNotebookReconciler::reconcile(const Request& r, std::string* err) {
  Json nb;
  ApiError e = c_->get("kubeflow.org/v1", "Notebook", r.ns, r.name, nb);
  if (e.code == 404) return {};
  if (e) {
    *err = e.message;
    return {};
  }
  // Conscious deviation: the reference reconciles a Notebook that is being deleted and so keeps
  // re-creating its network policies / Route / OAuth objects while a foreground deletion waits for
  // them (the GC deletes them again: deletion took 10-40 s on kube-lite). A terminating Notebook
  // owns nothing new, as in the core notebook controller (notebook_controller.go:135-137).
  if (nb.at_path({"metadata", "deletionTimestamp"}).is_string()) return {};
  auto owned = [&](Json obj) {
    set_controller_reference(nb, obj);
    return obj;
  };
  bool skipped = false;
  if ((e = reconcile_cert_configmap(nb, &skipped))) {
    *err = e.message;
    return {};
  }
  {
    // IsConfigMapDeleted -> UnsetNotebookCertConfig
    Json cm;
    if (c_->get("v1", "ConfigMap", r.ns, "workbench-trusted-ca-bundle", cm)) {
      bool mounted = false;
      for (const auto& v : nb.at_path({"spec", "template", "spec", "volumes"}).as_array())
        mounted = mounted || v.at_path({"configMap", "name"}).as_string() == "workbench-trusted-ca-bundle";
      if (mounted) {
        e = c_->update_with_retry("kubeflow.org/v1", "Notebook", r.ns, r.name, [](Json& o) { return odh_unset_cert_config(o); });
        if (e) {
          *err = "Unable to update the notebook for removing the env variables: " + e.message;
          return {};
        }
      }
    }
  }
  if ((e = reconcile_simple(owned(odh_network_policy(nb, o_.controller_namespace)), true))) {
    *err = "error creating Notebook network policy: " + e.message;
    return {};
  }
  if (!odh_service_mesh_enabled(nb) && (e = reconcile_simple(owned(odh_oauth_network_policy(nb)), true))) {
    *err = "error creating Notebook OAuth network policy: " + e.message;
    return {};
  }
  if (o_.set_pipeline_rbac) {
    Json role;
    if (!c_->get("rbac.authorization.k8s.io/v1", "Role", r.ns, "ds-pipeline-user-access-dspa", role)) {
      Json rb = owned(odh_role_binding(nb, "elyra-pipelines-" + r.name, "Role", "ds-pipeline-user-access-dspa"));
      Json found;
      ApiError ge = c_->get("rbac.authorization.k8s.io/v1", "RoleBinding", r.ns, "elyra-pipelines-" + r.name, found);
      if (ge.code == 404) ge = c_->create(rb);
      else if (!ge && found["subjects"] != rb["subjects"]) {
        found["subjects"] = rb["subjects"];
        ge = c_->update(found);
      }
      if (ge) {
        *err = "Unable to Reconcile Rolebinding: " + ge.message;
        return {};
      }
    }
  }
  if (!odh_service_mesh_enabled(nb)) {
    if (odh_oauth_enabled(nb)) {
      for (const Json& obj : {odh_service_account(nb), odh_oauth_service(nb), odh_oauth_secret(nb)}) {
        if ((e = reconcile_simple(owned(obj), false))) {
          *err = e.message;
          return {};
        }
      }
      e = reconcile_simple(owned(odh_oauth_route(nb)), true);
    } else {
      e = reconcile_simple(owned(odh_route(nb)), true);
    }
    if (e) {
      *err = e.message;
      return {};
    }
  }
  if (odh_lock_enabled(nb)) return remove_lock(nb, err);
  return {};
}

void OdhNotebookReconciler::setup(Manager& mgr, int workers) {
  ctl_ = std::make_shared<Controller>("odh-notebook-controller", [this](const Request& r, std::string* e) { return reconcile(r, e); },
                                      workers);
  Informer& nbs = mgr.informer("kubeflow.org/v1", "Notebook");
  ctl_->For(nbs);
  ctl_->Owns(mgr.informer("route.openshift.io/v1", "Route"), "Notebook");
  ctl_->Owns(mgr.informer("v1", "ServiceAccount"), "Notebook");
  ctl_->Owns(mgr.informer("v1", "Service"), "Notebook");
  ctl_->Owns(mgr.informer("v1", "Secret"), "Notebook");
  ctl_->Owns(mgr.informer("networking.k8s.io/v1", "NetworkPolicy"), "Notebook");
  ctl_->Owns(mgr.informer("rbac.authorization.k8s.io/v1", "RoleBinding"), "Notebook");
  ctl_->Watches(mgr.informer("v1", "ConfigMap"), [&nbs](const std::string&, const Json& cm) {
    std::vector<Request> out;
    const std::string ns = cm.str_at({"metadata", "namespace"}), name = cm.str_at({"metadata", "name"});
    if (name == "odh-trusted-ca-bundle") {
      // conscious fix: every notebook of the namespace (the reference returns after the first)
      for (const auto& nb : nbs.list(ns)) out.push_back({ns, nb.str_at({"metadata", "name"})});
    } else if (name == "workbench-trusted-ca-bundle") {
      for (const auto& nb : nbs.list(ns))
        for (const auto& v : nb.at_path({"spec", "template", "spec", "volumes"}).as_array())
          if (v.at_path({"configMap", "name"}).as_string() == name) {
            out.push_back({ns, nb.str_at({"metadata", "name"})});
            break;
          }
    }
    return out;
  });
  mgr.add(ctl_);
}

}  // namespace kf
