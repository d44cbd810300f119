// split_main.h — shared main() of the per-component binaries (the reference ships one manager
// binary per component: notebook-controller/main.go, odh-notebook-controller/main.go,
// profile-controller/main.go, tensorboard-controller/main.go, pvcviewer-controller/main.go,
// admission-webhook/main.go, access-management/main.go). Each talks to an API server over REST
// (--server / KFAMD_API_URL / in-cluster KUBERNETES_SERVICE_HOST:PORT + SA token) and runs the
// same components kflite hosts in-process.
#pragma once

#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <functional>
#include <set>
#include <string>

#include "cmd/components.h"
#include "core/http.h"
#include "core/util.h"
#include "runtime/runtime.h"

namespace kf {

struct SplitSpec {
  std::string name;                  // binary name (logs)
  std::set<std::string> components;  // Components::setup selection
  std::string leader_election_id;
  std::string metrics_addr = ":8080";
  std::string probe_addr = ":8081";
  // extra flag names the reference uses for the same settings (aliases)
  std::function<void(Flags&, ComponentFlags&)> extra_flags;
  int64_t default_webhook_port = -1;  // serve the component's admission webhooks over HTTP
  int64_t default_kfam_port = -1;
};

inline std::atomic<bool>& split_stop_flag() {
  static std::atomic<bool> s{false};
  return s;
}

inline int run_split(int argc, char** argv, SplitSpec spec) {
  Flags f;
  std::string server, token_file, metrics_addr = spec.metrics_addr, probe_addr = spec.probe_addr, le_ns, ca_file,
      client_cert, client_key;
  bool leader = false, log_json = false, debug = false, insecure = false;
  int64_t qps = 0, burst = 0, workers = 1;
  f.add_string("server", &server, "", "API server URL (default: $KFAMD_API_URL or in-cluster service env)");
  f.add_string("token-file", &token_file, "/var/run/secrets/kubernetes.io/serviceaccount/token", "bearer token file");
  f.add_string("certificate-authority", &ca_file, "/var/run/secrets/kubernetes.io/serviceaccount/ca.crt",
               "CA bundle that signs the API server's certificate (https servers)");
  f.add_string("client-certificate", &client_cert, "", "client certificate for the API server (mutual TLS)");
  f.add_string("client-key", &client_key, "", "client key for --client-certificate");
  f.add_bool("insecure-skip-tls-verify", &insecure, false, "do not verify the API server's certificate");
  f.add_string("metrics-addr", &metrics_addr, spec.metrics_addr, "metrics endpoint address");
  f.add_string("metrics-bind-address", &metrics_addr, spec.metrics_addr, "metrics endpoint address (alias)");
  f.add_string("probe-addr", &probe_addr, spec.probe_addr, "health probe address");
  f.add_string("health-probe-bind-address", &probe_addr, spec.probe_addr, "health probe address (alias)");
  f.add_bool("enable-leader-election", &leader, false, "leader election (Lease)");
  f.add_bool("leader-elect", &leader, false, "leader election (alias)");
  f.add_string("leader-election-namespace", &le_ns, "kube-system", "namespace of the leader-election Lease");
  f.add_int("qps", &qps, 0, "client QPS limit (0 = unlimited)");
  f.add_int("burst", &burst, 0, "client burst (accepted for compatibility)");
  f.add_int("workers", &workers, 1, "reconcile workers per controller");
  f.add_bool("log-json", &log_json, false, "zap-style JSON logs");
  f.add_bool("debug-log", &debug, false, "debug logging");
  ComponentFlags cf;
  cf.register_flags(f);
  if (spec.extra_flags) spec.extra_flags(f, cf);
  std::string err;
  if (!f.parse(argc, argv, &err) || f.help_requested()) {
    std::fprintf(stderr, "%s\nusage: %s [flags]\n%s", err.c_str(), spec.name.c_str(), f.usage().c_str());
    return err.empty() ? 0 : 2;
  }
  if (cf.webhook_port < 0) cf.webhook_port = spec.default_webhook_port;
  if (cf.kfam_port < 0) cf.kfam_port = spec.default_kfam_port;
  Logger::get().set_json(log_json);
  if (debug) Logger::get().set_level(LogLevel::Debug);
  ::signal(SIGINT, [](int) { split_stop_flag() = true; });
  ::signal(SIGTERM, [](int) { split_stop_flag() = true; });
  if (server.empty()) server = getenv_or("KFAMD_API_URL", "");
  // in-cluster: the kubernetes service is HTTPS, verified with the service account's ca.crt
  // (client-go rest.InClusterConfig)
  if (server.empty() && !getenv_or("KUBERNETES_SERVICE_HOST", "").empty())
    server = "https://" + getenv_or("KUBERNETES_SERVICE_HOST", "") + ":" + getenv_or("KUBERNETES_SERVICE_PORT", "443");
  {
    TlsClientOptions tls;
    if (!ca_file.empty() && file_exists(ca_file)) tls.ca_file = ca_file;
    tls.cert_file = client_cert;
    tls.key_file = client_key;
    tls.insecure_skip_verify = insecure;
    set_default_tls_client(tls);
  }
  if (server.empty()) {
    std::fprintf(stderr, "%s: no API server (--server / KFAMD_API_URL)\n", spec.name.c_str());
    return 2;
  }
  std::string token;
  read_file(token_file, token);
  token = trim(token);
  // controller namespace from the SA mount when not given (odh main.go:63-72)
  std::string ns_file;
  if (read_file("/var/run/secrets/kubernetes.io/serviceaccount/namespace", ns_file) && !trim(ns_file).empty() &&
      cf.controller_namespace == "opendatahub")
    cf.controller_namespace = trim(ns_file);
  auto client = std::make_shared<RestClient>(server, token, static_cast<int>(qps));
  set_host_resolver([client](const std::string& host, int port, std::string& ip, int& out_port) {
    return resolve_service_via(*client, host, port, ip, out_port);
  });
  Manager::Options mo;
  mo.metrics_addr = metrics_addr;
  mo.probe_addr = probe_addr;
  mo.leader_election = leader;
  mo.leader_election_id = spec.leader_election_id;
  mo.leader_election_namespace = le_ns;
  Manager mgr(client, mo);
  Components comps(cf, client, nullptr, server, "");
  if (!comps.setup(mgr, spec.components, static_cast<int>(workers), &err)) {
    std::fprintf(stderr, "%s: setup: %s\n", spec.name.c_str(), err.c_str());
    return 1;
  }
  if (!mgr.start(&err)) {
    std::fprintf(stderr, "%s: manager: %s\n", spec.name.c_str(), err.c_str());
    return 1;
  }
  comps.start();
  KF_INFO(spec.name, "started", Json{{"server", server}, {"webhook_port", comps.webhook_port()}, {"kfam_port", comps.kfam_port()},
                                     {"metrics_port", mgr.metrics_port()}, {"probe_port", mgr.probe_port()}});
  while (!split_stop_flag()) ::usleep(100000);
  comps.stop();
  mgr.stop();
  return 0;
}

}  // namespace kf
