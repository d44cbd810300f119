// kflite — the all-in-one MI355X-native control plane binary.
//
// One process hosts the kube-lite API server and, selectable with --controllers, every
// reconciler of the reference (notebook, culler, odh, profile, tensorboard, pvcviewer), the
// admission webhooks (poddefault, odh notebook, pvcviewer, quota), KFAM, and the built-in node
// stack that the reference delegates to kube-controller-manager / kube-scheduler / kubelet:
// statefulset, deployment/replicaset, pvc binder, GPU-topology-aware scheduler + device plugin,
// the local kubelet (process pods), and the Istio-style HTTP gateway.
//
// The split binaries in cmd/ (notebook-controller, odh-notebook-controller, ...) run the same
// components against any API server over REST.
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <set>

#include "apiserver/apiserver.h"
#include "cmd/components.h"
#include "core/http.h"
#include "core/util.h"
#include "runtime/runtime.h"

using namespace kf;

static std::atomic<bool> g_stop{false};
static void on_signal(int) { g_stop = true; }

int main(int argc, char** argv) {
  Flags f;
  std::string data_dir, api_addr, controllers, metrics_addr, probe_addr, token_file, authz, tls_cert, tls_key, client_ca;
  int64_t api_port = 0, workers = 1;
  bool log_json = false, debug = false;
  f.add_string("data-dir", &data_dir, "", "directory for the WAL and pod sandboxes (empty = in-memory)");
  f.add_string("bind-address", &api_addr, "127.0.0.1", "API server bind address");
  f.add_int("port", &api_port, 0, "API server port (0 = ephemeral)");
  f.add_string("tls-cert-file", &tls_cert, "", "serve the API over HTTPS with this certificate (kube-apiserver flag)");
  f.add_string("tls-private-key-file", &tls_key, "", "private key for --tls-cert-file");
  f.add_string("client-ca-file", &client_ca, "", "verify client certificates against this CA (optional mTLS)");
  f.add_string("controllers", &controllers, "all",
               "comma list: notebook,culler,odh,profile,tensorboard,pvcviewer,webhooks,kfam,builtin,scheduler,kubelet,gateway (or all)");
  f.add_string("metrics-addr", &metrics_addr, "0", "controller metrics address (0 = disabled; the API server serves /metrics)");
  f.add_string("probe-addr", &probe_addr, "0", "controller health probe address");
  f.add_string("authorization-mode", &authz, "AlwaysAllow", "AlwaysAllow | RBAC");
  f.add_string("token-auth-file", &token_file, "", "JSON {token: {username, groups}} for bearer-token authentication");
  f.add_int("workers", &workers, 1, "reconcile workers per controller (the reference uses 1)");
  f.add_bool("log-json", &log_json, false, "zap-style JSON logs");
  f.add_bool("debug", &debug, false, "debug logging");
  ComponentFlags cf;
  cf.register_flags(f);
  std::string err;
  if (!f.parse(argc, argv, &err) || f.help_requested()) {
    std::fprintf(stderr, "%s\nusage: kflite [flags]\n%s", err.c_str(), f.usage().c_str());
    return err.empty() ? 0 : 2;
  }
  Logger::get().set_json(log_json);
  if (debug) Logger::get().set_level(LogLevel::Debug);
  ::signal(SIGINT, on_signal);
  ::signal(SIGTERM, on_signal);

  ApiServer::Config cfg;
  cfg.data_dir = data_dir.empty() ? "" : data_dir + "/etcd";
  cfg.authz_rbac = authz == "RBAC";
  if (!token_file.empty()) {
    std::string t;
    Json tokens;
    if (!read_file(token_file, t) || !Json::try_parse(t, tokens)) {
      std::fprintf(stderr, "cannot read token file %s\n", token_file.c_str());
      return 2;
    }
    for (const auto& m : tokens.as_object()) {
      UserInfo u;
      u.username = m.second["username"].as_string();
      u.groups.clear();
      for (const auto& g : m.second["groups"].as_array()) u.groups.push_back(g.as_string());
      cfg.tokens[m.first] = u;
    }
  }
  ApiServer api(cfg);
  api.bootstrap();
  api.start_background();
  set_host_resolver([&api](const std::string& host, int port, std::string& ip, int& out_port) {
    return api.resolve_service(host, port, ip, out_port);
  });

  HttpServer srv;
  if (!tls_cert.empty()) {
    TlsServerConfig tls{tls_cert, tls_key.empty() ? tls_cert : tls_key, client_ca, false};
    if (!srv.enable_tls(tls, &err)) {
      std::fprintf(stderr, "apiserver: %s\n", err.c_str());
      return 1;
    }
  }
  if (!srv.listen(api_addr, static_cast<int>(api_port), &err)) {
    std::fprintf(stderr, "apiserver: %s\n", err.c_str());
    return 1;
  }
  srv.set_handler([&api](HttpRequest& req, HttpResponse& resp) { api.handle_http(req, resp); });
  srv.start();
  const std::string url = std::string(srv.tls() ? "https://" : "http://") + api_addr + ":" + std::to_string(srv.port());
  if (!data_dir.empty()) {
    make_dirs(data_dir);
    write_file(data_dir + "/kflite.json", Json{{"server", url}, {"pid", static_cast<int64_t>(::getpid())}}.dump() + "\n");
  }
  std::printf("kflite: API server listening on %s\n", url.c_str());
  std::fflush(stdout);

  std::set<std::string> enabled;
  for (auto& c : split(controllers, ',', true)) enabled.insert(trim(c));
  if (enabled.count("all"))
    enabled = {"notebook", "culler", "odh", "profile", "tensorboard", "pvcviewer", "webhooks", "kfam",
               "builtin", "scheduler", "kubelet", "gateway"};

  auto client = std::make_shared<LocalClient>(&api);
  Manager::Options mo;
  mo.metrics_addr = metrics_addr;
  mo.probe_addr = probe_addr;
  Manager mgr(client, mo);
  Components comps(cf, client, &api, url, data_dir);
  if (!comps.setup(mgr, enabled, static_cast<int>(workers), &err)) {
    std::fprintf(stderr, "setup: %s\n", err.c_str());
    return 1;
  }
  if (!mgr.start(&err)) {
    std::fprintf(stderr, "manager: %s\n", err.c_str());
    return 1;
  }
  comps.start();
  if (comps.gateway_port()) std::printf("kflite: gateway listening on http://%s:%d\n", cf.gateway_addr.c_str(), comps.gateway_port());
  if (!data_dir.empty())
    write_file(data_dir + "/kflite.json", Json{{"server", url}, {"pid", static_cast<int64_t>(::getpid())},
                                               {"gateway", comps.gateway_port() ? "http://" + cf.gateway_addr + ":" + std::to_string(comps.gateway_port()) : ""},
                                               {"mesh", comps.mesh_port() ? "http://" + cf.gateway_addr + ":" + std::to_string(comps.mesh_port()) : ""},
                                               {"kfam", comps.kfam_port() ? "http://127.0.0.1:" + std::to_string(comps.kfam_port()) : ""}}
                                                  .dump() + "\n");
  std::printf("kflite: controllers running: %s\n", join(std::vector<std::string>(enabled.begin(), enabled.end()), ",").c_str());
  std::fflush(stdout);
  while (!g_stop) ::usleep(100000);
  std::printf("kflite: shutting down\n");
  comps.stop();
  mgr.stop();
  srv.stop();
  api.stop();
  return 0;
}
