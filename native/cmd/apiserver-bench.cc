// apiserver-bench.cc — in-process kube-lite throughput/latency micro-benchmark.
//
// Measures the storage path every controller write takes (admission -> validation -> commit ->
// WAL -> watch fan-out) without HTTP or the controllers: create N pods, then M status updates
// spread over them, with W concurrent watchers draining the Pod watch (the informer count of a
// kflite process). Prints one JSON line: per-op mean / p50 / p99 in microseconds.
//
//   apiserver-bench [--pods 1000] [--updates 5000] [--watchers 6] [--wal DIR]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#include "apiserver/apiserver.h"
#include "core/util.h"

using namespace kf;

namespace {
double pct(std::vector<double> v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, static_cast<size_t>(q * static_cast<double>(v.size() - 1) + 0.5))];
}

Json stats(const std::vector<double>& us) {
  double s = 0;
  for (double x : us) s += x;
  return Json{{"n", static_cast<int64_t>(us.size())},
              {"mean_us", us.empty() ? 0.0 : s / static_cast<double>(us.size())},
              {"p50_us", pct(us, 0.5)},
              {"p99_us", pct(us, 0.99)}};
}

Json make_pod(int i) {
  Json c{{"name", "notebook"},
         {"image", "kfamd/jupyter-pytorch-rocm:latest"},
         {"resources", Json{{"limits", Json{{"amd.com/gpu", "1"}}}, {"requests", Json{{"cpu", "500m"}, {"memory", "1Gi"}}}}},
         {"env", Json::array({Json{{"name", "NB_PREFIX"}, {"value", "/notebook/bench/nb-" + std::to_string(i)}}})},
         {"ports", Json::array({Json{{"containerPort", 8888}, {"name", "notebook-port"}, {"protocol", "TCP"}}})},
         {"volumeMounts", Json::array({Json{{"mountPath", "/dev/shm"}, {"name", "dshm"}}})}};
  return Json{{"apiVersion", "v1"},
              {"kind", "Pod"},
              {"metadata", Json{{"name", "nb-" + std::to_string(i) + "-0"},
                                {"namespace", "bench"},
                                {"labels", Json{{"notebook-name", "nb-" + std::to_string(i)}, {"statefulset", "nb-" + std::to_string(i)}}}}},
              {"spec", Json{{"containers", Json::array({c})},
                            {"volumes", Json::array({Json{{"name", "dshm"}, {"emptyDir", Json{{"medium", "Memory"}}}}})}}}};
}
}  // namespace

int main(int argc, char** argv) {
  Flags f;
  int64_t pods = 1000, updates = 5000, watchers = 6;
  std::string wal;
  f.add_int("pods", &pods, 1000, "pods to create");
  f.add_int("updates", &updates, 5000, "status updates (round-robin over the pods)");
  f.add_int("watchers", &watchers, 6, "concurrent Pod watchers (informers) draining events");
  f.add_string("wal", &wal, "", "data dir for the WAL (empty = in-memory)");
  std::string err;
  if (!f.parse(argc, argv, &err) || f.help_requested()) {
    std::fprintf(stderr, "%s\n%s", err.c_str(), f.usage().c_str());
    return err.empty() ? 0 : 2;
  }
  ApiServer::Config cfg;
  cfg.data_dir = wal;
  ApiServer api(cfg);
  api.bootstrap();
  Json ns{{"apiVersion", "v1"}, {"kind", "Namespace"}, {"metadata", Json{{"name", "bench"}}}};
  api.create(ns);

  std::atomic<bool> stop{false};
  std::atomic<int64_t> delivered{0};
  std::vector<std::thread> ws;
  for (int64_t w = 0; w < watchers; ++w) {
    ApiError e;
    WatchPtr wp = api.watch("v1", "Pod", "", ListOptions(), &e);
    ws.emplace_back([wp, &stop, &delivered] {
      WatchEvent ev;
      while (!stop) {
        if (wp->next(ev, 50)) delivered++;
      }
      wp->stop();
    });
  }

  std::vector<double> create_us, get_us, update_us;
  for (int64_t i = 0; i < pods; ++i) {
    Json p = make_pod(static_cast<int>(i));
    double t0 = now_seconds();
    ApiError e = api.create(p);
    create_us.push_back((now_seconds() - t0) * 1e6);
    if (e) {
      std::fprintf(stderr, "create: %s\n", e.message.c_str());
      return 1;
    }
  }
  for (int64_t u = 0; u < updates; ++u) {
    const std::string name = "nb-" + std::to_string(u % pods) + "-0";
    Json cur;
    double t0 = now_seconds();
    api.get("v1", "Pod", "bench", name, cur);
    double t1 = now_seconds();
    cur["status"]["phase"] = "Running";
    cur["status"]["conditions"] = Json::array({Json{{"type", "Ready"}, {"status", (u & 1) ? "True" : "False"},
                                                    {"lastTransitionTime", rfc3339_ms_now()}}});
    ApiError e = api.update_status(cur);
    double t2 = now_seconds();
    get_us.push_back((t1 - t0) * 1e6);
    update_us.push_back((t2 - t1) * 1e6);
    if (e) {
      std::fprintf(stderr, "update: %s\n", e.message.c_str());
      return 1;
    }
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(200));
  stop = true;
  for (auto& t : ws) t.join();
  Json out{{"pods", pods}, {"updates", updates}, {"watchers", watchers}, {"wal", !wal.empty()},
           {"create", stats(create_us)}, {"get", stats(get_us)}, {"update_status", stats(update_us)},
           {"watch_events_delivered", delivered.load()}};
  std::printf("%s\n", out.dump().c_str());
  api.stop();
  return 0;
}
