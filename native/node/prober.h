// Container probes off the kubelet's reconcile workers: the kubelet's prober manager equivalent
// (k8s.io/kubernetes/pkg/kubelet/prober, one worker per container probe). A reconcile pass never
// runs a probe itself: it asks poll() whether the last probe of (container, kind) has a verdict,
// and hands it a closure to run when one is due. The closure runs on a prober thread (the pool grows
// to one thread per in-flight probe, up to a cap), the verdict is cached, and the pod's key is
// re-queued so the next pass reads it at once.
//
// A started container gets a new generation; verdicts of an older generation (a probe that was in
// flight across a restart) are dropped.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <vector>

namespace kf {

class Prober {
 public:
  using Notify = std::function<void(const std::string& ns, const std::string& name)>;
  explicit Prober(Notify notify, size_t max_threads = 64);
  ~Prober();
  Prober(const Prober&) = delete;
  Prober& operator=(const Prober&) = delete;

  // key: "<pod uid>/<container>/<kind>". Returns the verdict of a finished probe of generation
  // `gen` (consumed: each verdict is returned once). Otherwise, when `due` and none is in flight,
  // starts `run` on a prober thread; its verdict re-queues ns/name.
  std::optional<bool> poll(const std::string& key, uint64_t gen, bool due, const std::string& ns,
                           const std::string& name, std::function<bool()> run);
  bool in_flight(const std::string& key);
  void forget_pod(const std::string& uid);  // drop every key of the pod (its verdicts are moot)
  void stop();
  static uint64_t next_generation();

  // counters for /metrics and tests
  uint64_t started() const;
  size_t threads() const;

 private:
  struct State {
    uint64_t gen = 0;
    bool inflight = false, has_result = false, ok = false;
  };
  struct Job {
    std::string key, ns, name;
    uint64_t gen = 0;
    std::function<bool()> run;
  };
  void worker();
  Notify notify_;
  size_t max_threads_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, State> st_;
  std::deque<Job> q_;
  std::vector<std::thread> threads_;
  size_t idle_ = 0;
  uint64_t started_ = 0;
  bool stop_ = false;
};

}  // namespace kf
