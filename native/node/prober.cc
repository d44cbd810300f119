// Prober: see prober.h.
#include "node/prober.h"

#include <atomic>

#include "core/util.h"

namespace kf {

Prober::Prober(Notify notify, size_t max_threads) : notify_(std::move(notify)), max_threads_(max_threads ? max_threads : 1) {}

Prober::~Prober() { stop(); }

uint64_t Prober::next_generation() {
  static std::atomic<uint64_t> g{0};
  return ++g;
}

std::optional<bool> Prober::poll(const std::string& key, uint64_t gen, bool due, const std::string& ns,
                                 const std::string& name, std::function<bool()> run) {
  std::unique_lock<std::mutex> g(mu_);
  if (stop_) return std::nullopt;
  State& s = st_[key];
  if (s.gen != gen) s = State{gen};  // a new container start: older verdicts and jobs are moot
  if (s.has_result) {
    s.has_result = false;
    return s.ok;
  }
  if (s.inflight || !due) return std::nullopt;
  s.inflight = true;
  ++started_;
  q_.push_back(Job{key, ns, name, gen, std::move(run)});
  if (idle_ == 0 && threads_.size() < max_threads_) {
    threads_.emplace_back([this] {
      set_thread_name("kubelet-probe");
      worker();
    });
  } else {
    cv_.notify_one();
  }
  return std::nullopt;
}

bool Prober::in_flight(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = st_.find(key);
  return it != st_.end() && it->second.inflight;
}

void Prober::forget_pod(const std::string& uid) {
  std::lock_guard<std::mutex> g(mu_);
  const std::string prefix = uid + "/";
  for (auto it = st_.lower_bound(prefix); it != st_.end() && it->first.compare(0, prefix.size(), prefix) == 0;)
    it = st_.erase(it);
}

void Prober::worker() {
  std::unique_lock<std::mutex> g(mu_);
  for (;;) {
    ++idle_;
    cv_.wait(g, [this] { return stop_ || !q_.empty(); });
    --idle_;
    if (stop_) return;
    Job j = std::move(q_.front());
    q_.pop_front();
    g.unlock();
    bool ok = false;
    try {
      ok = j.run();
    } catch (...) {
      ok = false;
    }
    g.lock();
    auto it = st_.find(j.key);
    const bool current = it != st_.end() && it->second.gen == j.gen;
    if (current) {
      it->second.inflight = false;
      it->second.has_result = true;
      it->second.ok = ok;
    }
    if (current && notify_ && !stop_) {
      g.unlock();
      notify_(j.ns, j.name);
      g.lock();
    }
  }
}

void Prober::stop() {
  std::vector<std::thread> ts;
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    q_.clear();
    ts.swap(threads_);
  }
  cv_.notify_all();
  for (auto& t : ts)
    if (t.joinable()) t.join();
}

uint64_t Prober::started() const {
  std::lock_guard<std::mutex> g(mu_);
  return started_;
}

size_t Prober::threads() const {
  std::lock_guard<std::mutex> g(mu_);
  return threads_.size();
}

}  // namespace kf
