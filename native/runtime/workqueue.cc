// workqueue.cc — rate-limited delaying de-duplicating queue (see runtime.h).
#include <algorithm>
#include <chrono>
#include <cmath>

#include "core/util.h"
#include "runtime/runtime.h"

namespace kf {

WorkQueue::WorkQueue(std::string name, double base_delay, double max_delay, double qps, int burst)
    : name_(std::move(name)), base_(base_delay), max_(max_delay), qps_(qps), burst_(burst),
      tokens_(burst), last_refill_(now_seconds()) {
  depth_ = Registry::global().gauge("workqueue_depth", "Current depth of workqueue", {"name"});
  adds_ = Registry::global().counter("workqueue_adds_total", "Total number of adds handled by workqueue", {"name"});
  retries_ = Registry::global().counter("workqueue_retries_total", "Total number of retries handled by workqueue", {"name"});
  // client-go parity: time from an item becoming dirty (watch event / requeue) to a worker taking it.
  // Watch-event -> reconcile-done latency = this + controller_runtime_reconcile_time_seconds.
  queue_dur_ = Registry::global().histogram("workqueue_queue_duration_seconds",
                                            "How long in seconds an item stays in workqueue before being requested",
                                            {"name"}, HistogramVec::exponential(0.00001, 2, 24));
  delay_th_ = std::thread([this] {
    set_thread_name("q:" + name_);
    delay_loop();
  });
}

WorkQueue::~WorkQueue() {
  shutdown();
  if (delay_th_.joinable()) delay_th_.join();
}

void WorkQueue::add(const Request& r) {
  std::lock_guard<std::mutex> g(mu_);
  if (shutdown_) return;
  adds_->inc({name_});
  if (dirty_.count(r)) return;
  dirty_.insert(r);
  added_at_.emplace(r, now_seconds());
  if (processing_.count(r)) return;  // re-queued by done()
  queue_.push_back(r);
  depth_->set({name_}, static_cast<double>(queue_.size()));
  cv_.notify_one();
}

void WorkQueue::add_after(const Request& r, double seconds) {
  if (seconds <= 0) {
    add(r);
    return;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (shutdown_) return;
  // keep only the earliest pending timer for an item
  for (auto it = delayed_.begin(); it != delayed_.end(); ++it)
    if (it->second == r) {
      if (it->first <= now_seconds() + seconds) return;
      delayed_.erase(it);
      break;
    }
  delayed_.emplace(now_seconds() + seconds, r);
  delay_cv_.notify_one();
}

void WorkQueue::add_rate_limited(const Request& r) {
  double delay;
  {
    std::lock_guard<std::mutex> g(mu_);
    int n = failures_[r]++;
    delay = std::min(max_, base_ * std::pow(2.0, n));
    // token bucket (overall)
    double now = now_seconds();
    tokens_ = std::min<double>(burst_, tokens_ + (now - last_refill_) * qps_);
    last_refill_ = now;
    if (tokens_ >= 1) {
      tokens_ -= 1;
    } else {
      delay = std::max(delay, (1 - tokens_) / qps_);
      tokens_ -= 1;
    }
    retries_->inc({name_});
  }
  add_after(r, delay);
}

void WorkQueue::forget(const Request& r) {
  std::lock_guard<std::mutex> g(mu_);
  failures_.erase(r);
}

int WorkQueue::num_requeues(const Request& r) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = failures_.find(r);
  return it == failures_.end() ? 0 : it->second;
}

bool WorkQueue::get(Request& out, int timeout_ms) {
  std::unique_lock<std::mutex> g(mu_);
  if (!cv_.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return !queue_.empty() || shutdown_; })) return false;
  if (queue_.empty()) return false;
  out = queue_.front();
  queue_.pop_front();
  dirty_.erase(out);
  processing_.insert(out);
  auto at = added_at_.find(out);
  if (at != added_at_.end()) {
    queue_dur_->observe({name_}, now_seconds() - at->second);
    added_at_.erase(at);
  }
  depth_->set({name_}, static_cast<double>(queue_.size()));
  return true;
}

void WorkQueue::done(const Request& r) {
  std::lock_guard<std::mutex> g(mu_);
  processing_.erase(r);
  if (dirty_.count(r)) {
    queue_.push_back(r);
    cv_.notify_one();
  }
}

void WorkQueue::shutdown() {
  {
    std::lock_guard<std::mutex> g(mu_);
    shutdown_ = true;
  }
  cv_.notify_all();
  delay_cv_.notify_all();
}

size_t WorkQueue::len() const {
  std::lock_guard<std::mutex> g(mu_);
  return queue_.size();
}

void WorkQueue::delay_loop() {
  std::unique_lock<std::mutex> g(mu_);
  while (!shutdown_) {
    if (delayed_.empty()) {
      delay_cv_.wait_for(g, std::chrono::milliseconds(500));
      continue;
    }
    double now = now_seconds();
    auto it = delayed_.begin();
    if (it->first > now) {
      delay_cv_.wait_for(g, std::chrono::microseconds(static_cast<int64_t>((it->first - now) * 1e6) + 100));
      continue;
    }
    Request r = it->second;
    delayed_.erase(it);
    if (!dirty_.count(r)) {
      dirty_.insert(r);
      added_at_.emplace(r, now);
      if (!processing_.count(r)) {
        queue_.push_back(r);
        cv_.notify_one();
      }
    }
  }
}

}  // namespace kf
