// metrics.cc — see metrics.h.
#include "core/metrics.h"

#include <cmath>
#include <cstdio>

namespace kf {

namespace {
std::string fmt(double v) {
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  if (std::isnan(v)) return "NaN";
  char buf[64];
  if (v == std::floor(v) && std::fabs(v) < 1e15) std::snprintf(buf, sizeof buf, "%.0f", v);
  else std::snprintf(buf, sizeof buf, "%.9g", v);
  return buf;
}
std::string esc(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '\\') o += "\\\\";
    else if (c == '"') o += "\\\"";
    else if (c == '\n') o += "\\n";
    else o += c;
  }
  return o;
}
}  // namespace

std::string MetricFamily::label_str(const Labels& values, const std::string& extra) const {
  std::string s;
  for (size_t i = 0; i < label_names_.size() && i < values.size(); ++i) {
    if (!s.empty()) s += ",";
    s += label_names_[i] + "=\"" + esc(values[i]) + "\"";
  }
  if (!extra.empty()) {
    if (!s.empty()) s += ",";
    s += extra;
  }
  return s.empty() ? "" : "{" + s + "}";
}

void CounterVec::inc(const Labels& lv, double by) {
  std::lock_guard<std::mutex> g(mu_);
  vals_[lv] += by;
}
double CounterVec::value(const Labels& lv) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = vals_.find(lv);
  return it == vals_.end() ? 0.0 : it->second;
}
void CounterVec::expose(std::string& out) const {
  std::lock_guard<std::mutex> g(mu_);
  out += "# HELP " + name_ + " " + help_ + "\n# TYPE " + name_ + " counter\n";
  for (const auto& kv : vals_) out += name_ + label_str(kv.first) + " " + fmt(kv.second) + "\n";
}

void GaugeVec::set(const Labels& lv, double v) {
  std::lock_guard<std::mutex> g(mu_);
  vals_[lv] = v;
}
void GaugeVec::add(const Labels& lv, double v) {
  std::lock_guard<std::mutex> g(mu_);
  vals_[lv] += v;
}
double GaugeVec::value(const Labels& lv) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = vals_.find(lv);
  return it == vals_.end() ? 0.0 : it->second;
}
void GaugeVec::reset() {
  std::lock_guard<std::mutex> g(mu_);
  vals_.clear();
}
void GaugeVec::expose(std::string& out) const {
  std::lock_guard<std::mutex> g(mu_);
  out += "# HELP " + name_ + " " + help_ + "\n# TYPE " + name_ + " gauge\n";
  for (const auto& kv : vals_) out += name_ + label_str(kv.first) + " " + fmt(kv.second) + "\n";
}

HistogramVec::HistogramVec(std::string name, std::string help, std::vector<std::string> labels,
                           std::vector<double> buckets)
    : MetricFamily(std::move(name), std::move(help), "histogram", std::move(labels)), buckets_(std::move(buckets)) {}

std::vector<double> HistogramVec::exponential(double start, double factor, int count) {
  std::vector<double> b;
  double v = start;
  for (int i = 0; i < count; ++i) {
    b.push_back(v);
    v *= factor;
  }
  return b;
}

void HistogramVec::observe(const Labels& lv, double v) {
  std::lock_guard<std::mutex> g(mu_);
  H& h = vals_[lv];
  if (h.counts.empty()) h.counts.assign(buckets_.size(), 0);
  for (size_t i = 0; i < buckets_.size(); ++i)
    if (v <= buckets_[i]) h.counts[i]++;
  h.sum += v;
  h.n++;
}

uint64_t HistogramVec::count(const Labels& lv) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = vals_.find(lv);
  return it == vals_.end() ? 0 : it->second.n;
}

double HistogramVec::quantile(const Labels& lv, double q) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = vals_.find(lv);
  if (it == vals_.end() || it->second.n == 0) return NAN;
  const H& h = it->second;
  double rank = q * static_cast<double>(h.n);
  double prev_bound = 0;
  uint64_t prev_count = 0;
  for (size_t i = 0; i < buckets_.size(); ++i) {
    if (static_cast<double>(h.counts[i]) >= rank) {
      uint64_t in_bucket = h.counts[i] - prev_count;
      if (in_bucket == 0) return buckets_[i];
      return prev_bound + (buckets_[i] - prev_bound) * (rank - static_cast<double>(prev_count)) / static_cast<double>(in_bucket);
    }
    prev_bound = buckets_[i];
    prev_count = h.counts[i];
  }
  return buckets_.empty() ? NAN : buckets_.back();
}

void HistogramVec::expose(std::string& out) const {
  std::lock_guard<std::mutex> g(mu_);
  out += "# HELP " + name_ + " " + help_ + "\n# TYPE " + name_ + " histogram\n";
  for (const auto& kv : vals_) {
    for (size_t i = 0; i < buckets_.size(); ++i)
      out += name_ + "_bucket" + label_str(kv.first, "le=\"" + fmt(buckets_[i]) + "\"") + " " +
             std::to_string(kv.second.counts[i]) + "\n";
    out += name_ + "_bucket" + label_str(kv.first, "le=\"+Inf\"") + " " + std::to_string(kv.second.n) + "\n";
    out += name_ + "_sum" + label_str(kv.first) + " " + fmt(kv.second.sum) + "\n";
    out += name_ + "_count" + label_str(kv.first) + " " + std::to_string(kv.second.n) + "\n";
  }
}

void CollectorFamily::expose(std::string& out) const {
  out += "# HELP " + name_ + " " + help_ + "\n# TYPE " + name_ + " " + type_ + "\n";
  for (const auto& kv : fn_()) out += name_ + label_str(kv.first) + " " + fmt(kv.second) + "\n";
}

Registry& Registry::global() {
  static Registry r;
  return r;
}

std::shared_ptr<CounterVec> Registry::counter(const std::string& name, const std::string& help, std::vector<std::string> labels) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = fams_.find(name);
  if (it != fams_.end()) return std::dynamic_pointer_cast<CounterVec>(it->second);
  auto c = std::make_shared<CounterVec>(name, help, std::move(labels));
  fams_[name] = c;
  return c;
}
std::shared_ptr<GaugeVec> Registry::gauge(const std::string& name, const std::string& help, std::vector<std::string> labels) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = fams_.find(name);
  if (it != fams_.end()) return std::dynamic_pointer_cast<GaugeVec>(it->second);
  auto c = std::make_shared<GaugeVec>(name, help, std::move(labels));
  fams_[name] = c;
  return c;
}
std::shared_ptr<HistogramVec> Registry::histogram(const std::string& name, const std::string& help,
                                                  std::vector<std::string> labels, std::vector<double> buckets) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = fams_.find(name);
  if (it != fams_.end()) return std::dynamic_pointer_cast<HistogramVec>(it->second);
  auto c = std::make_shared<HistogramVec>(name, help, std::move(labels), std::move(buckets));
  fams_[name] = c;
  return c;
}
void Registry::add_collector(std::shared_ptr<MetricFamily> f) {
  std::lock_guard<std::mutex> g(mu_);
  fams_[f->name()] = std::move(f);
}
bool Registry::unregister(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  return fams_.erase(name) > 0;
}
std::string Registry::expose() const {
  std::vector<std::shared_ptr<MetricFamily>> fams;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& kv : fams_) fams.push_back(kv.second);
  }
  std::string out;
  for (const auto& f : fams) f->expose(out);
  return out;
}

}  // namespace kf
