// metrics.h — Prometheus client: counters, gauges, histograms (with label vectors), scrape-time
// collectors, and text exposition format 0.0.4. Replaces client_golang in the reference
// controllers (notebook-controller/pkg/metrics/metrics.go, profile-controller/controllers/monitoring.go,
// access-management/kfam/monitoring.go).
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace kf {

using Labels = std::vector<std::string>;  // label values in declaration order

class MetricFamily {
 public:
  MetricFamily(std::string name, std::string help, std::string type, std::vector<std::string> label_names)
      : name_(std::move(name)), help_(std::move(help)), type_(std::move(type)), label_names_(std::move(label_names)) {}
  virtual ~MetricFamily() = default;
  const std::string& name() const { return name_; }
  virtual void expose(std::string& out) const = 0;

 protected:
  std::string label_str(const Labels& values, const std::string& extra = "") const;
  std::string name_, help_, type_;
  std::vector<std::string> label_names_;
};

class CounterVec : public MetricFamily {
 public:
  CounterVec(std::string name, std::string help, std::vector<std::string> labels)
      : MetricFamily(std::move(name), std::move(help), "counter", std::move(labels)) {}
  void inc(const Labels& lv = {}, double by = 1.0);
  double value(const Labels& lv = {}) const;
  void expose(std::string& out) const override;

 private:
  mutable std::mutex mu_;
  std::map<Labels, double> vals_;
};

class GaugeVec : public MetricFamily {
 public:
  GaugeVec(std::string name, std::string help, std::vector<std::string> labels)
      : MetricFamily(std::move(name), std::move(help), "gauge", std::move(labels)) {}
  void set(const Labels& lv, double v);
  void add(const Labels& lv, double v);
  double value(const Labels& lv = {}) const;
  void reset();
  void expose(std::string& out) const override;

 private:
  mutable std::mutex mu_;
  std::map<Labels, double> vals_;
};

class HistogramVec : public MetricFamily {
 public:
  HistogramVec(std::string name, std::string help, std::vector<std::string> labels, std::vector<double> buckets);
  void observe(const Labels& lv, double v);
  // quantile estimate from buckets (linear interpolation), for in-process reporting
  double quantile(const Labels& lv, double q) const;
  uint64_t count(const Labels& lv) const;
  void expose(std::string& out) const override;
  static std::vector<double> exponential(double start, double factor, int count);

 private:
  struct H {
    std::vector<uint64_t> counts;
    double sum = 0;
    uint64_t n = 0;
  };
  std::vector<double> buckets_;
  mutable std::mutex mu_;
  std::map<Labels, H> vals_;
};

// Scrape-time collector (e.g. notebook_running computed from the StatefulSet list).
class CollectorFamily : public MetricFamily {
 public:
  using Fn = std::function<std::vector<std::pair<Labels, double>>()>;
  CollectorFamily(std::string name, std::string help, std::string type, std::vector<std::string> labels, Fn fn)
      : MetricFamily(std::move(name), std::move(help), std::move(type), std::move(labels)), fn_(std::move(fn)) {}
  void expose(std::string& out) const override;

 private:
  Fn fn_;
};

class Registry {
 public:
  static Registry& global();
  std::shared_ptr<CounterVec> counter(const std::string& name, const std::string& help, std::vector<std::string> labels = {});
  std::shared_ptr<GaugeVec> gauge(const std::string& name, const std::string& help, std::vector<std::string> labels = {});
  std::shared_ptr<HistogramVec> histogram(const std::string& name, const std::string& help,
                                          std::vector<std::string> labels, std::vector<double> buckets);
  void add_collector(std::shared_ptr<MetricFamily> f);
  bool unregister(const std::string& name);
  std::string expose() const;

 private:
  mutable std::mutex mu_;
  std::map<std::string, std::shared_ptr<MetricFamily>> fams_;
};

}  // namespace kf
