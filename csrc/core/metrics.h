// SPDX-License-Identifier: Apache-2.0
// Prometheus text-exposition registry (counters, gauges, histograms).
//
// The reference exposes controller-runtime's default registry on
// --metrics-bind-address (main.go:70,90): reconcile totals/errors/latency and
// workqueue depth/latency.  pdo exposes the same families under the same
// names plus launch-path metrics (SURVEY §5.5 [design]):
//   pdo_job_phase_transition_seconds{from,to}, pdo_job_ready_seconds,
//   pdo_reconcile_actions_total{kind}.
#pragma once

#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace pdo {

using Labels = std::map<std::string, std::string>;

class Metrics {
 public:
  static Metrics& global();
  void inc(const std::string& name, const Labels& l = {}, double v = 1.0);
  void set(const std::string& name, const Labels& l, double v);
  void observe(const std::string& name, const Labels& l, double v);
  void help(const std::string& name, const std::string& type, const std::string& text);
  double get(const std::string& name, const Labels& l = {}) const;  // counter/gauge value
  std::string expose() const;
  void reset();

  std::vector<double> buckets = {0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60};

 private:
  struct Hist {
    std::vector<double> counts;
    double sum = 0;
    double count = 0;
  };
  static std::string key(const std::string& name, const Labels& l);
  mutable std::mutex mu_;
  std::map<std::string, std::pair<std::string, std::string>> meta_;  // name → (type, help)
  std::map<std::string, std::map<std::string, double>> scalars_;     // name → labelstr → v
  std::map<std::string, std::map<std::string, Hist>> hists_;
};

std::string label_str(const Labels& l);

}  // namespace pdo
