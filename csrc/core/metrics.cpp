// SPDX-License-Identifier: Apache-2.0
#include "metrics.h"

#include <cmath>
#include <cstdio>
#include <sstream>

namespace pdo {

Metrics& Metrics::global() {
  static Metrics m;
  return m;
}

std::string label_str(const Labels& l) {
  if (l.empty()) return "";
  std::string s = "{";
  bool first = true;
  for (auto& kv : l) {
    if (!first) s += ",";
    first = false;
    s += kv.first + "=\"";
    for (char c : kv.second) {
      if (c == '"' || c == '\\') s.push_back('\\');
      if (c == '\n') {
        s += "\\n";
        continue;
      }
      s.push_back(c);
    }
    s += "\"";
  }
  return s + "}";
}

void Metrics::help(const std::string& name, const std::string& type, const std::string& text) {
  std::lock_guard<std::mutex> g(mu_);
  meta_[name] = {type, text};
}

void Metrics::inc(const std::string& name, const Labels& l, double v) {
  std::lock_guard<std::mutex> g(mu_);
  if (!meta_.count(name)) meta_[name] = {"counter", name};
  scalars_[name][label_str(l)] += v;
}

void Metrics::set(const std::string& name, const Labels& l, double v) {
  std::lock_guard<std::mutex> g(mu_);
  if (!meta_.count(name)) meta_[name] = {"gauge", name};
  scalars_[name][label_str(l)] = v;
}

void Metrics::observe(const std::string& name, const Labels& l, double v) {
  std::lock_guard<std::mutex> g(mu_);
  if (!meta_.count(name)) meta_[name] = {"histogram", name};
  Hist& h = hists_[name][label_str(l)];
  if (h.counts.empty()) h.counts.assign(buckets.size(), 0);
  for (size_t i = 0; i < buckets.size(); ++i)
    if (v <= buckets[i]) h.counts[i] += 1;
  h.sum += v;
  h.count += 1;
}

double Metrics::get(const std::string& name, const Labels& l) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = scalars_.find(name);
  if (it == scalars_.end()) return 0;
  auto jt = it->second.find(label_str(l));
  return jt == it->second.end() ? 0 : jt->second;
}

static std::string num(double v) {
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  char b[64];
  snprintf(b, sizeof b, "%.9g", v);
  return b;
}

static std::string with_le(const std::string& ls, const std::string& le) {
  if (ls.empty()) return "{le=\"" + le + "\"}";
  return ls.substr(0, ls.size() - 1) + ",le=\"" + le + "\"}";
}

std::string Metrics::expose() const {
  std::lock_guard<std::mutex> g(mu_);
  std::ostringstream out;
  for (auto& m : meta_) {
    const std::string& name = m.first;
    out << "# HELP " << name << " " << m.second.second << "\n# TYPE " << name << " " << m.second.first << "\n";
    auto s = scalars_.find(name);
    if (s != scalars_.end())
      for (auto& kv : s->second) out << name << kv.first << " " << num(kv.second) << "\n";
    auto h = hists_.find(name);
    if (h != hists_.end()) {
      for (auto& kv : h->second) {
        for (size_t i = 0; i < buckets.size(); ++i)
          out << name << "_bucket" << with_le(kv.first, num(buckets[i])) << " " << num(kv.second.counts[i]) << "\n";
        out << name << "_bucket" << with_le(kv.first, "+Inf") << " " << num(kv.second.count) << "\n";
        out << name << "_sum" << kv.first << " " << num(kv.second.sum) << "\n";
        out << name << "_count" << kv.first << " " << num(kv.second.count) << "\n";
      }
    }
  }
  return out.str();
}

void Metrics::reset() {
  std::lock_guard<std::mutex> g(mu_);
  scalars_.clear();
  hists_.clear();
}

}  // namespace pdo
