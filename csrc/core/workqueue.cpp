// SPDX-License-Identifier: Apache-2.0
#include "workqueue.h"

#include <chrono>
#include <cmath>
#include <limits>

namespace pdo {

void WorkQueue::add_locked(const std::string& key) {
  if (shutdown_ || dirty_.count(key)) return;
  dirty_.insert(key);
  if (processing_.count(key)) return;  // re-queued by done()
  queue_.push_back(key);
  cv_.notify_one();
}

void WorkQueue::add(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  add_locked(key);
}

void WorkQueue::add_after(const std::string& key, double delay_s) {
  std::lock_guard<std::mutex> g(mu_);
  if (shutdown_) return;
  if (delay_s <= 0) {
    add_locked(key);
    return;
  }
  const double t = clock_() + delay_s;
  // keep only the earliest pending time for a key
  for (auto it = waiting_.begin(); it != waiting_.end(); ++it) {
    if (it->second == key) {
      if (it->first <= t) return;
      waiting_.erase(it);
      break;
    }
  }
  waiting_.emplace(t, key);
  cv_.notify_all();
}

void WorkQueue::add_rate_limited(const std::string& key) {
  double d;
  {
    std::lock_guard<std::mutex> g(mu_);
    int n = failures_[key]++;
    d = base_delay * std::pow(2.0, std::min(n, 40));
    if (d > max_delay) d = max_delay;
  }
  add_after(key, d);
}

void WorkQueue::forget(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  failures_.erase(key);
}

int WorkQueue::retries(const std::string& key) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = failures_.find(key);
  return it == failures_.end() ? 0 : it->second;
}

void WorkQueue::promote_locked(double now) {
  while (!waiting_.empty() && waiting_.begin()->first <= now) {
    std::string k = waiting_.begin()->second;
    waiting_.erase(waiting_.begin());
    add_locked(k);
  }
}

void WorkQueue::promote_due() {
  std::lock_guard<std::mutex> g(mu_);
  promote_locked(clock_());
}

bool WorkQueue::get(std::string* key, double timeout_s) {
  std::unique_lock<std::mutex> l(mu_);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (true) {
    promote_locked(clock_());
    if (!queue_.empty()) break;
    if (shutdown_) return false;
    const auto now = std::chrono::steady_clock::now();
    if (timeout_s <= 0 || now >= deadline) return false;
    auto until = deadline;
    if (!waiting_.empty()) {
      const double dt = waiting_.begin()->first - clock_();
      auto w = now + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                         std::chrono::duration<double>(std::max(0.0, dt)));
      if (w < until) until = w;
    }
    // system_clock wait → pthread_cond_timedwait.  (A steady_clock wait is
    // pthread_cond_clockwait in libstdc++ 11, which gcc-11's TSan does not
    // intercept: every wait then reads as a held lock / false data race.)
    cv_.wait_until(l, std::chrono::system_clock::now() +
                          std::chrono::duration_cast<std::chrono::system_clock::duration>(until - now));
  }
  *key = queue_.front();
  queue_.pop_front();
  processing_.insert(*key);
  dirty_.erase(*key);
  return true;
}

void WorkQueue::done(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  processing_.erase(key);
  if (dirty_.count(key)) {
    queue_.push_back(key);
    cv_.notify_one();
  }
}

void WorkQueue::shutdown() {
  std::lock_guard<std::mutex> g(mu_);
  shutdown_ = true;
  cv_.notify_all();
}

bool WorkQueue::shutting_down() const {
  std::lock_guard<std::mutex> g(mu_);
  return shutdown_;
}

size_t WorkQueue::len() const {
  std::lock_guard<std::mutex> g(mu_);
  return queue_.size() + waiting_.size();
}

double WorkQueue::next_ready_in() const {
  std::lock_guard<std::mutex> g(mu_);
  if (!queue_.empty()) return 0;
  if (waiting_.empty()) return std::numeric_limits<double>::infinity();
  return std::max(0.0, waiting_.begin()->first - clock_());
}

}  // namespace pdo
