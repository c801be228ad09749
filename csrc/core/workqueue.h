// SPDX-License-Identifier: Apache-2.0
// Deduplicating, rate-limited work queue with delayed requeue.
//
// Semantics of client-go's workqueue as controller-runtime uses it for the
// reference reconciler (`Requeue`, `RequeueAfter`, error backoff): a key is
// never processed by two workers at once; adding a key that is queued is a
// no-op; adding a key that is being processed re-queues it after `done`;
// `add_rate_limited` backs off per key exponentially (5 ms · 2^n, ≤ 1000 s)
// until `forget`.  Time is injectable so tests can run on a virtual clock.
#pragma once

#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "api.h"

namespace pdo {

class WorkQueue {
 public:
  explicit WorkQueue(api::Clock clock = api::wall_clock) : clock_(std::move(clock)) {}

  void add(const std::string& key);
  void add_after(const std::string& key, double delay_s);
  void add_rate_limited(const std::string& key);
  void forget(const std::string& key);
  int retries(const std::string& key) const;

  // next ready key; blocks up to timeout_s (0 = poll). false if none.
  bool get(std::string* key, double timeout_s);
  void done(const std::string& key);

  void shutdown();
  bool shutting_down() const;
  size_t len() const;            // ready + waiting-for-time
  double next_ready_in() const;  // seconds until the earliest delayed key (inf if none)
  void promote_due();            // move due delayed keys to ready (virtual clock)

  double base_delay = 0.005;
  double max_delay = 1000.0;

 private:
  void add_locked(const std::string& key);
  void promote_locked(double now);

  api::Clock clock_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::string> queue_;
  std::set<std::string> dirty_, processing_;
  std::multimap<double, std::string> waiting_;
  std::map<std::string, int> failures_;
  bool shutdown_ = false;
};

}  // namespace pdo
