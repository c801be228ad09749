// SPDX-License-Identifier: Apache-2.0
// Host-network port-block allocator (Intranet=Host).
//
// Reference: controllers/paddlejob_controller.go:407-458 (HostPortMap,
// allocNewPort) + main.go:101-112,146-150.  Same observable allocation
// sequence (rolling cursor, blocks of 20, first block = start+20, wrap to
// start, fallback 40000 when exhausted) but thread-safe (the reference's
// unsynchronised map is safe only with one reconcile worker)
// and with O(1) membership.
#pragma once

#include <mutex>
#include <set>
#include <string>

namespace pdo {

class HostPorts {
 public:
  static constexpr int kBlock = 20;
  static constexpr int kFallback = 40000;
  HostPorts(int start = 35000, int end = 65000) : start_(start), end_(end), cur_(start) {}
  static bool parse_range(const std::string& spec, int* start, int* end);  // "35000,65000"

  void reset(int start, int end) {
    std::lock_guard<std::mutex> g(mu_);
    start_ = start;
    end_ = end;
    cur_ = start;
    used_.clear();
  }
  int allocate();                      // new block base port
  bool registered(int port) const;     // in the map (allocated or re-registered)
  void register_port(int port);        // after controller restart (annotation seen)
  bool release(int port);              // finalizer; true if it was registered
  size_t size() const;
  int start() const { return start_; }
  int end() const { return end_; }

 private:
  int alloc_locked(int depth);
  mutable std::mutex mu_;
  int start_, end_, cur_;
  std::set<int> used_;
};

}  // namespace pdo
