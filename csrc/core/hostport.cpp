// SPDX-License-Identifier: Apache-2.0
#include "hostport.h"

#include <cstdlib>

namespace pdo {

bool HostPorts::parse_range(const std::string& spec, int* start, int* end) {
  size_t c = spec.find(',');
  if (c == std::string::npos) return false;
  char* e1 = nullptr;
  char* e2 = nullptr;
  long a = strtol(spec.substr(0, c).c_str(), &e1, 10);
  std::string tail = spec.substr(c + 1);
  long b = strtol(tail.c_str(), &e2, 10);
  if (!e1 || *e1 || !e2 || *e2 || a <= 0 || b <= a || b > 65535) return false;
  *start = (int)a;
  *end = (int)b;
  return true;
}

int HostPorts::allocate() {
  std::lock_guard<std::mutex> g(mu_);
  return alloc_locked(0);
}

int HostPorts::alloc_locked(int depth) {
  // capacity check mirrors `len(map)*20 > end-start` (the map also holds the
  // three bookkeeping keys in the reference, hence +3)
  if ((int)(used_.size() + 3) * kBlock > end_ - start_) return kFallback;
  if (depth > (end_ - start_) / kBlock + 1) return kFallback;
  int next = cur_ + kBlock;
  if (next > end_) next = start_;
  cur_ = next;
  if (used_.count(next)) return alloc_locked(depth + 1);
  used_.insert(next);
  return next;
}

bool HostPorts::registered(int port) const {
  std::lock_guard<std::mutex> g(mu_);
  return used_.count(port) > 0;
}

void HostPorts::register_port(int port) {
  std::lock_guard<std::mutex> g(mu_);
  used_.insert(port);
}

bool HostPorts::release(int port) {
  std::lock_guard<std::mutex> g(mu_);
  return used_.erase(port) > 0;
}

size_t HostPorts::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return used_.size();
}

}  // namespace pdo
