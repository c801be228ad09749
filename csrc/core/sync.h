// SPDX-License-Identifier: Apache-2.0
// Condition-variable timed waits on system_clock.
//
// libstdc++ 11 implements steady_clock waits with pthread_cond_clockwait,
// which gcc-11's ThreadSanitizer does not intercept: the TSan build then sees
// every timed wait as a mutex that is never released (false "double lock" /
// data-race reports).  system_clock waits go through pthread_cond_timedwait.
#pragma once

#include <chrono>
#include <condition_variable>
#include <mutex>

namespace pdo {

template <class Pred>
bool wait_for_s(std::condition_variable& cv, std::unique_lock<std::mutex>& l, double seconds, Pred pred) {
  const auto until = std::chrono::system_clock::now() +
                     std::chrono::duration_cast<std::chrono::system_clock::duration>(
                         std::chrono::duration<double>(seconds));
  return cv.wait_until(l, until, pred);
}

}  // namespace pdo
