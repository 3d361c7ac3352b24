// A host delay accurate to a few microseconds: a straggling dataSource (the straggler bench,
// benchmarks/stragglers.py; `mxar-gpu --source-delay-us`). The OS sleep overshoots by tens of
// microseconds, so it covers all but the last 100 us, which are spun.
#pragma once

#include <chrono>
#include <thread>

namespace mxar {

inline void precise_delay_us(double us) {
  if (us <= 0.0) return;
  const auto until = std::chrono::steady_clock::now() + std::chrono::nanoseconds(static_cast<int64_t>(us * 1e3));
  if (us > 150.0) std::this_thread::sleep_for(std::chrono::microseconds(static_cast<int64_t>(us - 100.0)));
  while (std::chrono::steady_clock::now() < until) {
  }
}

}  // namespace mxar
