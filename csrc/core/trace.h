// Process-wide event tracer: a Chrome-trace ("traceEvents") JSON timeline of protocol and
// engine events, plus roctx ranges so the same spans show up in `rocprofv3 --marker-trace`.
// The reference has no tracing at all; this records per-round
// fetch / scatter / reduce / complete spans of every worker, forced catch-ups, cluster
// membership events and allreduce launches. Off by default (MXAR_TRACE=1 or
// Tracer::get().enable(true)); a disabled tracer costs one relaxed atomic load per site.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <mutex>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

namespace mxar {

class Tracer {
 public:
  static Tracer& get();
  bool enabled() const { return enabled_.load(std::memory_order_relaxed); }
  void enable(bool on);
  void set_roctx(bool on) { roctx_ = on; }
  bool roctx() const { return roctx_; }
  // ph = 'X' complete event (dur_ns) or 'i' instant event
  void record(const char* cat, const std::string& name, uint64_t ts_ns, uint64_t dur_ns, char ph,
              const std::string& args_json = "");
  std::string dump_json();
  size_t size();
  void clear();
  static uint64_t now_ns() {
    return static_cast<uint64_t>(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
            .count());
  }

 private:
  Tracer();
  struct Event {
    std::string cat, name, args;
    uint64_t ts, dur;
    uint32_t tid;
    char ph;
  };
  std::atomic<bool> enabled_{false};
  bool roctx_ = false;
  std::mutex mu_;
  std::vector<Event> ev_;
  size_t cap_ = 1u << 20;
  uint64_t dropped_ = 0;
};

// RAII span: records a complete event (and a roctx range) when the tracer is on.
// The lazy form takes a callable returning {name, args_json}; it is only invoked when the
// tracer or roctx is on, so a hot path pays no string building while tracing is off.
class TraceScope {
 public:
  TraceScope(const char* cat, std::string name, std::string args = "");
  template <class Fn, class = std::enable_if_t<std::is_invocable_v<Fn>>>
  TraceScope(const char* cat, Fn&& make) : cat_(cat) {
    Tracer& t = Tracer::get();
    on_ = t.enabled();
    rx_ = t.roctx();
    if (on_ || rx_) {
      auto na = make();
      name_ = std::move(na.first);
      args_ = std::move(na.second);
      begin();
    }
  }
  ~TraceScope();
  TraceScope(const TraceScope&) = delete;
  TraceScope& operator=(const TraceScope&) = delete;

 private:
  void begin();
  const char* cat_;
  std::string name_, args_;
  uint64_t t0_ = 0;
  bool on_ = false, rx_ = false;
};

inline void trace_instant(const char* cat, const std::string& name, const std::string& args = "") {
  Tracer& t = Tracer::get();
  if (t.enabled()) t.record(cat, name, Tracer::now_ns(), 0, 'i', args);
}

}  // namespace mxar
