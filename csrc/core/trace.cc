#include "trace.h"

#include <unistd.h>

#include <cstdlib>
#include <functional>
#include <iomanip>
#include <sstream>
#include <thread>

#ifndef MXAR_NO_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#else  // host-only sanitizer builds (tools/sanitize.py) do not link roctx
static inline void roctxRangePushA(const char*) {}
static inline void roctxRangePop() {}
#endif

namespace mxar {

namespace {
uint32_t thread_tag() {
  static thread_local uint32_t tag =
      static_cast<uint32_t>(std::hash<std::thread::id>()(std::this_thread::get_id()) & 0x7fffffff);
  return tag;
}

void json_escape(std::ostringstream& os, const std::string& s) {
  for (char c : s) {
    if (c == '"' || c == '\\')
      os << '\\' << c;
    else if (static_cast<unsigned char>(c) < 0x20)
      os << ' ';
    else
      os << c;
  }
}
}  // namespace

Tracer::Tracer() {
  if (const char* e = std::getenv("MXAR_TRACE")) enabled_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("MXAR_ROCTX")) roctx_ = std::atoi(e) != 0;
}

Tracer& Tracer::get() {
  static Tracer t;
  return t;
}

void Tracer::enable(bool on) { enabled_.store(on); }

void Tracer::record(const char* cat, const std::string& name, uint64_t ts_ns, uint64_t dur_ns, char ph,
                    const std::string& args_json) {
  std::lock_guard<std::mutex> g(mu_);
  if (ev_.size() >= cap_) {
    ++dropped_;
    return;
  }
  ev_.push_back(Event{cat, name, args_json, ts_ns, dur_ns, thread_tag(), ph});
}

std::string Tracer::dump_json() {
  std::lock_guard<std::mutex> g(mu_);
  std::ostringstream os;
  // microseconds with ns resolution: the default 6 significant digits would collapse every
  // event of a process that has been up for more than a second onto one timestamp
  os << std::fixed << std::setprecision(3);
  const int pid = static_cast<int>(getpid());
  os << "{\"displayTimeUnit\":\"ms\",\"otherData\":{\"dropped\":" << dropped_ << "},\"traceEvents\":[";
  bool first = true;
  for (const auto& e : ev_) {
    if (!first) os << ",";
    first = false;
    os << "{\"cat\":\"";
    json_escape(os, e.cat);
    os << "\",\"name\":\"";
    json_escape(os, e.name);
    os << "\",\"ph\":\"" << e.ph << "\",\"pid\":" << pid << ",\"tid\":" << e.tid << ",\"ts\":" << (e.ts / 1000.0);
    if (e.ph == 'X') os << ",\"dur\":" << (e.dur / 1000.0);
    if (e.ph == 'i') os << ",\"s\":\"t\"";
    if (!e.args.empty()) os << ",\"args\":" << e.args;
    os << "}";
  }
  os << "]}";
  return os.str();
}

size_t Tracer::size() {
  std::lock_guard<std::mutex> g(mu_);
  return ev_.size();
}

void Tracer::clear() {
  std::lock_guard<std::mutex> g(mu_);
  ev_.clear();
  dropped_ = 0;
}

TraceScope::TraceScope(const char* cat, std::string name, std::string args)
    : cat_(cat), name_(std::move(name)), args_(std::move(args)) {
  Tracer& t = Tracer::get();
  on_ = t.enabled();
  rx_ = t.roctx();
  begin();
}

void TraceScope::begin() {
  if (rx_) roctxRangePushA(name_.c_str());
  if (on_) t0_ = Tracer::now_ns();
}

TraceScope::~TraceScope() {
  if (on_) {
    const uint64_t t1 = Tracer::now_ns();
    Tracer::get().record(cat_, name_, t0_, t1 - t0_, 'X', args_);
  }
  if (rx_) roctxRangePop();
}

}  // namespace mxar
