// Leveled logger with the reference's event vocabulary.
//   reference: akka.actor.ActorLogging in AllreduceMaster.scala:24, AllreduceWorker.scala:10,
//              level from application.conf:22 (akka.loglevel = "INFO").
// Payload dumps (the reference logs full arrays at INFO/DEBUG) are emitted at TRACE only.
// Level: MXAR_LOGLEVEL=TRACE|DEBUG|INFO|WARNING|ERROR|OFF (default WARNING). The sink is
// stderr unless the Python layer installs its own (it forwards to `logging`).
#pragma once

#include <atomic>
#include <functional>
#include <mutex>
#include <sstream>
#include <string>

namespace mxar {

enum class LogLevel : int { TRACE = 0, DEBUG = 1, INFO = 2, WARNING = 3, ERROR = 4, OFF = 5 };

class Logger {
 public:
  using Sink = std::function<void(LogLevel, const std::string& source, const std::string& msg)>;
  static Logger& get();
  bool enabled(LogLevel l) const { return static_cast<int>(l) >= level_.load(std::memory_order_relaxed); }
  void set_level(LogLevel l) { level_.store(static_cast<int>(l)); }
  LogLevel level() const { return static_cast<LogLevel>(level_.load()); }
  void set_sink(Sink s);
  void log(LogLevel l, const std::string& source, const std::string& msg);
  static const char* level_name(LogLevel l);
  static LogLevel parse(const std::string& s);

 private:
  Logger();
  std::atomic<int> level_;
  std::mutex mu_;
  Sink sink_;
};

}  // namespace mxar

#define MXAR_LOG(lvl, src, expr)                                              \
  do {                                                                        \
    if (::mxar::Logger::get().enabled(::mxar::LogLevel::lvl)) {               \
      std::ostringstream _mxar_os;                                            \
      _mxar_os << expr;                                                       \
      ::mxar::Logger::get().log(::mxar::LogLevel::lvl, (src), _mxar_os.str()); \
    }                                                                         \
  } while (0)
