#include "log.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace mxar {

Logger& Logger::get() {
  static Logger inst;
  return inst;
}

Logger::Logger() : level_(static_cast<int>(LogLevel::WARNING)) {
  if (const char* e = std::getenv("MXAR_LOGLEVEL")) level_ = static_cast<int>(parse(e));
}

void Logger::set_sink(Sink s) {
  std::lock_guard<std::mutex> g(mu_);
  sink_ = std::move(s);
}

void Logger::log(LogLevel l, const std::string& source, const std::string& msg) {
  Sink s;
  {
    std::lock_guard<std::mutex> g(mu_);
    s = sink_;
  }
  if (s) {
    s(l, source, msg);
    return;
  }
  using namespace std::chrono;
  const double t = duration<double>(system_clock::now().time_since_epoch()).count();
  std::fprintf(stderr, "[%.6f] [%s] [%s] %s\n", t, level_name(l), source.c_str(), msg.c_str());
}

const char* Logger::level_name(LogLevel l) {
  switch (l) {
    case LogLevel::TRACE: return "TRACE";
    case LogLevel::DEBUG: return "DEBUG";
    case LogLevel::INFO: return "INFO";
    case LogLevel::WARNING: return "WARNING";
    case LogLevel::ERROR: return "ERROR";
    default: return "OFF";
  }
}

LogLevel Logger::parse(const std::string& s) {
  if (s == "TRACE" || s == "trace") return LogLevel::TRACE;
  if (s == "DEBUG" || s == "debug") return LogLevel::DEBUG;
  if (s == "INFO" || s == "info") return LogLevel::INFO;
  if (s == "WARNING" || s == "warning" || s == "WARN" || s == "warn") return LogLevel::WARNING;
  if (s == "ERROR" || s == "error") return LogLevel::ERROR;
  return LogLevel::OFF;
}

}  // namespace mxar
