// Environment knobs (docs/TUNING.md). Production knobs are plain std::getenv reads at
// construction. Study knobs - A/B settings, negative controls and measurement switches that
// can make a run slower or wrong - are read through study_env(): it returns the value only
// when MXAR_STUDY=1 is set as well, so a stray variable never changes a production run.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>
#include <string>

namespace mxar {

inline bool study_mode() {
  static const bool on = [] {
    const char* s = std::getenv("MXAR_STUDY");
    return s != nullptr && s[0] != '\0' && s[0] != '0';
  }();
  return on;
}

// The study knob `name`, or nullptr outside study mode (a set knob is then reported once per
// process, however many communicators or planes read it).
inline const char* study_env(const char* name) {
  const char* v = std::getenv(name);
  if (v == nullptr) return nullptr;
  if (study_mode()) return v;
  static std::mutex mu;
  static std::set<std::string> reported;
  std::lock_guard<std::mutex> g(mu);
  if (reported.insert(name).second)
    std::fprintf(stderr, "[mxar] %s ignored: study knob, needs MXAR_STUDY=1 (docs/TUNING.md)\n", name);
  return nullptr;
}

}  // namespace mxar
