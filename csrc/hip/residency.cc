#include "residency.h"

#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <map>
#include <mutex>

#include "../core/data_buffer.h"

namespace mxar {

struct Residency::Impl {
  std::mutex mu;
  std::map<int, int> cap;
  std::map<int, std::map<uint64_t, ResidencyHolder>> held;  // device -> token id -> holder
  uint64_t next = 1;
};

Residency& Residency::get() {
  static Residency r;
  return r;
}

Residency::Impl& Residency::impl() {
  static Impl m;
  return m;
}

int Residency::capacity(int device) {
  Impl& m = impl();
  std::lock_guard<std::mutex> g(m.mu);
  auto it = m.cap.find(device);
  if (it != m.cap.end()) return it->second;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  (void)hipGetLastError();
  int c = 2 * cus;
  if (const char* e = std::getenv("MXAR_RESIDENCY_WGS")) c = std::max(1, std::atoi(e));
  m.cap[device] = c;
  return c;
}

int Residency::used(int device) {
  Impl& m = impl();
  std::lock_guard<std::mutex> g(m.mu);
  int u = 0;
  for (auto& [id, h] : m.held[device]) u += h.wgs;
  return u;
}

std::vector<ResidencyHolder> Residency::holders(int device) {
  Impl& m = impl();
  std::lock_guard<std::mutex> g(m.mu);
  std::vector<ResidencyHolder> v;
  for (auto& [id, h] : m.held[device]) v.push_back(h);
  return v;
}

std::shared_ptr<void> Residency::try_reserve(int device, int wgs, const std::string& who) {
  const int cap = capacity(device);
  Impl& m = impl();
  std::lock_guard<std::mutex> g(m.mu);
  int u = 0;
  for (auto& [id, h] : m.held[device]) u += h.wgs;
  if (wgs <= 0 || u + wgs > cap) return nullptr;
  const uint64_t id = m.next++;
  m.held[device][id] = ResidencyHolder{who, wgs};
  return std::shared_ptr<void>(reinterpret_cast<void*>(id), [device, id](void*) {
    Impl& mm = Residency::get().impl();
    std::lock_guard<std::mutex> gg(mm.mu);
    mm.held[device].erase(id);
  });
}

std::shared_ptr<void> Residency::reserve(int device, int wgs, const std::string& who) {
  if (auto t = try_reserve(device, wgs, who)) return t;
  std::string held;
  for (const ResidencyHolder& h : holders(device)) held += " " + h.who + "=" + std::to_string(h.wgs);
  throw ProtocolError("residency budget: " + who + " needs " + std::to_string(wgs) + " spinning workgroups on device " +
                      std::to_string(device) + ", " + std::to_string(capacity(device) - used(device)) + " of " +
                      std::to_string(capacity(device)) + " free (held:" + (held.empty() ? " none" : held) +
                      "; MXAR_RESIDENCY_WGS sets the budget)");
}

}  // namespace mxar
