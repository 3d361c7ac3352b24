// Device-wide budget of SPINNING workgroups in this process. The protocol engine's kernels
// wait for each other inside one launch (a plane group's slices, a resident kernel's
// workgroups and their peers): every workgroup of such a kernel must be resident at once, or
// the resident ones spin forever on work that never gets a CU. One group checking only its
// own size (Y x grid <= 2 x CUs) cannot see a second job's group kernel, a lone worker's
// resident kernel or anything else that spins beside it, so every kernel that stays on the
// GPU waiting reserves its workgroups here first: what does not fit fails loudly with the
// budget named (or, for an optional resident kernel, falls back to one launch per round)
// instead of timing out on the device.
//
// Capacity: 2 workgroups of 256 threads per CU (the plane default of round 3 onward: every
// threshold / group kernel fits twice per CU by registers and LDS), MXAR_RESIDENCY_WGS
// overrides it per device.
#pragma once

#include <memory>
#include <string>
#include <vector>

namespace mxar {

struct ResidencyHolder {
  std::string who;
  int wgs = 0;
};

class Residency {
 public:
  static Residency& get();
  // Reserves `wgs` workgroups on `device` for as long as the returned token lives. Throws
  // ProtocolError naming the budget, what is held and by whom, when they do not fit.
  std::shared_ptr<void> reserve(int device, int wgs, const std::string& who);
  // The same, but returns nullptr instead of throwing (optional resident kernels).
  std::shared_ptr<void> try_reserve(int device, int wgs, const std::string& who);
  int capacity(int device);
  int used(int device);
  std::vector<ResidencyHolder> holders(int device);

 private:
  Residency() = default;
  struct Impl;
  Impl& impl();
};

}  // namespace mxar
