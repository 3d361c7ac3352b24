// SdmaComm (sdma_comm.h): bucket allreduce with the cross-rank traffic on the SDMA copy
// engines. Host side: HSA agents / engines, the per-call signal ring and the SDMA
// submissions. Device side: the signal release, the bounded flag wait, and the small-grid
// reduce and gather kernels.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <stdexcept>
#include <string>

#include "sdma_comm.h"
#include "xgmi_device.h"

namespace mxar {

namespace {

constexpr int kSlots = 16;              // calls in flight at most (signal / epoch-word ring)
constexpr int64_t kFlagBytes = 64 * 1024;
constexpr int kFrWord = 64;             // FR flags start at word 64 (FS at word 0)

void hsa_check(hsa_status_t s, const char* what) {
  if (s != HSA_STATUS_SUCCESS) {
    const char* m = nullptr;
    hsa_status_string(s, &m);
    throw std::runtime_error(std::string("HSA error in ") + what + ": " + (m ? m : "?"));
  }
}

int64_t rup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
int64_t hclamp(int64_t avail, int64_t cap) { return avail <= 0 ? 0 : (avail < cap ? avail : cap); }
int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// PCI location of a HIP device / an HSA agent: (domain << 32) | bdf
uint64_t hip_location(int device) {
  int bus = 0, dev = 0, dom = 0;
  (void)hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device);
  (void)hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device);
  (void)hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device);
  return (static_cast<uint64_t>(dom) << 32) | static_cast<uint64_t>((bus << 8) | (dev << 3));
}

struct AgentSearch {
  uint64_t want = 0;
  hsa_agent_t found{0};
  hsa_agent_t cpu{0};
};

hsa_status_t agent_cb(hsa_agent_t a, void* data) {
  auto* s = static_cast<AgentSearch*>(data);
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && s->cpu.handle == 0) s->cpu = a;
  if (t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, dom = 0;
  hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
  hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
  const uint64_t loc = (static_cast<uint64_t>(dom) << 32) | (bdf & ~0x7u);
  if (loc == s->want) s->found = a;
  return HSA_STATUS_SUCCESS;
}

}  // namespace

// ---------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------
__global__ void sdma_release_kernel(int64_t* sig) {
  if (threadIdx.x == 0) __hip_atomic_store(sig, int64_t{0}, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One wave: lane k < nflags (k != skip) waits for flags[k] >= epoch, bounded by the deadline.
__global__ __launch_bounds__(64) void sdma_wait_kernel(const uint32_t* flags, int nflags, int skip, uint32_t epoch,
                                                       uint64_t timeout, uint32_t* err) {
  const int k = static_cast<int>(threadIdx.x);
  const uint64_t deadline = wall_ticks() + timeout;
  const uint32_t* f = (k < nflags && k != skip) ? flags + k : nullptr;
  bool ok = f == nullptr || reached(ld_flag(f), epoch);
  while (!__all(ok)) {
    __builtin_amdgcn_s_sleep(2);
    if (!ok) ok = reached(ld_flag(f), epoch);
    if (wall_ticks() > deadline) break;
  }
  if (!__all(ok) && k == 0) __hip_atomic_fetch_or(err, ERR_TIMEOUT_SCATTER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Own block = scale x (own input + the P-1 SD slots), fixed order s = 0..P-1, fp32; written
// through (the engines read it from memory for phase 2). Workgroup b takes piece b.
template <class E>
__global__ __launch_bounds__(kCommThreads) void sdma_reduce_kernel(const char* in_own, const char* sd, int64_t slot,
                                                                   int P, int r, char* out_own, int64_t len,
                                                                   int64_t piece, float scale) {
  constexpr int es = 16 / E::ELEMS;
  // the engines wrote SD: drop any stale line of an earlier call from this CU's caches
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * piece;
  const int64_t l = clamp_len(len - b0, piece);
  if (l <= 0) return;
  const RedSrc src{in_own + b0 * es, sd + b0 * es, slot, r};
  reduce_to<E, 0>(P, src, 1, 0, [&](int) -> char* { return out_own + b0 * es; }, l, scale, true);
}

// out[block s] = RD slot s for every s != r (blockIdx.y = s). Plain-memory consumers follow
// on this stream: the stores go through to memory.
template <class E>
__global__ __launch_bounds__(kCommThreads) void sdma_gather_kernel(char* out, const char* rd, int64_t slot, int r,
                                                                   int64_t n, int64_t block, int64_t piece) {
  constexpr int es = 16 / E::ELEMS;
  const int s = static_cast<int>(blockIdx.y);
  if (s == r) return;
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  const int64_t blen = clamp_len(n - static_cast<int64_t>(s) * block, block);
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * piece;
  const int64_t l = clamp_len(blen - b0, piece);
  if (l <= 0) return;
  copy_from_slab<E>(out + (static_cast<int64_t>(s) * block + b0) * es, rd + s * slot + b0 * es, l);
}

// ---------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------
uint64_t pci_location(int device) { return hip_location(device); }

std::string sdma_diagnose(int device) {
  std::string out;
  hip_check(hipSetDevice(device), "hipSetDevice");
  hsa_status_t st = hsa_init();
  out += "hsa_init=" + std::to_string(static_cast<int>(st));
  const uint64_t want = hip_location(device);
  out += " want=" + std::to_string(want);
  struct Ctx {
    std::string* out;
  } ctx{&out};
  hsa_iterate_agents(
      [](hsa_agent_t a, void* d) -> hsa_status_t {
        auto* c = static_cast<Ctx*>(d);
        hsa_device_type_t t;
        hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
        uint32_t bdf = 0, dom = 0, mask = 0;
        hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
        hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
        hsa_status_t s = HSA_STATUS_SUCCESS;
        uint32_t m2 = 0;
        if (t == HSA_DEVICE_TYPE_GPU) s = hsa_amd_memory_copy_engine_status(a, a, &mask);
        *c->out += " | gpu<-gpu status=" + std::to_string(static_cast<int>(s)) + " mask=" + std::to_string(mask);
        if (t == HSA_DEVICE_TYPE_GPU) {
          hsa_agent_t cpu{0};
          hsa_iterate_agents(
              [](hsa_agent_t x, void* d) -> hsa_status_t {
                hsa_device_type_t tt;
                hsa_agent_get_info(x, HSA_AGENT_INFO_DEVICE, &tt);
                if (tt == HSA_DEVICE_TYPE_CPU && static_cast<hsa_agent_t*>(d)->handle == 0) *static_cast<hsa_agent_t*>(d) = x;
                return HSA_STATUS_SUCCESS;
              },
              &cpu);
          s = hsa_amd_memory_copy_engine_status(a, cpu, &m2);
          *c->out += " gpu<-cpu status=" + std::to_string(static_cast<int>(s)) + " mask=" + std::to_string(m2);
          s = hsa_amd_memory_copy_engine_status(cpu, a, &m2);
          *c->out += " cpu<-gpu status=" + std::to_string(static_cast<int>(s)) + " mask=" + std::to_string(m2);
        }
        *c->out += " | agent type=" + std::to_string(static_cast<int>(t)) + " bdf=" + std::to_string(bdf) +
                   " dom=" + std::to_string(dom) + " status=" + std::to_string(static_cast<int>(s)) +
                   " mask=" + std::to_string(mask);
        return HSA_STATUS_SUCCESS;
      },
      &ctx);
  if (st == HSA_STATUS_SUCCESS) hsa_shut_down();
  return out;
}

struct SdmaComm::Impl {
  hsa_agent_t own{0}, cpu{0};
  std::vector<hsa_agent_t> peer_agent;
  std::vector<std::vector<hsa_amd_sdma_engine_id_t>> peer_engines;  // engines towards peer k
  struct Slot {
    hsa_signal_t start{0}, mid{0}, sc{0}, scf{0}, gd{0}, gdf{0};
    int64_t* start_p = nullptr;
    int64_t* mid_p = nullptr;
    bool used = false;
  };
  Slot slots[kSlots];
  uint32_t* words = nullptr;  // pinned epoch words, one per slot (the flag copies' source)
  hipEvent_t sysrel = nullptr;
  bool hsa_up = false;
};

SdmaComm::SdmaComm(int rank, int world, int device, int64_t slot_bytes, int grid, int engines_per_peer,
                   double timeout_s)
    : rank_(rank), world_(world), device_(device), slot_bytes_(rup(std::max<int64_t>(slot_bytes, 4096), 4096)),
      grid_(std::max(1, grid)), epp_(std::max(0, engines_per_peer)), timeout_s_(timeout_s),
      impl_(std::make_unique<Impl>()) {
  if (world < 1 || world > 32 || rank < 0 || rank >= world) throw std::invalid_argument("SdmaComm: bad rank / world");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hsa_check(hsa_init(), "hsa_init");
  impl_->hsa_up = true;
  AgentSearch s;
  s.want = hip_location(device_);
  hsa_check(hsa_iterate_agents(agent_cb, &s), "hsa_iterate_agents");
  if (s.found.handle == 0) throw std::runtime_error("SdmaComm: no HSA agent at the HIP device's PCI location");
  impl_->own = s.found;
  impl_->cpu = s.cpu;
  // The device's SDMA engines. The ROCm 7.0 runtime torch ships answers the same-agent query
  // with HSA_STATUS_ERROR_INVALID_AGENT (7.2 answers it); the host <-> device directions name
  // the same engines there.
  uint32_t mask = 0, m2 = 0;
  if (hsa_amd_memory_copy_engine_status(impl_->own, impl_->own, &mask) != HSA_STATUS_SUCCESS) {
    mask = 0;
    if (impl_->cpu.handle != 0) {
      if (hsa_amd_memory_copy_engine_status(impl_->own, impl_->cpu, &m2) == HSA_STATUS_SUCCESS) mask |= m2;
      if (hsa_amd_memory_copy_engine_status(impl_->cpu, impl_->own, &m2) == HSA_STATUS_SUCCESS) mask |= m2;
    }
  }
  for (int b = 0; b < 32; ++b)
    if (mask & (1u << b)) local_engines_.push_back(1u << b);
  if (local_engines_.empty()) throw std::runtime_error("SdmaComm: the device reports no SDMA engine");

  slab_bytes_ = XgmiComm::ipc_safe_bytes(kFlagBytes + 4 * static_cast<int64_t>(world_) * slot_bytes_);
  hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&slab_), slab_bytes_, hipDeviceMallocFinegrained),
            "hipExtMallocWithFlags(sdma slab)");
  hip_check(hipMemset(slab_, 0, kFlagBytes), "hipMemset(sdma flags)");
  hip_check(hipMalloc(reinterpret_cast<void**>(&err_), 64), "hipMalloc(err)");
  hip_check(hipMemset(err_, 0, 64), "hipMemset(err)");
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&impl_->words), kSlots * 64, hipHostMallocCoherent),
            "hipHostMalloc(epoch words)");
  std::memset(impl_->words, 0, kSlots * 64);
  hip_check(hipEventCreateWithFlags(&impl_->sysrel, hipEventDisableTiming | hipEventReleaseToSystem),
            "hipEventCreate(release to system)");
  for (auto& sl : impl_->slots) {
    hsa_check(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_IPC, &sl.start), "signal(start)");
    hsa_check(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_IPC, &sl.mid), "signal(mid)");
    for (hsa_signal_t* x : {&sl.sc, &sl.scf, &sl.gd, &sl.gdf}) hsa_check(hsa_signal_create(0, 0, nullptr, x), "signal");
    volatile hsa_signal_value_t* p = nullptr;
    hsa_check(hsa_amd_signal_value_pointer(sl.start, &p), "signal_value_pointer(start)");
    sl.start_p = const_cast<int64_t*>(reinterpret_cast<volatile int64_t*>(p));
    hsa_check(hsa_amd_signal_value_pointer(sl.mid, &p), "signal_value_pointer(mid)");
    sl.mid_p = const_cast<int64_t*>(reinterpret_cast<volatile int64_t*>(p));
  }
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  peers_.assign(world_, nullptr);
  opened_.assign(world_, false);
  peers_[rank_] = slab_;
}

SdmaComm::~SdmaComm() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  if (impl_) {
    // no copy of ours may still target a peer slab we are about to unmap
    for (auto& sl : impl_->slots)
      for (hsa_signal_t x : {sl.sc, sl.scf, sl.gd, sl.gdf})
        if (x.handle) (void)hsa_signal_wait_scacquire(x, HSA_SIGNAL_CONDITION_EQ, 0, 2000000000ull, HSA_WAIT_STATE_BLOCKED);
    for (auto& sl : impl_->slots)
      for (hsa_signal_t x : {sl.start, sl.mid, sl.sc, sl.scf, sl.gd, sl.gdf})
        if (x.handle) hsa_signal_destroy(x);
    if (impl_->sysrel) (void)hipEventDestroy(impl_->sysrel);
    if (impl_->words) (void)hipHostFree(impl_->words);
  }
  for (int k = 0; k < world_; ++k)
    if (opened_[k] && peers_[k]) (void)hipIpcCloseMemHandle(peers_[k]);
  if (err_) (void)hipFree(err_);
  if (slab_) (void)hipFree(slab_);
  if (impl_ && impl_->hsa_up) hsa_shut_down();
}

std::string SdmaComm::handle() const {
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, slab_), "hipIpcGetMemHandle(sdma slab)");
  const uint64_t loc = hip_location(device_);
  std::string out(reinterpret_cast<const char*>(&h), sizeof(h));
  out.append(reinterpret_cast<const char*>(&loc), sizeof(loc));
  return out;
}

static std::vector<hsa_amd_sdma_engine_id_t> pick_engines(hsa_agent_t dst, hsa_agent_t src, int k, int epp,
                                                          const std::vector<uint32_t>& allowed) {
  uint32_t mask = 0;
  if (hsa_amd_memory_copy_engine_status(dst, src, &mask) != HSA_STATUS_SUCCESS) mask = 0;
  std::vector<uint32_t> avail;
  for (uint32_t e : allowed)
    if (mask & e) avail.push_back(e);
  if (avail.empty()) avail = allowed;  // peer direction unknown to the query: the local engines
  std::vector<hsa_amd_sdma_engine_id_t> out;
  for (int p = 0; p < epp; ++p)
    out.push_back(static_cast<hsa_amd_sdma_engine_id_t>(avail[(static_cast<size_t>(k) * epp + p) % avail.size()]));
  return out;
}

void SdmaComm::connect(const std::vector<std::string>& handles) {
  if (static_cast<int>(handles.size()) != world_) throw std::invalid_argument("SdmaComm.connect: one handle per rank");
  impl_->peer_agent.assign(world_, impl_->own);
  impl_->peer_engines.assign(world_, {});
  if (epp_ == 0)  // auto: the device's engines spread over the peers
    epp_ = std::max(1, static_cast<int>(local_engines_.size()) / std::max(1, world_ - 1));
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (int k = 0; k < world_; ++k) {
    if (k == rank_) continue;
    const std::string& h = handles[k];
    if (h.size() != sizeof(hipIpcMemHandle_t) + 8) throw std::invalid_argument("SdmaComm.connect: bad handle");
    hipIpcMemHandle_t ih;
    std::memcpy(&ih, h.data(), sizeof(ih));
    uint64_t loc = 0;
    std::memcpy(&loc, h.data() + sizeof(ih), 8);
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, ih, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(sdma slab)");
    peers_[k] = static_cast<char*>(p);
    opened_[k] = true;
    AgentSearch s;
    s.want = loc;
    hsa_check(hsa_iterate_agents(agent_cb, &s), "hsa_iterate_agents");
    if (s.found.handle != 0) impl_->peer_agent[k] = s.found;
    impl_->peer_engines[k] = pick_engines(impl_->peer_agent[k], impl_->own, k, epp_, local_engines_);
  }
  connected_ = true;
}

void SdmaComm::connect_local(const std::vector<SdmaComm*>& comms) {
  if (static_cast<int>(comms.size()) != world_) throw std::invalid_argument("SdmaComm.connect_local: one comm per rank");
  // Ranks of one process share its SDMA queues (one per engine): a rank's phase-2 copies
  // wait in an engine queue for its own reduce, which needs the peers' phase-1 copies - so
  // each local rank gets engines of its own (no copy of a peer ever queues behind them).
  const int nloc = world_;
  std::vector<uint32_t> mine;
  for (size_t i = 0; i < local_engines_.size(); ++i)
    if (static_cast<int>(i % nloc) == rank_) mine.push_back(local_engines_[i]);
  if (mine.empty()) throw std::runtime_error("SdmaComm.connect_local: fewer SDMA engines than local ranks");
  local_engines_ = mine;
  if (epp_ == 0) epp_ = std::max(1, static_cast<int>(local_engines_.size()) / std::max(1, world_ - 1));
  impl_->peer_agent.assign(world_, impl_->own);
  impl_->peer_engines.assign(world_, {});
  for (int k = 0; k < world_; ++k) {
    if (comms[k]->slot_bytes_ != slot_bytes_ || comms[k]->device_ != device_)
      throw std::invalid_argument("SdmaComm.connect_local: slab geometry / device differs");
    peers_[k] = comms[k]->slab_;
    if (k != rank_) impl_->peer_engines[k] = pick_engines(impl_->own, impl_->own, k, epp_, local_engines_);
  }
  connected_ = true;
}

std::string SdmaComm::debug_state() const {
  std::string out = "epoch=" + std::to_string(epoch_) + " engines=";
  for (uint32_t e : local_engines_) out += std::to_string(e) + ",";
  for (int k = 0; k < world_; ++k) {
    out += " peer" + std::to_string(k) + "_engines=";
    if (k < static_cast<int>(impl_->peer_engines.size()))
      for (auto e : impl_->peer_engines[k]) out += std::to_string(static_cast<uint32_t>(e)) + ",";
  }
  for (int i = 0; i < kSlots; ++i) {
    const Impl::Slot& sl = impl_->slots[i];
    if (!sl.used) continue;
    out += " | slot" + std::to_string(i) + " start=" + std::to_string(hsa_signal_load_relaxed(sl.start)) +
           " mid=" + std::to_string(hsa_signal_load_relaxed(sl.mid)) +
           " sc=" + std::to_string(hsa_signal_load_relaxed(sl.sc)) +
           " scf=" + std::to_string(hsa_signal_load_relaxed(sl.scf)) +
           " gd=" + std::to_string(hsa_signal_load_relaxed(sl.gd)) +
           " gdf=" + std::to_string(hsa_signal_load_relaxed(sl.gdf));
  }
  std::vector<uint32_t> f(128, 0);
  (void)hipMemcpy(f.data(), slab_, f.size() * 4, hipMemcpyDeviceToHost);
  out += " | FS=";
  for (int k = 0; k < world_; ++k) out += std::to_string(f[k]) + ",";
  out += " FR=";
  for (int k = 0; k < world_; ++k) out += std::to_string(f[kFrWord + k]) + ",";
  return out;
}

uint32_t SdmaComm::error() const {
  uint32_t e = 0;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipMemcpy(&e, err_, 4, hipMemcpyDeviceToHost), "hipMemcpy(err)");
  return e;
}

void SdmaComm::clear_error() {
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipMemset(err_, 0, 4), "hipMemset(err)");
}

void SdmaComm::allreduce(const void* in, void* out, int64_t n, DType dt, hipStream_t stream, float scale) {
  allreduce_local({this}, {in}, {out}, n, dt, stream, scale);
}

// The ranks of one process on one stream: for each segment every rank's copies are queued
// first, then the stream releases every rank's phase 1, then runs every rank's wait + reduce
// + phase-2 release, then every rank's wait + gather. Each wait only needs releases queued
// before it on the same stream, so one stream carries all local ranks (a wait holding a
// hardware queue never blocks a peer's release behind it).
void SdmaComm::allreduce_local(const std::vector<SdmaComm*>& comms, const std::vector<const void*>& ins,
                               const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream, float scale) {
  if (comms.empty() || ins.size() != comms.size() || outs.size() != comms.size())
    throw std::invalid_argument("SdmaComm: one input and one output per local rank");
  SdmaComm& c0 = *comms[0];
  for (size_t y = 0; y < comms.size(); ++y) {
    const SdmaComm& c = *comms[y];
    if (!c.connected_) throw std::runtime_error("SdmaComm: connect() first");
    if (c.device_ != c0.device_ || c.world_ != c0.world_ || c.slot_bytes_ != c0.slot_bytes_)
      throw std::invalid_argument("SdmaComm: local ranks must share device, world and slot size");
    if ((reinterpret_cast<uintptr_t>(ins[y]) | reinterpret_cast<uintptr_t>(outs[y])) & 15)
      throw std::invalid_argument("SdmaComm: buffers must be 16-byte aligned");
  }
  if (n <= 0) return;
  hip_check(hipSetDevice(c0.device_), "hipSetDevice");
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  const int64_t seg = c0.world_ * (c0.slot_bytes_ / es);
  std::vector<Plan> plans(comms.size());
  for (int64_t off = 0; off < n; off += seg) {
    const int64_t len = std::min(seg, n - off);
    for (size_t y = 0; y < comms.size(); ++y)
      plans[y] = comms[y]->plan(static_cast<const char*>(ins[y]) + off * es, static_cast<char*>(outs[y]) + off * es,
                                len, dt);
    hip_check(hipEventRecord(c0.impl_->sysrel, stream), "hipEventRecord(release to system)");
    for (size_t y = 0; y < comms.size(); ++y)
      hipLaunchKernelGGL(sdma_release_kernel, dim3(1), dim3(64), 0, stream,
                         comms[y]->impl_->slots[plans[y].slot].start_p);
    for (size_t y = 0; y < comms.size(); ++y) comms[y]->enqueue_reduce(plans[y], stream, scale);
    for (size_t y = 0; y < comms.size(); ++y) comms[y]->enqueue_gather(plans[y], stream);
    hip_check(hipGetLastError(), "sdma kernels");
  }
}

SdmaComm::Plan SdmaComm::plan(const char* in, char* out, int64_t n, DType dt) {
  Impl& m = *impl_;
  const int W = world_, r = rank_;
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  const int64_t elems = 16 / es;
  Plan pl;
  pl.in = in;
  pl.out = out;
  pl.n = n;
  pl.dt = dt;
  const uint64_t e64 = ++epoch_;
  pl.epoch = static_cast<uint32_t>(e64);
  pl.par = static_cast<int>(e64 & 1u);
  pl.slot = static_cast<int>(e64 % kSlots);
  Impl::Slot& sl = m.slots[pl.slot];
  // the slot's previous call: every copy it submitted has completed (the host is at most
  // kSlots calls ahead of the engines; a peer that stopped turns into an error here)
  if (sl.used) {
    for (hsa_signal_t x : {sl.sc, sl.scf, sl.gd, sl.gdf}) {
      if (hsa_signal_load_scacquire(x) == 0) continue;
      ++st_.host_waits;
      const uint64_t ns = static_cast<uint64_t>(timeout_s_ * 1e9);
      if (hsa_signal_wait_scacquire(x, HSA_SIGNAL_CONDITION_EQ, 0, ns, HSA_WAIT_STATE_BLOCKED) != 0)
        throw std::runtime_error("SdmaComm: copies of an earlier call did not complete (peer gone?)");
    }
  }
  sl.used = true;
  pl.block = rup(cdiv(n, W), elems);
  const int64_t block = pl.block;
  auto blen = [&](int j) { return hclamp(n - static_cast<int64_t>(j) * block, block); };
  if (block * es > slot_bytes_) throw std::logic_error("SdmaComm: segment exceeds the slot");
  // split of one block over epp engines, 4 KiB aligned pieces
  auto parts = [&](int64_t bytes, int p, int64_t* off, int64_t* len) {
    const int64_t piece = rup(cdiv(bytes, epp_), 4096);
    *off = std::min<int64_t>(bytes, p * piece);
    *len = std::min<int64_t>(bytes - *off, piece);
  };
  int n1 = 0, n2 = 0;
  for (int j = 0; j < W; ++j) {
    if (j == r) continue;
    for (int p = 0; p < epp_; ++p) {
      int64_t o, l;
      parts(blen(j) * es, p, &o, &l);
      n1 += l > 0;
      parts(blen(r) * es, p, &o, &l);
      n2 += l > 0;
    }
  }
  uint32_t* word = m.words + static_cast<int64_t>(pl.slot) * 16;
  *word = pl.epoch;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  hsa_signal_store_relaxed(sl.start, 1);
  hsa_signal_store_relaxed(sl.mid, 1);
  hsa_signal_store_relaxed(sl.sc, n1);
  hsa_signal_store_relaxed(sl.scf, W - 1);
  hsa_signal_store_relaxed(sl.gd, n2);
  hsa_signal_store_relaxed(sl.gdf, W > 1 ? W : 0);  // W - 1 peer flags + the own "phase 2 sent" flag
  const int64_t off_SD = kFlagBytes, off_RD = kFlagBytes + 2 * static_cast<int64_t>(W) * slot_bytes_;
  auto copy = [&](void* dst, hsa_agent_t da, const void* src, hsa_agent_t sa, int64_t bytes, int ndep,
                  const hsa_signal_t* deps, hsa_signal_t done, hsa_amd_sdma_engine_id_t eng) {
    hsa_check(hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, static_cast<size_t>(bytes), ndep, deps, done, eng,
                                                  true),
              "hsa_amd_memory_async_copy_on_engine");
    ++st_.copies;
    st_.bytes += static_cast<uint64_t>(bytes);
  };
  const int par = pl.par;
  // phase 1: block j -> rank j's SD[par][r], then its FS[r] flag
  for (int j = 0; j < W; ++j) {
    if (j == r) continue;
    for (int p = 0; p < epp_; ++p) {
      int64_t o, l;
      parts(blen(j) * es, p, &o, &l);
      if (l > 0)
        copy(peers_[j] + off_SD + (static_cast<int64_t>(par) * W + r) * slot_bytes_ + o, m.peer_agent[j],
             in + static_cast<int64_t>(j) * block * es + o, m.own, l, 1, &sl.start, sl.sc, m.peer_engines[j][p]);
    }
  }
  const hsa_signal_t dep1[2] = {sl.start, sl.sc};
  for (int j = 0; j < W; ++j)
    if (j != r) copy(peers_[j] + r * 4, m.peer_agent[j], word, m.cpu, 4, 2, dep1, sl.scf, m.peer_engines[j][0]);
  // phase 2: the reduced own block -> every peer's RD[par][r], then its FR[r] flag
  for (int k = 0; k < W; ++k) {
    if (k == r) continue;
    for (int p = 0; p < epp_; ++p) {
      int64_t o, l;
      parts(blen(r) * es, p, &o, &l);
      if (l > 0)
        copy(peers_[k] + off_RD + (static_cast<int64_t>(par) * W + r) * slot_bytes_ + o, m.peer_agent[k],
             out + static_cast<int64_t>(r) * block * es + o, m.own, l, 1, &sl.mid, sl.gd, m.peer_engines[k][p]);
    }
  }
  const hsa_signal_t dep2[2] = {sl.mid, sl.gd};
  for (int k = 0; k < W; ++k)
    if (k != r)
      copy(peers_[k] + (kFrWord + r) * 4, m.peer_agent[k], word, m.cpu, 4, 2, dep2, sl.gdf, m.peer_engines[k][0]);
  // and the own FR[r] word once every phase-2 copy has completed: the engines read the own
  // block of `out` for them, so the call may not count as done (and the caller may not write
  // `out`) before they are - enqueue_gather waits for this word with the peers' 
  if (W > 1) {
    const int k0 = (r + 1) % W;
    copy(slab_ + (kFrWord + r) * 4, m.own, word, m.cpu, 4, 2, dep2, sl.gdf, m.peer_engines[k0][0]);
  }
  ++st_.calls;
  return pl;
}

// wait for every peer's phase-1 flag, reduce the own block, release phase 2
void SdmaComm::enqueue_reduce(const Plan& pl, hipStream_t stream, float scale) {
  const int W = world_, r = rank_;
  const int64_t es = static_cast<int64_t>(dtype_size(pl.dt));
  const int64_t elems = 16 / es;
  const uint64_t ticks = static_cast<uint64_t>(timeout_s_ * 1e8);
  hipLaunchKernelGGL(sdma_wait_kernel, dim3(1), dim3(64), 0, stream, reinterpret_cast<const uint32_t*>(slab_), W, r,
                     pl.epoch, ticks, err_);
  const int64_t rl = hclamp(pl.n - static_cast<int64_t>(r) * pl.block, pl.block);
  const int64_t piece = std::max<int64_t>(elems, rup(cdiv(rl, grid_), elems));
  const int g1 = static_cast<int>(std::max<int64_t>(1, cdiv(rl, piece)));
  const char* sd = slab_ + kFlagBytes + static_cast<int64_t>(pl.par) * W * slot_bytes_;
  if (rl > 0)
    dispatch_dtype(static_cast<int>(pl.dt), [&](auto tag) {
      using E = decltype(tag);
      hipLaunchKernelGGL(sdma_reduce_kernel<E>, dim3(g1), dim3(kCommThreads), 0, stream,
                         pl.in + static_cast<int64_t>(r) * pl.block * es, sd, slot_bytes_, W, r,
                         pl.out + static_cast<int64_t>(r) * pl.block * es, rl, piece, scale);
    });
  hipLaunchKernelGGL(sdma_release_kernel, dim3(1), dim3(64), 0, stream, impl_->slots[pl.slot].mid_p);
}

// wait for every peer's reduced block, copy them into the output
void SdmaComm::enqueue_gather(const Plan& pl, hipStream_t stream) {
  const int W = world_, r = rank_;
  const int64_t es = static_cast<int64_t>(dtype_size(pl.dt));
  const int64_t elems = 16 / es;
  const uint64_t ticks = static_cast<uint64_t>(timeout_s_ * 1e8);
  // every peer's reduced block AND the own phase-2 copies (FR[r], written behind them)
  hipLaunchKernelGGL(sdma_wait_kernel, dim3(1), dim3(64), 0, stream,
                     reinterpret_cast<const uint32_t*>(slab_) + kFrWord, W, W > 1 ? -1 : r, pl.epoch, ticks, err_);
  if (W < 2) return;
  const int64_t gpiece = std::max<int64_t>(elems, rup(cdiv(pl.block, std::max(1, grid_ / (W - 1))), elems));
  const int g2 = static_cast<int>(std::max<int64_t>(1, cdiv(pl.block, gpiece)));
  const char* rd = slab_ + kFlagBytes + 2 * static_cast<int64_t>(W) * slot_bytes_ +
                   static_cast<int64_t>(pl.par) * W * slot_bytes_;
  dispatch_dtype(static_cast<int>(pl.dt), [&](auto tag) {
    using E = decltype(tag);
    hipLaunchKernelGGL(sdma_gather_kernel<E>, dim3(g2, W), dim3(kCommThreads), 0, stream, pl.out, rd, slot_bytes_, r,
                       pl.n, pl.block, gpiece);
  });
}

}  // namespace mxar
