// SdmaComm (sdma_comm.h): bucket allreduce with the cross-rank traffic on the SDMA copy
// engines. Host side: HSA agents / engines, the per-call signal ring and the SDMA
// submissions. Device side: the signal release, the bounded flag wait, and the small-grid
// reduce and gather kernels.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <cstring>
#include <stdexcept>
#include <string>

#include "sdma_comm.h"

#include <chrono>
#include "xgmi_device.h"

namespace mxar {

namespace {

constexpr int kSlots = 16;              // calls in flight at most (signal / epoch-word ring)
constexpr int64_t kFlagBytes = 64 * 1024;
// flag words: FS[s][k] at s * kSdmaMaxPieces + k, FR[s][k] at kFrWord + s * kSdmaMaxPieces + k
constexpr int kFrWord = 32 * kSdmaMaxPieces;
constexpr int64_t kPieceBytes = int64_t{64} << 20;  // auto pieces: one per 64 MiB of the block (2..8)

void hsa_check(hsa_status_t s, const char* what) {
  if (s != HSA_STATUS_SUCCESS) {
    const char* m = nullptr;
    hsa_status_string(s, &m);
    throw std::runtime_error(std::string("HSA error in ") + what + ": " + (m ? m : "?"));
  }
}

__host__ __device__ inline int64_t rup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
int64_t hclamp(int64_t avail, int64_t cap) { return avail <= 0 ? 0 : (avail < cap ? avail : cap); }
__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

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

// The engines towards `dst` from `src`, first answer per (dst, src) kept for the process.
uint32_t cached_engine_status(hsa_agent_t dst, hsa_agent_t src) {
  static std::mutex mu;
  static std::map<std::pair<uint64_t, uint64_t>, uint32_t> seen;
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_pair(dst.handle, src.handle);
  auto it = seen.find(key);
  if (it != seen.end()) return it->second;
  uint32_t m = 0;
  if (hsa_amd_memory_copy_engine_status(dst, src, &m) != HSA_STATUS_SUCCESS) m = 0;
  seen[key] = m;
  return m;
}

uint32_t engine_mask(int device, hsa_agent_t own, hsa_agent_t cpu) {
  (void)device;
  uint32_t mask = cached_engine_status(own, own);
  if (mask == 0 && cpu.handle != 0) mask = cached_engine_status(own, cpu) | cached_engine_status(cpu, own);
  return mask;
}

}  // namespace

// Engine copies of `bytes` from src to dst on this device, split over `nengines` engines
// (from index `engine` of the device's mask) running at once, `iters` times back to back;
// ms per copy by the host clock. The probe behind profiles/round6 section 3 (which
// buffers, and how many engines at once, the engines are slow on).
double sdma_copy_probe(int device, uint64_t dst, uint64_t src, int64_t bytes, int engine, int iters, int nengines) {
  hip_check(hipSetDevice(device), "hipSetDevice");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  hsa_check(hsa_init(), "hsa_init");
  AgentSearch s;
  s.want = hip_location(device);
  hsa_check(hsa_iterate_agents(agent_cb, &s), "hsa_iterate_agents");
  if (s.found.handle == 0) throw std::runtime_error("sdma_copy_probe: no HSA agent for the device");
  const uint32_t mask = engine_mask(device, s.found, s.cpu);
  std::vector<uint32_t> engines;
  for (int b = 0; b < 32; ++b)
    if (mask & (1u << b)) engines.push_back(1u << b);
  if (engines.empty()) throw std::runtime_error("sdma_copy_probe: no SDMA engine");
  const int ne = std::max(1, nengines);
  const int64_t part = rup(cdiv(bytes, ne), 4096);
  hsa_signal_t done;
  hsa_check(hsa_signal_create(1, 0, nullptr, &done), "signal");
  auto one = [&] {
    int parts = 0;
    for (int e = 0; e < ne; ++e) parts += std::min<int64_t>(bytes, e * part) < bytes;
    hsa_signal_store_relaxed(done, parts);
    for (int e = 0; e < ne; ++e) {
      const int64_t off = std::min<int64_t>(bytes, e * part), len = std::min<int64_t>(bytes - off, part);
      if (len <= 0) continue;
      const auto eng = static_cast<hsa_amd_sdma_engine_id_t>(engines[static_cast<size_t>(engine + e) % engines.size()]);
      hsa_check(hsa_amd_memory_async_copy_on_engine(reinterpret_cast<void*>(dst + off), s.found,
                                                    reinterpret_cast<const void*>(src + off), s.found,
                                                    static_cast<size_t>(len), 0, nullptr, done, eng, true),
                "hsa_amd_memory_async_copy_on_engine");
    }
    if (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_EQ, 0, 10'000'000'000ull, HSA_WAIT_STATE_ACTIVE) != 0)
      throw std::runtime_error("sdma_copy_probe: copy did not complete");
  };
  one();  // warm
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) one();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / iters;
  hsa_signal_destroy(done);
  hsa_shut_down();
  return ms;
}

// ---------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------
__global__ void sdma_release_kernel(int64_t* sig) {
  if (threadIdx.x == 0) __hip_atomic_store(sig, int64_t{0}, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One launch of the pipelined reduce / gather for the local ranks of a call (blockIdx.y).
struct SdmaRankArgs {
  const char* in;         // the rank's input (whole tensor segment)
  char* out;              // its output
  const char* sd;         // its SD slots of this call's parity (slot s at s * slot)
  const char* rd;         // its RD slots of this call's parity
  const uint32_t* flags;  // its flag words (FS at 0, FR at kFrWord)
  int64_t* mid[kSdmaMaxPieces];  // phase-2 release signal of each piece (value pointer)
  uint32_t* cnt;          // per-piece workgroup tickets (device, zero between launches)
  uint32_t* err;
  uint32_t epoch;
  int r;
};
struct SdmaLaunch {
  SdmaRankArgs y[kSdmaMaxLocal];
  int64_t n, block, pe, slot;  // elements (slot: bytes)
  uint64_t timeout;            // 100 MHz ticks
  int W, K;
  float scale;
};

__device__ __forceinline__ int64_t sdma_blen(const SdmaLaunch& L, int s) {
  return clamp_len(L.n - static_cast<int64_t>(s) * L.block, L.block);
}

// Own block = scale x (own input + the P-1 SD slots), fixed order s = 0..P-1, fp32, written
// through (the engines read it from memory for phase 2), piece by piece: piece k is reduced
// once every peer's FS[s][k] shows the epoch, and its last workgroup releases mid[k] - the
// signal the engines' phase-2 copies of piece k wait on. No workgroup waits for another.
template <class E>
__global__ __launch_bounds__(kCommThreads) void sdma_reduce_kernel(SdmaLaunch L) {
  constexpr int es = 16 / E::ELEMS;
  const SdmaRankArgs& a = L.y[blockIdx.y];
  const int G = static_cast<int>(gridDim.x);
  const uint64_t deadline = wall_ticks() + L.timeout;
  const int64_t rl = sdma_blen(L, a.r);
  const int64_t own0 = static_cast<int64_t>(a.r) * L.block;
  for (int k = 0; k < L.K; ++k) {
    const int64_t p0 = static_cast<int64_t>(k) * L.pe;
    const int64_t lk = clamp_len(rl - p0, L.pe);
    if (lk <= 0) break;  // uniform
    wait_flags([&](int s) -> const uint32_t* { return s == a.r ? nullptr : a.flags + s * kSdmaMaxPieces + k; }, L.W,
               a.epoch, deadline, a.err, ERR_TIMEOUT_SCATTER);
    const int64_t sub = rup(cdiv(lk, G), E::ELEMS);
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * sub;
    const int64_t l = clamp_len(lk - b0, sub);
    if (l > 0) {
      const RedSrc src{a.in + (own0 + p0 + b0) * es, a.sd + (p0 + b0) * es, L.slot, a.r};
      char* dst = a.out + (own0 + p0 + b0) * es;
      reduce_to<E, 0>(L.W, src, 1, 0, [&](int) -> char* { return dst; }, l, L.scale, true);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the engines read the piece
      const uint32_t t = __hip_atomic_fetch_add(&a.cnt[k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == static_cast<uint32_t>(G - 1)) {
        __hip_atomic_store(&a.cnt[k], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.mid[k], int64_t{0}, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// out[block s, piece k] = RD slot s piece k for every s != r, piece by piece as the FR[s][k]
// flags arrive (and the own FR[r][k]: the engines have finished READING the own block's
// piece k for phase 2, so the call is complete for the stream). Plain-memory consumers
// follow on this stream: the stores go through to memory.
template <class E>
__global__ __launch_bounds__(kCommThreads) void sdma_gather_kernel(SdmaLaunch L) {
  constexpr int es = 16 / E::ELEMS;
  const SdmaRankArgs& a = L.y[blockIdx.y];
  const int G = static_cast<int>(gridDim.x);
  const uint64_t deadline = wall_ticks() + L.timeout;
  for (int k = 0; k < L.K; ++k) {
    const int64_t p0 = static_cast<int64_t>(k) * L.pe;
    if (p0 >= L.block) break;  // uniform
    wait_flags([&](int s) -> const uint32_t* {
                 return sdma_blen(L, s) > p0 ? a.flags + kFrWord + s * kSdmaMaxPieces + k : nullptr;
               },
               L.W, a.epoch, deadline, a.err, ERR_TIMEOUT_REDUCE);
    const int64_t sub = rup(cdiv(L.pe, G), E::ELEMS);
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * sub;
    for (int s = 0; s < L.W; ++s) {
      if (s == a.r) continue;
      const int64_t l = clamp_len(clamp_len(sdma_blen(L, s) - p0, L.pe) - b0, sub);
      if (l > 0)
        copy_from_slab<E>(a.out + (static_cast<int64_t>(s) * L.block + p0 + b0) * es,
                          a.rd + s * L.slot + (p0 + b0) * es, l);
    }
  }
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
    hsa_signal_t start{0}, scf{0}, gdf{0};
    hsa_signal_t mid[kSdmaMaxPieces]{};
    int64_t* start_p = nullptr;
    int64_t* mid_p[kSdmaMaxPieces]{};
    // completion of a piece's data parts: phase 1 per peer ([j * K + k]), phase 2 over every
    // peer ([k]: the own FR flag needs them all, and a copy with one dependency is the form the
    // engines are known to take), armed to the part count - every part's completion
    // decrements it, the piece's flag copies wait for 0. Memory-only signals (the host never waits on them, so
    // no interrupt events - KFD has few), grown on demand.
    std::vector<hsa_signal_t> c1, c2;
    bool used = false;
  };
  static void grow(std::vector<hsa_signal_t>& v, size_t need) {
    while (v.size() < need) {
      hsa_signal_t x{0};
      hsa_check(hsa_amd_signal_create(0, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &x), "signal(piece)");
      v.push_back(x);
    }
  }
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
  // the same engines there. The first answer per (dst, src) agent pair is kept for the
  // process, so every communicator of it picks its engines from the same mask.
  uint32_t mask = engine_mask(device_, impl_->own, impl_->cpu);
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
  hip_check(hipMalloc(reinterpret_cast<void**>(&cnt_), kSdmaMaxPieces * 4), "hipMalloc(piece tickets)");
  hip_check(hipMemset(cnt_, 0, kSdmaMaxPieces * 4), "hipMemset(piece tickets)");
  for (auto& sl : impl_->slots) {
    volatile hsa_signal_value_t* p = nullptr;
    hsa_check(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_IPC, &sl.start), "signal(start)");
    hsa_check(hsa_amd_signal_value_pointer(sl.start, &p), "signal_value_pointer(start)");
    sl.start_p = const_cast<int64_t*>(reinterpret_cast<volatile int64_t*>(p));
    for (int k = 0; k < kSdmaMaxPieces; ++k) {
      hsa_check(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_IPC, &sl.mid[k]), "signal(mid)");
      hsa_check(hsa_amd_signal_value_pointer(sl.mid[k], &p), "signal_value_pointer(mid)");
      sl.mid_p[k] = const_cast<int64_t*>(reinterpret_cast<volatile int64_t*>(p));
    }
    for (hsa_signal_t* x : {&sl.scf, &sl.gdf}) hsa_check(hsa_signal_create(0, 0, nullptr, x), "signal");
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
    // (every data part precedes a flag copy counted in scf / gdf)
    for (auto& sl : impl_->slots)
      for (hsa_signal_t x : {sl.scf, sl.gdf})
        if (x.handle) (void)hsa_signal_wait_scacquire(x, HSA_SIGNAL_CONDITION_EQ, 0, 2000000000ull, HSA_WAIT_STATE_BLOCKED);
    for (auto& sl : impl_->slots) {
      for (hsa_signal_t x : {sl.start, sl.scf, sl.gdf})
        if (x.handle) hsa_signal_destroy(x);
      for (hsa_signal_t x : sl.mid)
        if (x.handle) hsa_signal_destroy(x);
      for (auto* v : {&sl.c1, &sl.c2})
        for (hsa_signal_t x : *v) hsa_signal_destroy(x);
    }
    if (impl_->sysrel) (void)hipEventDestroy(impl_->sysrel);
    if (impl_->words) (void)hipHostFree(impl_->words);
  }
  for (int k = 0; k < world_; ++k)
    if (opened_[k] && peers_[k]) (void)hipIpcCloseMemHandle(peers_[k]);
  if (err_) (void)hipFree(err_);
  if (cnt_) (void)hipFree(cnt_);
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
  const uint32_t mask = cached_engine_status(dst, src);
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
           " mid=";
    for (hsa_signal_t x : sl.mid) out += std::to_string(hsa_signal_load_relaxed(x)) + ",";
    out += " scf=" + std::to_string(hsa_signal_load_relaxed(sl.scf)) +
           " gdf=" + std::to_string(hsa_signal_load_relaxed(sl.gdf));
  }
  std::vector<uint32_t> f(2 * kFrWord, 0);
  (void)hipMemcpy(f.data(), slab_, f.size() * 4, hipMemcpyDeviceToHost);
  for (const char* what : {"FS", "FR"}) {
    const int base = what[1] == 'S' ? 0 : kFrWord;
    out += std::string(" | ") + what + "[rank][piece]=";
    for (int k = 0; k < world_; ++k) {
      for (int q = 0; q < kSdmaMaxPieces; ++q) out += std::to_string(f[base + k * kSdmaMaxPieces + q]) + ",";
      out += ";";
    }
  }
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
// first, then the stream releases every rank's phase 1, then ONE pipelined reduce launch for
// every local rank (blockIdx.y) and ONE pipelined gather launch. Each wait inside them only
// needs copies released before the launch, so one stream carries all local ranks.
void SdmaComm::allreduce_local(const std::vector<SdmaComm*>& comms, const std::vector<const void*>& ins,
                               const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream, float scale) {
  if (comms.empty() || ins.size() != comms.size() || outs.size() != comms.size())
    throw std::invalid_argument("SdmaComm: one input and one output per local rank");
  SdmaComm& c0 = *comms[0];
  for (size_t y = 0; y < comms.size(); ++y) {
    const SdmaComm& c = *comms[y];
    if (!c.connected_) throw std::runtime_error("SdmaComm: connect() first");
    if (c.device_ != c0.device_ || c.world_ != c0.world_ || c.slot_bytes_ != c0.slot_bytes_ ||
        c.pieces_ != c0.pieces_ || c.grid_ != c0.grid_)
      throw std::invalid_argument("SdmaComm: local ranks must share device, world, slot size, pieces and grid");
    if ((reinterpret_cast<uintptr_t>(ins[y]) | reinterpret_cast<uintptr_t>(outs[y])) & 15)
      throw std::invalid_argument("SdmaComm: buffers must be 16-byte aligned");
  }
  if (n <= 0) return;
  hip_check(hipSetDevice(c0.device_), "hipSetDevice");
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  const int64_t seg = c0.world_ * (c0.slot_bytes_ / es);
  const int W = c0.world_;
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
    for (size_t y0 = 0; y0 < comms.size(); y0 += kSdmaMaxLocal) {
      const size_t ny = std::min<size_t>(kSdmaMaxLocal, comms.size() - y0);
      SdmaLaunch L{};
      L.n = len;
      L.block = plans[y0].block;
      L.pe = plans[y0].pe;
      L.K = plans[y0].K;
      L.slot = c0.slot_bytes_;
      L.W = W;
      L.scale = scale;
      L.timeout = static_cast<uint64_t>(c0.timeout_s_ * 1e8);
      for (size_t i = 0; i < ny; ++i) {
        SdmaComm& c = *comms[y0 + i];
        const Plan& pl = plans[y0 + i];
        SdmaRankArgs& a = L.y[i];
        a.in = pl.in;
        a.out = pl.out;
        a.sd = c.slab_ + kFlagBytes + static_cast<int64_t>(pl.par) * W * c.slot_bytes_;
        a.rd = c.slab_ + kFlagBytes + (2 + static_cast<int64_t>(pl.par)) * W * c.slot_bytes_;
        a.flags = reinterpret_cast<const uint32_t*>(c.slab_);
        for (int k = 0; k < kSdmaMaxPieces; ++k) a.mid[k] = c.impl_->slots[pl.slot].mid_p[k];
        a.cnt = c.cnt_;
        a.err = c.err_;
        a.epoch = pl.epoch;
        a.r = c.rank_;
      }
      dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
        using E = decltype(tag);
        hipLaunchKernelGGL(sdma_reduce_kernel<E>, dim3(c0.grid_, ny), dim3(kCommThreads), 0, stream, L);
        if (W > 1)  // one rank: the reduce wrote the whole (scaled) output
          hipLaunchKernelGGL(sdma_gather_kernel<E>, dim3(c0.grid_, ny), dim3(kCommThreads), 0, stream, L);
      });
    }
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
    for (hsa_signal_t x : {sl.scf, sl.gdf}) {  // every part precedes a flag counted here
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
  if (block * es > slot_bytes_) throw std::logic_error("SdmaComm: segment exceeds the slot");
  auto blen = [&](int j) { return hclamp(n - static_cast<int64_t>(j) * block, block); };
  // pipeline pieces: 4 KiB aligned, the same on every rank (they derive it from n and W alone)
  const int want = pieces_ > 0 ? std::min(pieces_, kSdmaMaxPieces)
                               : static_cast<int>(std::clamp<int64_t>(cdiv(block * es, kPieceBytes), 2, kSdmaMaxPieces));
  pl.pe = rup(cdiv(block, want), std::max<int64_t>(elems, 4096 / es));
  pl.K = static_cast<int>(std::max<int64_t>(1, cdiv(block, pl.pe)));
  const int K = pl.K;
  auto kn = [&](int j) { return static_cast<int>(cdiv(blen(j), pl.pe)); };  // pieces holding data
  auto plen = [&](int j, int k) { return hclamp(blen(j) - static_cast<int64_t>(k) * pl.pe, pl.pe); };
  // part p of a piece of `bytes` (over the epp engines), 4 KiB aligned
  auto part = [&](int64_t bytes, int p, int64_t* off, int64_t* len) {
    const int64_t sz = rup(cdiv(bytes, epp_), 4096);
    *off = std::min<int64_t>(bytes, p * sz);
    *len = std::min<int64_t>(bytes - *off, sz);
  };
  auto nparts = [&](int j, int k) {
    int c = 0;
    for (int p = 0; p < epp_; ++p) {
      int64_t o, l;
      part(plen(j, k) * es, p, &o, &l);
      c += l > 0;
    }
    return c;
  };
  Impl::grow(sl.c1, static_cast<size_t>(W) * K);
  Impl::grow(sl.c2, static_cast<size_t>(K));
  for (int k = 0; k < K; ++k) {
    for (int j = 0; j < W; ++j) hsa_signal_store_relaxed(sl.c1[static_cast<size_t>(j) * K + k], j == r ? 0 : nparts(j, k));
    hsa_signal_store_relaxed(sl.c2[static_cast<size_t>(k)], (W - 1) * nparts(r, k));
  }
  int nflag1 = 0;
  for (int j = 0; j < W; ++j)
    if (j != r) nflag1 += kn(j);
  uint32_t* word = m.words + static_cast<int64_t>(pl.slot) * 16;
  *word = pl.epoch;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  hsa_signal_store_relaxed(sl.start, 1);
  for (int k = 0; k < kSdmaMaxPieces; ++k) hsa_signal_store_relaxed(sl.mid[k], 1);
  hsa_signal_store_relaxed(sl.scf, nflag1);
  hsa_signal_store_relaxed(sl.gdf, W > 1 ? W * kn(r) : 0);  // W - 1 peer flags + the own flag per piece
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
  // phase 1, piece by piece: piece k of block j -> rank j's SD[par][r], then its FS[r][k]
  for (int k = 0; k < K; ++k)
    for (int j = 0; j < W; ++j) {
      if (j == r || k >= kn(j)) continue;
      const hsa_signal_t done = sl.c1[static_cast<size_t>(j) * K + k];
      int last = 0;
      for (int p = 0; p < epp_; ++p) {
        int64_t o, l;
        part(plen(j, k) * es, p, &o, &l);
        if (l <= 0) continue;
        const int64_t at = static_cast<int64_t>(k) * pl.pe * es + o;
        copy(peers_[j] + off_SD + (static_cast<int64_t>(par) * W + r) * slot_bytes_ + at, m.peer_agent[j],
             in + static_cast<int64_t>(j) * block * es + at, m.own, l, 1, &sl.start, done, m.peer_engines[j][p]);
        last = p;
      }
      copy(peers_[j] + (r * kSdmaMaxPieces + k) * 4, m.peer_agent[j], word, m.cpu, 4, 1, &done, sl.scf,
           m.peer_engines[j][last]);
    }
  // phase 2, piece by piece: reduced piece k of the own block -> every peer's RD[par][r], then
  // its FR[r][k]; each part waits for mid[k] (released by the reduce kernel's last workgroup of
  // the piece)
  // (every part of the piece is queued before any of its flags: a flag waits in its engine's
  // queue for ALL the piece's parts, so none of them may be queued behind it)
  for (int k = 0; k < kn(r); ++k) {
    const hsa_signal_t done = sl.c2[static_cast<size_t>(k)];
    for (int q = 0; q < W; ++q) {
      if (q == r) continue;
      for (int p = 0; p < epp_; ++p) {
        int64_t o, l;
        part(plen(r, k) * es, p, &o, &l);
        if (l <= 0) continue;
        const int64_t at = static_cast<int64_t>(k) * pl.pe * es + o;
        copy(peers_[q] + off_RD + (static_cast<int64_t>(par) * W + r) * slot_bytes_ + at, m.peer_agent[q],
             out + static_cast<int64_t>(r) * block * es + at, m.own, l, 1, &sl.mid[k], done, m.peer_engines[q][p]);
      }
    }
    for (int q = 0; q < W; ++q)
      if (q != r)
        copy(peers_[q] + (kFrWord + r * kSdmaMaxPieces + k) * 4, m.peer_agent[q], word, m.cpu, 4, 1, &done, sl.gdf,
             m.peer_engines[q][0]);
    // and the own FR[r][k] once every phase-2 part of the piece has completed: the engines
    // read the own block of `out` for them, so the call may not count as done (and the
    // caller may not write `out`) before they are - the gather kernel waits for this word
    // with the peers' 
    if (W < 2) break;
    const int q0 = (r + 1) % W;
    copy(slab_ + (kFrWord + r * kSdmaMaxPieces + k) * 4, m.own, word, m.cpu, 4, 1, &done, sl.gdf,
         m.peer_engines[q0][0]);
  }
  ++st_.calls;
  return pl;
}

}  // namespace mxar
