#include "../core/env.h"
#include "xgmi_plane.h"

#include "../runtime/plane_geometry.h"
#include "residency.h"

#include <sys/prctl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <functional>
#include <random>
#include <sstream>
#include <string>
#include <stdexcept>

#include "../core/data_buffer.h"
#include "../core/log.h"
#include "../core/trace.h"

namespace mxar {

namespace {

// Arenas of this process by id: a worker cannot open its own process's IPC handles, so
// in-process peers (several workers of one process on one GPU) are found here.
std::mutex g_arena_mu;

// Resident kernel generations, process-wide: a plane's device words (go = gen << 32 | seq)
// serve its own resident kernels and its group's in turn, and a kernel must never take a go
// that an earlier kernel of either kind wrote for the same entry (its STOP at an idle exit).
std::atomic<uint32_t> g_res_gen{0};

// Pinned state words of plane groups (64 B each) from blocks that are never freed: freeing
// pinned memory may synchronise the device while a co-located kernel spins.
std::mutex g_gword_mu;
std::vector<uint32_t*> g_gword_free;

uint32_t* take_group_word() {
  std::lock_guard<std::mutex> g(g_gword_mu);
  if (g_gword_free.empty()) {
    uint32_t* blk = nullptr;
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&blk), 64 * 256, hipHostMallocCoherent | hipHostMallocMapped),
              "hipHostMalloc(group words)");
    std::memset(blk, 0, 64 * 256);
    for (int i = 255; i >= 0; --i) g_gword_free.push_back(blk + 16 * i);
  }
  uint32_t* w = g_gword_free.back();
  g_gword_free.pop_back();
  return w;
}

void give_group_word(uint32_t* w) {
  std::lock_guard<std::mutex> g(g_gword_mu);
  g_gword_free.push_back(w);
}

std::map<uint64_t, char*> g_arenas;

std::string to_hex(const std::string& b) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (unsigned char c : b) {
    s += d[c >> 4];
    s += d[c & 15];
  }
  return s;
}

// "xgmi1 pid=<pid> dev=<device> bytes=<arena bytes> id=<arena id> grid=<G> wgc=<cap>
// coarsen=<0|1> h=<hex IPC handle>" (csrc/runtime/plane_geometry.h); the IPC handle is required
PlaneDesc parse_desc(const std::string& s) {
  PlaneDesc d = parse_plane_desc(s);
  if (d.handle.size() != sizeof(hipIpcMemHandle_t)) throw ProtocolError("plane descriptor without an IPC handle");
  return d;
}

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace

// The co-located workers of one membership (this process, this GPU, one InitWorkers epoch):
// ONE resident kernel runs all their rounds, worker k's on its own slice of workgroups, fed
// from k's door ring (xgmi_threshold.hip threshold_group_resident_kernel). Found by key
// (device, the workers' arena ids in rank order, the membership epoch), so every worker of
// the membership joins the same group and a new membership forms a new one. The kernel runs
// while any worker has rounds; it leaves after an idle spell (the dispatcher decides for the
// whole group) and the next post launches it again. It is launched only once every worker has
// joined (its slices need every worker's words) - except for rounds being abandoned.
// where the last group teardown of this process is (debug_state while a configure leaves a
// group): 1 waiting for the kernel to leave, 2 synchronising its stream, 3 freeing orphans, 0 done
std::atomic<int> g_group_teardown{0};

struct PlaneGroup {
  enum : int { kPending = 0, kJoined = 1, kLeft = 2 };
  std::string key;
  int device = 0;
  std::vector<int> state;                 // per worker
  std::vector<XgmiRoundPlane*> planes;    // joined workers
  std::vector<char> in_kernel;            // served by the kernel launched last
  uint32_t* gword = nullptr;              // pinned: [0] the kernel's state (kResRunning / ...)
  uint32_t* gword_dev = nullptr;
  uint64_t* gdm = nullptr;                // device words: [0] the dispatcher's heartbeat
  hipStream_t stream = nullptr;
  bool launched = false;                  // a kernel was launched (gword[0] says whether it left)
  // memory of workers whose STOP the kernel never took (XgmiRoundPlane::leave_group): the
  // kernel may still poll their doors and words, so it is freed only once the kernel is
  // known to have exited - or never (leaked) if it did not
  std::vector<std::function<void()>> orphans;
  std::shared_ptr<void> residency;  // the group kernel's workgroups in the device budget (residency.h)
  std::mutex mu;

  PlaneGroup(std::string k, int dev, int workers, bool high_priority) : key(std::move(k)), device(dev) {
    state.assign(static_cast<size_t>(workers), kPending);
    planes.assign(static_cast<size_t>(workers), nullptr);
    in_kernel.assign(static_cast<size_t>(workers), 0);
    hip_check(hipSetDevice(device), "hipSetDevice");
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    hip_check(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, high_priority ? hi : lo),
              "hipStreamCreate(plane group)");
    gword = take_group_word();
    reinterpret_cast<volatile uint32_t*>(gword)[0] = kResExited;
    hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&gword_dev), gword, 0), "hipHostGetDevicePointer(group)");
    hip_check(hipMallocAsync(reinterpret_cast<void**>(&gdm), 64, stream), "hipMallocAsync(group words)");
    hip_check(hipMemsetAsync(gdm, 0, 64, stream), "hipMemsetAsync(group words)");
    hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize(group)");
  }
  ~PlaneGroup() {
    // every worker left: the dispatcher saw each one's STOP (or no kernel ran)
    const volatile uint32_t* g = gword;
    g_group_teardown.store(1);
    const auto t0 = std::chrono::steady_clock::now();
    while (launched && g[0] != kResExited && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10))
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    (void)hipSetDevice(device);
    const bool exited = !launched || g[0] == kResExited;
    if (exited) {
      g_group_teardown.store(2);
      (void)hipStreamSynchronize(stream);
      g_group_teardown.store(3);
      for (auto& f : orphans) f();
    } else if (!orphans.empty()) {
      MXAR_LOG(ERROR, "plane", "group kernel still running at teardown: " << orphans.size()
                                                                            << " workers' round memory leaked");
    }
    (void)hipFreeAsync(gdm, stream);
    (void)hipStreamDestroy(stream);
    if (exited) give_group_word(gword);  // else leaked: a kernel may still write it
    g_group_teardown.store(0);
  }
  volatile uint32_t* state_word() const { return gword; }
  bool kernel_left() const { return !launched || reinterpret_cast<volatile uint32_t*>(gword)[0] == kResExited; }

  // Launches a kernel for every joined worker (mu held; no kernel running).
  void launch_locked(XgmiRoundPlane* by) {
    std::vector<XgmiComm*> comms;
    std::vector<const XgmiComm::ResidentPlan*> plans;
    std::vector<GroupResidentMember> mem;
    double idle_us = 1000.0;
    for (size_t k = 0; k < planes.size(); ++k) {
      in_kernel[k] = 0;
      if (state[k] != kJoined) continue;
      XgmiRoundPlane* p = planes[k];
      comms.push_back(p->comm_.get());
      plans.push_back(&p->gplan_);
      GroupResidentMember m{};
      m.door = p->door_dev_;
      m.hstate = p->rstate_dev_;
      m.dm = reinterpret_cast<uint64_t*>(p->rdm_);
      m.hforce = p->hforce_dev_;
      m.habort = p->hforce_dev_ + 1;
      m.seq0 = p->rstate_[1] + 1u;  // its first entry not consumed yet
      mem.push_back(m);
      in_kernel[k] = 1;
      idle_us = p->o_.resident_idle_us;
    }
    if (comms.empty()) return;
    reinterpret_cast<volatile uint32_t*>(gword)[0] = kResRunning;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    try {
      XgmiComm::launch_group_resident(comms, plans, mem, gword_dev, gdm, g_res_gen.fetch_add(1) + 1u,
                                      static_cast<uint64_t>(idle_us * 100.0), stream);
    } catch (...) {
      reinterpret_cast<volatile uint32_t*>(gword)[0] = kResExited;
      std::fill(in_kernel.begin(), in_kernel.end(), 0);
      throw;
    }
    launched = true;
    by->st_.group_launches++;
  }

  // Worker k posted an entry: make sure a kernel takes it. A kernel launched before k joined
  // does not serve k: wait for it to leave (bounded), then launch one that does. With workers
  // still to join, the last of them launches it - unless `partial` (k's rounds are being
  // abandoned: they must run now, without the missing worker).
  void ensure(XgmiRoundPlane* by, int k, bool partial, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      {
        std::lock_guard<std::mutex> g(mu);
        if (kernel_left()) {
          const bool waiting = std::find(state.begin(), state.end(), kPending) != state.end();
          if (waiting && !partial) return;
          launch_locked(by);
          return;
        }
        if (in_kernel[static_cast<size_t>(k)]) return;  // running (or deciding to leave: it re-reads the doors)
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::duration<double>(2 * timeout_s + 5))
        throw ProtocolError("xgmi plane group: a kernel without this worker never left");
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
};

namespace {
std::mutex g_group_mu;
std::map<std::string, std::weak_ptr<PlaneGroup>> g_groups;
}  // namespace

XgmiRoundPlane::XgmiRoundPlane(const XgmiPlaneOptions& o) : o_(o) {
  if (o_.capacity <= 0) throw std::invalid_argument("xgmi plane: capacity (elements per round) must be > 0");
  if (o_.max_peers < 1 || o_.max_peers > 32 || o_.max_peers > kMaxRanks)
    throw std::invalid_argument("xgmi plane: max_peers must be in [1, 16]");
  if (o_.max_lag < 0 || o_.max_lag > 62) throw std::invalid_argument("xgmi plane: max_lag must be in [0, 62]");
  o_.ring = std::max(4, o_.ring);
  if (const char* e = study_env("MXAR_PLANE_SPLIT")) o_.split = std::atoi(e) != 0;  // A/B knob
  if (const char* e = study_env("MXAR_PLANE_COARSEN")) coarsen_full_ = std::atoi(e) != 0;  // A/B knob
  if (const char* e = study_env("MXAR_PLANE_WG_CHUNKS")) wg_chunks_ = std::max(0, std::atoi(e));  // A/B knob
  if (const char* q = std::getenv("GPU_MAX_HW_QUEUES"); q != nullptr && std::atoi(q) == 1)
    o_.resident_max = 0;  // one hardware queue per process: a resident kernel would hold it for every stream
  if (const char* e = std::getenv("MXAR_PLANE_RESIDENT")) o_.resident_max = std::atoll(e);
  if (const char* e = std::getenv("MXAR_PLANE_RESIDENT_IDLE_US")) o_.resident_idle_us = std::atof(e);
  if (const char* e = std::getenv("MXAR_PLANE_RESIDENT_GRID")) o_.resident_grid = std::atoi(e);
  o_.resident_grid = std::max(1, std::min(256, o_.resident_grid));
  const int64_t es = static_cast<int64_t>(dtype_size(o_.dtype));
  flag_gran_ = o_.min_chunk > 0 ? std::min<int64_t>(XgmiComm::min_chunk_bytes(), o_.min_chunk * es)
                                : XgmiComm::min_chunk_bytes();
  // The flag table is reserved at its largest size over every membership of <= max_peers
  // workers and maxLag <= max_lag, so it sits at the same place in every layout: a late
  // store of an older layout can only hit a flag word (holding an older, smaller epoch),
  // never turn data into a flag. Then the largest layout any such membership needs.
  for (int P = 1; P <= o_.max_peers; ++P) {
    const int64_t block = static_cast<int64_t>(f32_ceil_div(o_.capacity, P));
    for (int lag = 0; lag <= o_.max_lag; ++lag)
      flag_bytes_ =
          std::max(flag_bytes_, XgmiComm::flag_bytes(P, std::max<int64_t>(block * es, 16), lag + 1, flag_gran_));
  }
  int64_t max_counts = 1;  // P x chunks per round, over every membership this plane may see
  for (int P = 1; P <= o_.max_peers; ++P) {
    const int64_t block = static_cast<int64_t>(f32_ceil_div(o_.capacity, P));
    const XgmiComm::Layout L =
        XgmiComm::layout(P, std::max<int64_t>(block * es, 16), o_.max_lag + 1, flag_bytes_, flag_gran_);
    arena_bytes_ = std::max(arena_bytes_, L.slab_bytes);
    for (int lag = 0; lag <= o_.max_lag; ++lag) {
      const int64_t maxch =
          XgmiComm::layout(P, std::max<int64_t>(block * es, 16), lag + 1, flag_bytes_, flag_gran_).maxch;
      max_counts = std::max<int64_t>(max_counts, static_cast<int64_t>(P) * maxch);
      split_bytes_ = std::max(split_bytes_, XgmiComm::split_scratch_bytes(P, maxch));
    }
  }
  arena_bytes_ = XgmiComm::ipc_safe_bytes(arena_bytes_);
  hip_check(hipSetDevice(o_.device), "hipSetDevice");
  hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&arena_), arena_bytes_, hipDeviceMallocFinegrained),
            "hipExtMallocWithFlags(plane arena)");
  // zeroed ONCE, before anyone can know the handle: every flag reads "epoch 0 done"
  hip_check(hipMemset(arena_, 0, arena_bytes_), "hipMemset(plane arena)");
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&hforce_), 64, hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(force word)");
  std::memset(hforce_, 0, 64);
  hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&hforce_dev_), hforce_, 0), "hipHostGetDevicePointer");
  // Per-round counts + error word: a pinned ring the host reads and its HBM twin the
  // workgroups write, both sized here for the largest membership. Never reallocated:
  // hipFree / hipHostFree in configure() could synchronise the device while a peer's round
  // kernel spins waiting for this worker's re-initialisation.
  ring_stride_ = static_cast<size_t>(max_counts) + 4;
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&ring_), ring_stride_ * 4 * o_.ring,
                          hipHostMallocMapped | hipHostMallocCoherent),
            "hipHostMalloc(plane ring)");
  std::memset(ring_, 0, ring_stride_ * 4 * o_.ring);
  hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&ring_dev_), ring_, 0), "hipHostGetDevicePointer(ring)");
  hip_check(hipMalloc(reinterpret_cast<void**>(&cnt_vram_), ring_stride_ * 4 * o_.ring), "hipMalloc(plane counts)");
  hip_check(hipMalloc(reinterpret_cast<void**>(&ctl_mem_), 256), "hipMalloc(plane ctl)");
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&door_), sizeof(ResidentDoor) * kResidentDoors + 64,
                          hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(resident door)");
  std::memset(door_, 0, sizeof(ResidentDoor) * kResidentDoors + 64);
  hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&door_dev_), door_, 0), "hipHostGetDevicePointer(door)");
  rstate_ = reinterpret_cast<volatile uint32_t*>(door_ + kResidentDoors);
  rstate_dev_ = reinterpret_cast<uint32_t*>(door_dev_ + kResidentDoors);
  hip_check(hipMalloc(reinterpret_cast<void**>(&rdm_), 256), "hipMalloc(resident words)");
  hip_check(hipMemset(rdm_, 0, 256), "hipMemset(resident words)");
  hip_check(hipMemset(ctl_mem_, 0, 256), "hipMemset(plane ctl)");
  // split-chunk scratch (decision words, slice counters; XgmiComm::RoundSpec::split_scratch)
  hip_check(hipMalloc(&split_mem_, split_bytes_), "hipMalloc(plane split scratch)");
  hip_check(hipMemset(split_mem_, 0, split_bytes_), "hipMemset(plane split scratch)");
  hip_check(hipEventCreateWithFlags(&rel_ev_, hipEventDisableTiming), "hipEventCreate(release)");
  for (int i = 0; i < o_.ring; ++i) {
    hipEvent_t e = nullptr;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    events_.push_back(e);
  }
  // High priority: HIP serves each priority level from its own hardware-queue pool, so the
  // plane's persistent round kernels never sit in the same hardware queue as the default
  // stream (a marker or kernel queued behind a spinning round in a shared queue would wait
  // for that round - a deadlock when the round waits for a peer fed by that work; seen in
  // a kernel trace with two workers in one process). Co-located workers of one job do not
  // need queues of their own: their rounds share one group kernel (PlaneGroup).
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  const hipError_t se = hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, o_.high_priority ? hi : lo);
  if (se != hipSuccess) {  // release what the constructor allocated so far
    for (hipEvent_t e : events_) (void)hipEventDestroy(e);
    if (rel_ev_) (void)hipEventDestroy(rel_ev_);
    (void)hipFree(split_mem_);
    (void)hipFree(rdm_);
    (void)hipFree(ctl_mem_);
    (void)hipFree(cnt_vram_);
    (void)hipHostFree(ring_);
    (void)hipHostFree(door_);
    (void)hipHostFree(hforce_);
    (void)hipFree(arena_);
    hip_check(se, "hipStreamCreate(plane)");
  }
  // keep freed round buffers in the device's default pool instead of returning them to the
  // driver at every synchronisation (the next round reuses them)
  hipMemPool_t mp = nullptr;
  if (hipDeviceGetDefaultMemPool(&mp, o_.device) == hipSuccess && mp != nullptr) {
    uint64_t keep = UINT64_MAX;
    (void)hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &keep);
  }
  (void)hipGetLastError();
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, arena_), "hipIpcGetMemHandle(plane arena)");
  std::random_device rd;
  arena_id_ = (static_cast<uint64_t>(rd()) << 32) ^ rd() ^ reinterpret_cast<uintptr_t>(arena_);
  {
    std::lock_guard<std::mutex> g(g_arena_mu);
    g_arenas[arena_id_] = arena_;
  }
  std::ostringstream os;
  // the knobs that shape a round's geometry travel in the descriptor: every worker of a job
  // derives the same chunking from InitWorkers alone (plane_geometry.h)
  int eff_grid = o_.grid;
  if (eff_grid <= 0) {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, o_.device);
    eff_grid = 2 * cus;
    if (const char* g = std::getenv("MXAR_GRID")) eff_grid = std::max(1, std::atoi(g));
  }
  os << "xgmi1 pid=" << static_cast<long>(getpid()) << " dev=" << o_.device << " bytes=" << arena_bytes_
     << " id=" << arena_id_ << " grid=" << eff_grid << " wgc=" << wg_chunks_ << " coarsen=" << (coarsen_full_ ? 1 : 0)
     << " h=" << to_hex(std::string(reinterpret_cast<const char*>(&h), sizeof(h)));
  desc_ = os.str();
  th_ = std::thread([this] { completion_loop(); });
  MXAR_LOG(INFO, "plane", "xgmi plane on device " << o_.device << ": arena " << (arena_bytes_ >> 20) << " MiB for <= "
                                                  << o_.max_peers << " workers, maxLag <= " << o_.max_lag);
}

XgmiRoundPlane::~XgmiRoundPlane() {
  *alive_ = false;
  try {
    abort(0x7fffffff);
    drain();
    leave_group();
    park_resident();
  } catch (...) {
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  stop_flag_.store(true);
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  (void)hipSetDevice(o_.device);
  (void)hipStreamSynchronize(stream_);
  {
    std::lock_guard<std::mutex> g(rel_->mu);
    if (!rel_->ptrs.empty()) (void)hipStreamSynchronize(nullptr);
    for (void* q : rel_->ptrs) (void)hipFree(q);
    for (void* q : rel_->free) (void)hipFree(q);
    rel_->ptrs.clear();
    rel_->free.clear();
    rel_->bytes = 0;  // outputs still held by users are freed stream-ordered when dropped
  }
  if (rel_ev_) (void)hipEventDestroy(rel_ev_);
  for (auto& [ev, v] : rel_pend_) {
    (void)hipEventDestroy(ev);
    for (void* q : v) (void)hipFree(q);
  }
  for (hipEvent_t ev : rel_spare_) (void)hipEventDestroy(ev);
  comm_.reset();
  for (auto& [h, p] : mapped_) (void)hipIpcCloseMemHandle(p);
  {
    std::lock_guard<std::mutex> g(g_arena_mu);
    g_arenas.erase(arena_id_);
  }
  for (hipEvent_t e : events_) (void)hipEventDestroy(e);
  if (ring_) (void)hipHostFree(ring_);
  if (cnt_vram_) (void)hipFree(cnt_vram_);
  if (ctl_mem_) (void)hipFree(ctl_mem_);
  if (split_mem_) (void)hipFree(split_mem_);
  if (hforce_) (void)hipHostFree(hforce_);
  if (door_) (void)hipHostFree(door_);
  if (rdm_) (void)hipFree(rdm_);
  if (stream_) (void)hipStreamDestroy(stream_);
  if (alloc_stream_) (void)hipStreamDestroy(alloc_stream_);
  if (arena_) (void)hipFree(arena_);
}

std::shared_ptr<void> XgmiRoundPlane::buffer(size_t bytes, bool user_visible) {
  void* p = nullptr;
  hip_check(hipMallocAsync(&p, std::max<size_t>(bytes, 256), stream_), "hipMallocAsync(plane)");
  const hipStream_t s = stream_;
  std::weak_ptr<bool> alive = alive_;
  // released on the plane stream (ordered after every round that may still read it); an
  // output the user keeps past the plane's lifetime is freed synchronously instead.
  // A round output went to the dataSink as a tensor: work the sink queued on the default
  // stream (torch's, e.g. a clone) may still read it when the last reference drops, so its
  // release is also ordered after the default stream - otherwise the next round could get
  // the same block from the pool and overwrite it under that work.
  std::weak_ptr<ReleaseQ> rq = rel_;
  static const bool via_event = [] {
    const char* e = study_env("MXAR_PLANE_RELEASE");
    return e != nullptr && std::string(e) == "event";
  }();
  return std::shared_ptr<void>(p, [s, alive, user_visible, rq](void* q) {
    auto a = alive.lock();
    if (a && *a) {
      if (user_visible) {
        if (!via_event) {
          // freed on the default stream itself: ordered after whatever the sink queued
          // there, and the stream-ordered pool orders a later reuse by the plane stream
          // after that free - no event or stream wait on the launch path
          (void)hipFreeAsync(q, nullptr);
          return;
        }
        if (auto r = rq.lock()) {  // MXAR_PLANE_RELEASE=event: freed by the next launch, behind an event
          std::lock_guard<std::mutex> g(r->mu);
          r->ptrs.push_back(q);
          return;
        }
      }
      (void)hipFreeAsync(q, s);
    } else {
      // the plane is gone: stream-ordered on the default stream - hipFree would wait for
      // every kernel on the device, e.g. another plane's round spinning on its peers
      // (profiles/round2/sync_probe.md)
      (void)hipFreeAsync(q, nullptr);
    }
  });
}

std::shared_ptr<void> XgmiRoundPlane::out_buffer(size_t bytes, std::shared_ptr<std::atomic<bool>>* exported) {
  bytes = std::max<size_t>(bytes, 256);
  void* p = nullptr;
  {
    std::lock_guard<std::mutex> g(rel_->mu);
    if (rel_->bytes == bytes && !rel_->free.empty()) {
      p = rel_->free.back();
      rel_->free.pop_back();
    }
  }
  if (p == nullptr) {
    hip_check(hipMallocAsync(&p, bytes, stream_), "hipMallocAsync(plane output)");
    st_.pool_grown++;
  }
  auto flag = std::make_shared<std::atomic<bool>>(false);
  *exported = flag;
  const hipStream_t s = stream_;
  std::weak_ptr<bool> alive = alive_;
  std::weak_ptr<ReleaseQ> rq = rel_;
  const bool ordered = o_.order_release;
  return std::shared_ptr<void>(p, [s, alive, rq, flag, bytes, ordered](void* q) {
    auto a = alive.lock();
    auto r = rq.lock();
    if (a && *a && r) {
      std::lock_guard<std::mutex> g(r->mu);
      if (r->bytes == bytes) {
        // exported: another stream may still read it - reusable only behind the default
        // stream (flush_releases at the next launch); otherwise at once, on the plane stream
        if (ordered && flag->load(std::memory_order_relaxed))
          r->ptrs.push_back(q);
        else
          r->free.push_back(q);
        return;
      }
      // an output of an older layout: freed, stream-ordered behind whoever may still read it
      (void)hipFreeAsync(q, ordered && flag->load() ? nullptr : s);
      return;
    }
    // the plane is gone: stream-ordered on the default stream - hipFree would wait for every
    // kernel on the device, e.g. another plane's round spinning on its peers
    (void)hipFreeAsync(q, nullptr);
  });
}

void XgmiRoundPlane::reset_pool(size_t bytes) {
  bytes = std::max<size_t>(bytes, 256);
  std::vector<void*> fr, pend;
  {
    std::lock_guard<std::mutex> g(rel_->mu);
    if (rel_->bytes == bytes) return;
    fr.swap(rel_->free);
    pend.swap(rel_->ptrs);
    rel_->bytes = bytes;
  }
  for (void* q : fr) (void)hipFreeAsync(q, stream_);
  for (void* q : pend) (void)hipFreeAsync(q, nullptr);
  // about 3 outputs are live at once (the round in flight, the one a sink holds, the one
  // being released): grow the pool now - growing it on the round path costs ~8 ms per
  // 256 MiB buffer (profiles/round2/sync_probe.md)
  // (resident-size rounds - every round then draws from this pool, see resident_out - keep
  // more: a sink holding a few outputs must not push rounds off the resident kernel)
  const bool resident_size = grouped_ || (o_.resident_max > 0 && static_cast<int64_t>(bytes) <= o_.resident_max);
  std::vector<void*> warm(resident_size ? 8 : 3, nullptr);
  for (void*& w : warm) hip_check(hipMallocAsync(&w, bytes, stream_), "hipMallocAsync(pool)");
  std::lock_guard<std::mutex> g(rel_->mu);
  for (void* w : warm) rel_->free.push_back(w);
}

void XgmiRoundPlane::flush_releases() {
  std::vector<void*> ptrs;
  {
    std::lock_guard<std::mutex> g(rel_->mu);
    ptrs.swap(rel_->ptrs);
  }
  // releases parked by resident rounds: their events were recorded on the default stream
  // before the one below, so its wait covers them
  for (auto& [ev, v] : rel_pend_) {
    ptrs.insert(ptrs.end(), v.begin(), v.end());
    rel_spare_.push_back(ev);
  }
  rel_pend_.clear();
  if (ptrs.empty()) return;
  // one event for every exported output released since the last launch: their reuse by
  // this and later launches comes after everything the default stream held at this point -
  // e.g. a sink's clone of the round output
  hip_check(hipEventRecord(rel_ev_, nullptr), "hipEventRecord(release)");
  hip_check(hipStreamWaitEvent(stream_, rel_ev_, 0), "hipStreamWaitEvent(release)");
  std::lock_guard<std::mutex> g(rel_->mu);
  for (void* q : ptrs) rel_->free.push_back(q);
}

void XgmiRoundPlane::set_done(DoneFn fn) {
  std::lock_guard<std::mutex> g(done_mu_);
  done_ = std::move(fn);
}

char* XgmiRoundPlane::map_peer(const std::string& desc) {
  const PlaneDesc d = parse_desc(desc);
  if (d.pid == static_cast<long>(getpid())) {  // a worker of this process: no IPC
    std::lock_guard<std::mutex> g(g_arena_mu);
    auto it = g_arenas.find(d.id);
    if (it == g_arenas.end()) throw ProtocolError("plane descriptor names an arena of this process that is gone");
    if (d.device != o_.device) {
      int can = 0;
      (void)hipDeviceCanAccessPeer(&can, o_.device, d.device);
      if (!can) throw ProtocolError("no peer access from device " + std::to_string(o_.device) + " to " +
                                    std::to_string(d.device));
      const hipError_t e = hipDeviceEnablePeerAccess(d.device, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) hip_check(e, "hipDeviceEnablePeerAccess");
      (void)hipGetLastError();
    }
    return it->second;
  }
  auto it = mapped_.find(d.handle);
  if (it != mapped_.end()) return it->second;
  hipIpcMemHandle_t h;
  std::memcpy(&h, d.handle.data(), sizeof(h));
  void* p = nullptr;
  hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(peer arena)");
  mapped_[d.handle] = static_cast<char*>(p);
  st_.peer_maps++;
  return static_cast<char*>(p);
}

void XgmiRoundPlane::configure(const PlaneConfig& cfg) {
  if (cfg.peers < 1 || cfg.peers > o_.max_peers)
    throw ProtocolError("xgmi plane sized for <= " + std::to_string(o_.max_peers) + " workers, InitWorkers has " +
                        std::to_string(cfg.peers));
  if (cfg.maxLag > o_.max_lag)
    throw ProtocolError("xgmi plane sized for maxLag <= " + std::to_string(o_.max_lag) + ", InitWorkers has " +
                        std::to_string(cfg.maxLag));
  if (cfg.dataSize <= 0 || cfg.dataSize > o_.capacity)
    throw ProtocolError("xgmi plane holds <= " + std::to_string(o_.capacity) + " elements per round, dataSize " +
                        std::to_string(cfg.dataSize));
  if (cfg.maxChunkSize <= 0) throw ProtocolError("maxChunkSize must be > 0");
  if (static_cast<int>(cfg.descriptors.size()) != cfg.peers)
    throw ProtocolError("InitWorkers.planes must hold one descriptor per worker");
  // the previous epoch's rounds are abandoned before the arena is laid out again (their
  // results would be dropped as an older epoch; a round still at its lag gate must not
  // wait for a peer that left the membership)
  struct StageReset {
    std::atomic<int>& s;
    ~StageReset() { s.store(0); }
  } stage_reset{cfg_stage_};
  if (configured_) {
    cfg_stage_.store(1);
    abort(last_round_);
    cfg_stage_.store(2);
    drain();
  }
  cfg_stage_.store(3);
  leave_group();
  if (orphaned_) {
    configured_ = false;
    throw ProtocolError("xgmi plane: the group kernel never released this worker (its STOP was not taken); "
                        "the plane cannot be configured again");
  }
  cfg_stage_.store(4);
  park_resident();  // the stream work below must not queue behind it
  cfg_stage_.store(5);
  rplan_tried_ = false;
  rplan_ = XgmiComm::ResidentPlan();
  res_token_.reset();
  hip_check(hipSetDevice(o_.device), "hipSetDevice");
  const int P = cfg.peers;
  const int64_t es = static_cast<int64_t>(dtype_size(o_.dtype));
  const int64_t slot = std::max<int64_t>(static_cast<int64_t>(f32_ceil_div(cfg.dataSize, P)) * es, 16);
  const XgmiComm::Layout L = XgmiComm::layout(P, slot, cfg.maxLag + 1, flag_bytes_, flag_gran_);
  if (L.slab_bytes > arena_bytes_) throw ProtocolError("xgmi plane arena too small for this membership");
  // the round geometry from InitWorkers alone: every worker of the job computes the same one
  const PlaneGeometry geo = plane_geometry(cfg, L.maxch, es);
  block_ = geo.block;
  chunk_ = geo.chunk;
  nch_ref_ = geo.nch_ref;
  coarse_ = geo.coarse;
  const int64_t nch = geo.nch;
  if (geo.coarse > 1) st_.coarsened++;
  if (geo.coarsened_for_flags)
    MXAR_LOG(INFO, "plane", "maxChunkSize " << cfg.maxChunkSize << " is finer than the flag table at thresholds 1: "
                                            << "kernel chunks of " << chunk_ << " elements, counts per reference chunk");
  nch_ = static_cast<int>(nch);
  std::vector<char*> bases(P, nullptr);
  for (int k = 0; k < P; ++k) {
    auto it = cfg.descriptors.find(k);
    if (it == cfg.descriptors.end() || it->second.empty()) throw ProtocolError("InitWorkers.planes misses worker " + std::to_string(k));
    bases[k] = k == cfg.id ? arena_ : map_peer(it->second);
  }
  cfg_stage_.store(6);
  comm_.reset();
  // No device-synchronising call from here on: a peer's round kernel of the new epoch may
  // already spin waiting for this worker (its lag gate opens on the progress published
  // below). The communicator reuses the plane's arena and control words; the control words
  // are reset stream-ordered, after the drained old epoch.
  hip_check(hipMemsetAsync(ctl_mem_, 0, 256, stream_), "hipMemsetAsync(plane ctl)");
  // a new membership may reuse round epochs of the abandoned one: no stale decision survives
  hip_check(hipMemsetAsync(split_mem_, 0, split_bytes_, stream_), "hipMemsetAsync(plane split scratch)");
  comm_ = std::make_unique<XgmiComm>(cfg.id, P, o_.device, slot, o_.grid, o_.timeout_s, cfg.maxLag + 1, arena_,
                                     arena_bytes_, flag_bytes_, ctl_mem_, flag_gran_);
  comm_->connect_ptrs(bases);
  comm_->set_phase_stamps(stamps_, stamp_slots_);
  // Every round of the previous epoch has finished here (drained): say so to the peers. Their
  // lag gates for this epoch's first maxLag + 1 rounds wait for exactly this value, so no
  // worker writes new-epoch data while any worker may still run an old-epoch round.
  // Grow the stream-ordered pool now for the rounds' output buffers (an output is released
  // one launch after its sink dropped it, so ~3 are live at once): growing it in the round
  // path costs ~8 ms per 256 MiB buffer (profiles/round2/sync_probe.md) - paid here instead.
  grouped_ = colocated(cfg).size() > 1;  // every round then draws its output from the pool
  reset_pool(static_cast<size_t>(cfg.dataSize) * static_cast<size_t>(dtype_size(o_.dtype)));
  comm_->publish_progress(cfg.roundBase, stream_);
  hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize(publish progress)");
  if (static_cast<size_t>(P) * nch_ + 4 > ring_stride_) throw ProtocolError("xgmi plane: counts ring too small");
  {
    // the kernel counts into the slot's HBM twin and copies them, with the error word, into
    // the pinned slot at round end (no per-round D2H copy); read after the completion event
    std::lock_guard<std::mutex> g(mu_);
    free_slots_.clear();
    for (int i = o_.ring - 1; i >= 0; --i) free_slots_.push_back(i);
  }
  cfg_ = cfg;
  configured_ = true;
  last_round_ = cfg.startRound - 1;
  err_seen_ = 0;
  cfg_stage_.store(7);
  if (grouped_) join_group(cfg);
  MXAR_LOG(INFO, "plane", "xgmi plane: worker " << cfg.id << " of " << P << ", block " << block_ << ", chunk "
                                                << chunk_ << " x " << nch_ << " (" << nch_ref_
                                                << " reference chunks), rows " << cfg.maxLag + 1
                                                << ", round epochs from " << cfg.roundBase + 1);
}

std::vector<std::pair<int, uint64_t>> XgmiRoundPlane::colocated(const PlaneConfig& cfg) const {
  std::vector<std::pair<int, uint64_t>> v;
  for (int k = 0; k < cfg.peers; ++k) {
    auto it = cfg.descriptors.find(k);
    if (it == cfg.descriptors.end() || it->second.empty()) continue;
    const PlaneDesc d = parse_desc(it->second);
    if (d.pid == static_cast<long>(getpid()) && d.device == o_.device) v.emplace_back(k, d.id);
  }
  return v;
}

void XgmiRoundPlane::join_group(const PlaneConfig& cfg) {
  const auto mates = colocated(cfg);
  const int Y = static_cast<int>(mates.size());
  if (Y > kMaxRanks)
    throw ProtocolError("xgmi plane: at most " + std::to_string(kMaxRanks) + " workers of a job per process and GPU");
  if (const char* q = std::getenv("GPU_MAX_HW_QUEUES"); q != nullptr && std::atoi(q) == 1)
    throw ProtocolError("xgmi plane: co-located workers need GPU_MAX_HW_QUEUES >= 2 (their group kernel holds a "
                        "hardware queue while the inputs are produced on another)");
  // the group kernel's geometry: round()'s for this membership, every chunk one workgroup's
  XgmiComm::RoundSpec spec;
  spec.block = block_;
  spec.chunk = chunk_;
  spec.order_ref = o_.order_ref;
  spec.host_force = hforce_dev_;
  spec.lag_wait_us = o_.lag_wait_us;
  spec.host_abort = hforce_dev_ + 1;
  if (o_.split) {  // few large chunks: slices over several workgroups, as the launch path does
    spec.split_scratch = split_mem_;
    spec.split_bytes = split_bytes_;
  }
  gplan_ = comm_->plan_resident(cfg.dataSize, o_.dtype, cfg.thReduce, cfg.thComplete, spec, 1 << 20, true);
  if (gplan_.grid <= 0) throw ProtocolError("xgmi plane: this membership's rounds do not fit the group kernel");
  // every slice's workgroups must be resident at once (they wait for each other's rounds):
  // two workgroups per CU over the workers, the PlaneJob default (grid = 512 / workers) - and
  // together with every other spinning kernel of this process on the device (residency.h)
  const int cap = Residency::get().capacity(o_.device);
  if (static_cast<int64_t>(Y) * gplan_.grid + 1 > cap)
    throw ProtocolError("xgmi plane: " + std::to_string(Y) + " co-located workers x " + std::to_string(gplan_.grid) +
                        " workgroups exceed the " + std::to_string(cap) +
                        " a group kernel keeps resident: build the planes with grid <= " + std::to_string((cap - 1) / Y));
  std::ostringstream key;
  key << "dev" << o_.device << " e" << cfg.epoch;
  int idx = -1;
  for (int i = 0; i < Y; ++i) {
    key << ' ' << mates[i].second;
    if (mates[i].first == cfg.id) idx = i;
  }
  if (idx < 0) throw ProtocolError("xgmi plane: this worker is not among its own co-located workers");
  std::shared_ptr<PlaneGroup> g;
  {
    std::lock_guard<std::mutex> lk(g_group_mu);
    for (auto it = g_groups.begin(); it != g_groups.end();) it = it->second.expired() ? g_groups.erase(it) : std::next(it);
    auto& w = g_groups[key.str()];
    g = w.lock();
    if (!g) {
      auto fresh = std::make_shared<PlaneGroup>(key.str(), o_.device, Y, o_.high_priority);
      if (!o_.residency_external)  // the dispatcher wave + every slice (throws with the budget named)
        fresh->residency = Residency::get().reserve(o_.device, Y * gplan_.grid + 1, "plane group " + key.str());
      g = fresh;
      w = g;
    }
  }
  rstate_[1] = res_seq_ - 1u;  // every entry before res_seq_ was taken (or dropped) before
  std::lock_guard<std::mutex> lk(g->mu);
  // (a worker that left this membership's group may join it again - the same InitWorkers
  // delivered twice; a kernel launched meanwhile does not serve it and leaves before one that
  // does is launched, PlaneGroup::ensure)
  if (g->state[static_cast<size_t>(idx)] == PlaneGroup::kJoined && g->planes[static_cast<size_t>(idx)] != this)
    throw ProtocolError("xgmi plane: two workers of one membership claim the same group slot");
  g->planes[static_cast<size_t>(idx)] = this;
  g->state[static_cast<size_t>(idx)] = PlaneGroup::kJoined;
  group_ = g;
  gidx_ = idx;
  st_.group_size = Y;
  // the last worker to join starts the kernel: the others' first rounds may be posted already
  if (std::find(g->state.begin(), g->state.end(), PlaneGroup::kPending) == g->state.end() && g->kernel_left())
    g->launch_locked(this);
}

void XgmiRoundPlane::leave_group() {
  if (!group_) return;
  std::shared_ptr<PlaneGroup> g = group_;
  cfg_stage_.store(31);  // leave_group: 31 deciding, 32 waiting for the STOP, 33 leaving, 34 group released
  bool serving = false;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    serving = g->in_kernel[static_cast<size_t>(gidx_)] != 0 && !g->kernel_left();
    // from here on no kernel launched for the group serves this worker: a co-located worker's
    // post could otherwise relaunch the group kernel between the running kernel taking our
    // STOP and our leaving, with a slice that then took this worker's NEXT membership's rounds
    // from its door (an old-membership kernel running a new-membership round until the
    // deadline; profiles/round6/README.md section 5)
    g->state[static_cast<size_t>(gidx_)] = PlaneGroup::kLeft;
  }
  bool lost = false;
  if (serving) {
    // a STOP entry ends this worker's slice; the kernel goes on for the others (or leaves
    // when this was the last)
    ResidentDoor e{};
    e.cmd = kResStop;
    const uint32_t seq = res_seq_;
    cfg_stage_.store(32);
    if (post_door(e, g->state_word())) {
      const auto t0 = std::chrono::steady_clock::now();
      while (static_cast<int32_t>(rstate_[1] - seq) < 0 && !g->kernel_left()) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::duration<double>(2 * o_.timeout_s + 5)) {
          MXAR_LOG(ERROR, "plane", "the group kernel did not take this worker's STOP");
          lost = true;
          break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
  }
  if (lost) {
    // The kernel may still serve this worker's slice: its door, device words, force / abort
    // words, counts, control words, split scratch and arena stay allocated until the group
    // sees the kernel exit (PlaneGroup::orphans), never freed under a running kernel
    std::lock_guard<std::mutex> lk(g->mu);
    g->orphans.push_back([door = door_, rdm = rdm_, hforce = hforce_, ctl = ctl_mem_, split = split_mem_,
                          cnt = cnt_vram_, ring = ring_, arena = arena_] {
      (void)hipHostFree(door);
      (void)hipHostFree(hforce);
      (void)hipHostFree(ring);
      (void)hipFree(rdm);
      (void)hipFree(ctl);
      (void)hipFree(split);
      (void)hipFree(cnt);
      (void)hipFree(arena);
    });
    door_ = nullptr;
    rdm_ = nullptr;
    hforce_ = nullptr;
    ctl_mem_ = nullptr;
    split_mem_ = nullptr;
    cnt_vram_ = nullptr;
    ring_ = nullptr;
    arena_ = nullptr;
    orphaned_ = true;
  }
  rstate_[1] = res_seq_ - 1u;  // entries no kernel took are dropped
  cfg_stage_.store(33);
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->state[static_cast<size_t>(gidx_)] = PlaneGroup::kLeft;
    g->planes[static_cast<size_t>(gidx_)] = nullptr;
    g->in_kernel[static_cast<size_t>(gidx_)] = 0;
  }
  group_.reset();
  cfg_stage_.store(34);
  g.reset();  // the last worker out tears the group down here (waits for its kernel to leave)
  cfg_stage_.store(35);
  gidx_ = -1;
  gplan_ = XgmiComm::ResidentPlan();
  st_.group_size = 0;
}

void XgmiRoundPlane::launch_group(int round, const Payload& input, bool cold) {
  const int64_t n = cfg_.dataSize;
  const int64_t es = static_cast<int64_t>(dtype_size(o_.dtype));
  const int dcode = static_cast<int>(o_.dtype);
  Rec rec;
  rec.round = round;
  rec.epoch = cfg_.epoch;
  rec.cold = cold;
  rec.round_epoch = epoch_of(round);
  const void* in_ptr = nullptr;
  if (!cold) {
    if (!input || static_cast<int64_t>(input->size()) != n) throw ProtocolError("xgmi plane: input must hold dataSize elements");
    auto* dp = dynamic_cast<const DevicePayload*>(input.get());
    if (dp != nullptr && dp->device() == o_.device && dp->dtype() == dcode) {
      // no stream orders the group kernel after the producer: the host waits for it (normal-
      // priority streams: never queued behind the group kernel's high-priority queue). A query
      // first: a finished producer - the usual case - costs no blocking runtime call
      if (dp->ready()) {
        const hipEvent_t ev = static_cast<hipEvent_t>(dp->ready().get());
        const hipError_t q = hipEventQuery(ev);
        if (q == hipErrorNotReady) {
          (void)hipGetLastError();
          hip_check(hipEventSynchronize(ev), "hipEventSynchronize(input)");
        } else {
          hip_check(q, "hipEventQuery(input)");
        }
      } else if (dp->stream() && dp->stream() != stream_) {
        const hipError_t q = hipStreamQuery(dp->stream());
        if (q == hipErrorNotReady) {
          (void)hipGetLastError();
          hip_check(hipStreamSynchronize(dp->stream()), "hipStreamSynchronize(input)");
        } else {
          hip_check(q, "hipStreamQuery(input)");
        }
      }
      in_ptr = dp->bytes();
      rec.input = input;  // held until the round completed
    } else {
      // staged on the side stream (normal priority) and waited for: a host payload, another
      // device's, or another dtype
      if (alloc_stream_ == nullptr)
        hip_check(hipStreamCreateWithFlags(&alloc_stream_, hipStreamNonBlocking), "hipStreamCreate(plane side)");
      const hipStream_t ss = alloc_stream_;
      auto side_buf = [&](size_t bytes) {
        void* p = nullptr;
        hip_check(hipMallocAsync(&p, std::max<size_t>(bytes, 256), ss), "hipMallocAsync(plane staging)");
        return std::shared_ptr<void>(p, [ss](void* q) { (void)hipFreeAsync(q, ss); });
      };
      void* src = nullptr;
      DType sdt = DType::F32;
      std::shared_ptr<void> up;
      if (dp != nullptr && dp->device() == o_.device) {
        if (dp->ready()) hip_check(hipStreamWaitEvent(ss, static_cast<hipEvent_t>(dp->ready().get()), 0), "hipStreamWaitEvent");
        else if (dp->stream()) hip_check(hipStreamSynchronize(dp->stream()), "hipStreamSynchronize(input)");
        src = const_cast<void*>(dp->bytes());
        sdt = static_cast<DType>(dp->dtype());
        rec.input = input;
      } else {
        const std::vector<float> h = input->to_host();
        up = side_buf(static_cast<size_t>(n * 4));
        hip_check(hipMemcpyAsync(up.get(), h.data(), n * 4, hipMemcpyHostToDevice, ss), "hipMemcpyAsync H2D");
        hip_check(hipStreamSynchronize(ss), "hipStreamSynchronize(upload)");  // h is pageable and local
        src = up.get();
      }
      if (sdt == o_.dtype && up) {
        rec.staging = up;
      } else {
        rec.staging = side_buf(static_cast<size_t>(n * es));
        launch_cast(src, sdt, rec.staging.get(), o_.dtype, n, ss);
      }
      hip_check(hipStreamSynchronize(ss), "hipStreamSynchronize(staging)");
      in_ptr = rec.staging.get();
    }
  }
  rec.out = resident_out(static_cast<size_t>(n * es), &rec.exported, true);
  if (!rec.out) throw ProtocolError("xgmi plane: no round output buffer for the group kernel");
  {
    std::unique_lock<std::mutex> lk(mu_);
    rec.slot = take_slot(lk);
  }
  int32_t* slot_dev = ring_dev_ + static_cast<size_t>(rec.slot) * ring_stride_;
  ResidentDoor e{};
  e.in = reinterpret_cast<uint64_t>(cold ? rec.out.get() : in_ptr);
  e.out = reinterpret_cast<uint64_t>(rec.out.get());
  e.counts = reinterpret_cast<uint64_t>(cnt_vram_ + static_cast<size_t>(rec.slot) * ring_stride_);
  e.counts_host = reinterpret_cast<uint64_t>(slot_dev);
  e.err_out = reinterpret_cast<uint64_t>(slot_dev + ring_stride_ - 1);
  e.done_out = reinterpret_cast<uint64_t>(slot_dev + ring_stride_ - 2);
  e.epoch = rec.round_epoch;
  e.cmd = cold ? kResCold : kResRound;
  try {
    TraceScope span("plane", [&] {
      return std::make_pair(std::string(cold ? "group cold round " : "group round ") + std::to_string(round),
                            "{\"worker\":" + std::to_string(cfg_.id) + ",\"bytes\":" + std::to_string(n * es) + "}");
    });
    bool taken = post_door(e, group_->state_word());
    {
      std::lock_guard<std::mutex> lk(group_->mu);
      taken = taken && group_->in_kernel[static_cast<size_t>(gidx_)] != 0;
    }
    if (!taken) group_->ensure(this, gidx_, false, o_.timeout_s);
  } catch (...) {
    std::lock_guard<std::mutex> g(mu_);
    free_slots_.push_back(rec.slot);
    throw;
  }
  std::unique_lock<std::mutex> lk(mu_);
  last_round_ = round;
  st_.launches++;
  st_.group_rounds++;
  if (cold) st_.cold++;
  st_.bytes += static_cast<uint64_t>(n * es);
  q_.push_back(std::move(rec));
  q_len_.fetch_add(1, std::memory_order_release);
  lk.unlock();
  if (comp_sleeping_.load(std::memory_order_seq_cst)) cv_.notify_all();
}

std::string XgmiRoundPlane::debug_state() const {
  std::ostringstream os;
  os << "{\"res_seq\":" << res_seq_ << ",\"consumed\":" << rstate_[1] << ",\"solo_state\":" << rstate_[0]
     << ",\"res_on\":" << (res_on_ ? 1 : 0) << ",\"last_round\":" << last_round_ << ",\"queued\":" << q_len_.load()
     << ",\"configure_stage\":" << cfg_stage_.load() << ",\"group_teardown\":" << g_group_teardown.load();
  if (res_seq_ > 1) {
    const ResidentDoor* d = door_ + (res_seq_ - 1u) % kResidentDoors;
    os << ",\"door_last\":{\"seq\":" << d->seq << ",\"cmd\":" << d->cmd << ",\"epoch\":" << d->epoch << "}";
  }
  if (group_) {
    os << ",\"group\":{\"idx\":" << gidx_ << ",\"state\":" << group_->state_word()[0]
       << ",\"launched\":" << (group_->launched ? 1 : 0)
       << ",\"in_kernel\":" << static_cast<int>(group_->in_kernel[static_cast<size_t>(gidx_)]) << "}";
    uint64_t hb = 0;
    (void)hipMemcpy(&hb, group_->gdm, 8, hipMemcpyDeviceToHost);
    os << ",\"heartbeat\":" << hb;
  }
  uint64_t dm[10] = {};
  (void)hipMemcpy(dm, rdm_, sizeof(dm), hipMemcpyDeviceToHost);
  os << ",\"go\":[" << (dm[0] >> 32) << "," << (dm[0] & 0xffffffffu) << "],\"dm_epoch_cmd\":[" << (dm[8] & 0xffffffffu)
     << "," << (dm[8] >> 32) << "]";
  uint32_t ctl[16] = {};
  (void)hipMemcpy(ctl, ctl_mem_, sizeof(ctl), hipMemcpyDeviceToHost);
  os << ",\"ctl\":[";
  for (int i = 0; i < 16; ++i) os << (i ? "," : "") << ctl[i];
  os << "]}";
  (void)hipGetLastError();
  return os.str();
}

int XgmiRoundPlane::take_slot(std::unique_lock<std::mutex>& lk) {
  cv_idle_.wait(lk, [&] { return !free_slots_.empty(); });
  const int s = free_slots_.back();
  free_slots_.pop_back();
  return s;
}

bool XgmiRoundPlane::post_door(const ResidentDoor& e, const volatile uint32_t* state) {
  const volatile uint32_t* sw = state != nullptr ? state : rstate_;
  const uint32_t seq = res_seq_++;
  // the door slot is free once the kernel consumed the entry kResidentDoors before this one
  // (rounds in flight are bounded by the ring's slots, so this does not wait in practice)
  const auto t0 = std::chrono::steady_clock::now();
  while (static_cast<int32_t>(seq - static_cast<uint32_t>(kResidentDoors) - rstate_[1]) > 0 &&
         sw[0] != kResExited) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::duration<double>(2 * o_.timeout_s + 5))
      throw ProtocolError("xgmi plane: the resident round kernel stopped taking rounds");
    __builtin_ia32_pause();
  }
  ResidentDoor* d = door_ + seq % kResidentDoors;
  d->in = e.in;
  d->out = e.out;
  d->counts = e.counts;
  d->counts_host = e.counts_host;
  d->err_out = e.err_out;
  d->done_out = e.done_out;
  d->epoch = e.epoch;
  d->cmd = e.cmd;
  d->check = door_check(reinterpret_cast<const uint32_t*>(&e), seq);
  __atomic_store_n(&d->seq, seq, __ATOMIC_RELEASE);  // sequence word last
  // Dekker hand-off with the kernel's idle exit (xgmi_threshold.hip, resident_door): the
  // entry is visible before the state word is read
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  uint32_t st = sw[0];
  while (st == kResExiting) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::duration<double>(2 * o_.timeout_s + 5))
      throw ProtocolError("xgmi plane: the resident round kernel neither took nor refused a round");
    __builtin_ia32_pause();
    st = sw[0];
  }
  return st != kResExited;
}

void XgmiRoundPlane::park_resident() {
  if (!res_on_) return;
  res_on_ = false;
  st_.resident_parks++;
  ResidentDoor e{};
  e.cmd = kResStop;
  if (!post_door(e)) return;  // it had left already
  const auto t0 = std::chrono::steady_clock::now();
  while (rstate_[0] != kResExited) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::duration<double>(2 * o_.timeout_s + 5)) {
      MXAR_LOG(ERROR, "plane", "resident round kernel did not stop");
      return;
    }
    std::this_thread::yield();
  }
}

std::shared_ptr<void> XgmiRoundPlane::resident_out(size_t bytes, std::shared_ptr<std::atomic<bool>>* exported,
                                                    bool wait) {
  bytes = std::max<size_t>(bytes, 256);
  std::vector<void*> ptrs;
  {
    std::lock_guard<std::mutex> g(rel_->mu);
    if (rel_->bytes != bytes) return nullptr;
    ptrs.swap(rel_->ptrs);
  }
  if (!ptrs.empty()) {  // exported outputs: reusable behind what the default stream holds now
    hipEvent_t ev = nullptr;
    if (!rel_spare_.empty()) {
      ev = rel_spare_.back();
      rel_spare_.pop_back();
    } else {
      hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate(release)");
    }
    hip_check(hipEventRecord(ev, nullptr), "hipEventRecord(release)");
    rel_pend_.emplace_back(ev, std::move(ptrs));
  }
  while (!rel_pend_.empty()) {
    const hipError_t q = hipEventQuery(rel_pend_.front().first);
    if (q != hipSuccess) {
      (void)hipGetLastError();  // hipErrorNotReady is sticky-free, but keep the error state clean
      break;
    }
    std::lock_guard<std::mutex> g(rel_->mu);
    for (void* p : rel_pend_.front().second) rel_->free.push_back(p);
    rel_spare_.push_back(rel_pend_.front().first);
    rel_pend_.pop_front();
  }
  bool empty = false;
  {
    std::lock_guard<std::mutex> g(rel_->mu);
    empty = rel_->free.empty();
  }
  if (empty) {
    // Grow the pool with pool memory (hipMallocAsync) on the plane's idle allocation stream:
    // the kernel already running on the plane stream may use it once that stream has passed
    // the allocation - never a plain hipMalloc, whose later hipFreeAsync would fall back to a
    // device-wide synchronous free (the hazard for co-located planes' spinning kernels; ADVICE
    // r4). If the allocation stream does not get there within 100 us (it shares a hardware
    // queue with busy work), this round takes the launch path instead - no host wait on
    // another plane's kernel. reset_pool pre-grows resident-size pools, so this is rare.
    void* p = nullptr;
    if (alloc_stream_ == nullptr)
      hip_check(hipStreamCreateWithFlags(&alloc_stream_, hipStreamNonBlocking), "hipStreamCreate(plane alloc)");
    hip_check(hipMallocAsync(&p, bytes, alloc_stream_), "hipMallocAsync(plane output)");
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t q;
    while ((q = hipStreamQuery(alloc_stream_)) == hipErrorNotReady &&
           std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(100))
      __builtin_ia32_pause();
    (void)hipGetLastError();
    // a grouped worker has no launch path: it waits (the allocation stream has normal
    // priority, never behind the group kernel's queue)
    if (q == hipErrorNotReady && wait) q = hipStreamSynchronize(alloc_stream_);
    std::lock_guard<std::mutex> g(rel_->mu);
    rel_->free.push_back(p);  // usable by the launch path in any case (stream-ordered after it)
    st_.pool_grown++;
    if (q != hipSuccess) {
      st_.resident_pool_misses++;
      return nullptr;
    }
  }
  return out_buffer(bytes, exported);
}

bool XgmiRoundPlane::launch_resident(int round, const Payload& input, bool cold) {
  if (o_.resident_max <= 0 || o_.ring > kResidentDoors) return false;
  const int64_t n = cfg_.dataSize;
  const int64_t es = static_cast<int64_t>(dtype_size(o_.dtype));
  if (n * es > o_.resident_max) return false;
  const void* in_ptr = nullptr;
  if (!cold) {
    // only inputs the kernel can read now: device memory of this GPU, the plane's dtype, its
    // producer finished (the launch path orders the rest on the plane stream)
    auto* dp = input ? dynamic_cast<const DevicePayload*>(input.get()) : nullptr;
    // (a producer on the plane stream itself may be queued behind the resident kernel: that
    // input takes the launch path, which orders it on the stream)
    if (dp == nullptr || static_cast<int64_t>(dp->size()) != n || dp->device() != o_.device ||
        dp->dtype() != static_cast<int>(o_.dtype) || dp->stream() == stream_)
      return false;
    // a producer still running (e.g. the demo source's fill kernel) gets a short host wait:
    // a few microseconds for a round this small, cheaper than leaving the resident kernel
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      hipError_t q = hipSuccess;
      if (dp->ready()) q = hipEventQuery(static_cast<hipEvent_t>(dp->ready().get()));
      else if (dp->stream() && dp->stream() != stream_) q = hipStreamQuery(dp->stream());
      if (q == hipSuccess) break;
      (void)hipGetLastError();
      if (q != hipErrorNotReady || std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) return false;
      for (int i = 0; i < 16; ++i) __builtin_ia32_pause();
    }
    in_ptr = dp->bytes();
  }
  XgmiComm::RoundSpec spec;
  spec.block = block_;
  spec.chunk = chunk_;
  spec.order_ref = o_.order_ref;
  spec.host_force = hforce_dev_;
  spec.lag_wait_us = o_.lag_wait_us;
  spec.host_abort = hforce_dev_ + 1;
  if (o_.split) {  // a geometry that splits its chunks takes the launch path (plan_resident)
    spec.split_scratch = split_mem_;
    spec.split_bytes = split_bytes_;
  }
  if (!rplan_tried_) {
    rplan_tried_ = true;
    rplan_ = comm_->plan_resident(n, o_.dtype, cfg_.thReduce, cfg_.thComplete, spec, o_.resident_grid);
    // an optional resident kernel: without room in the device budget the rounds are launched
    res_token_.reset();
    if (rplan_.grid > 0) {
      res_token_ = Residency::get().try_reserve(o_.device, rplan_.grid,
                                                "resident kernel of worker " + std::to_string(cfg_.id));
      if (!res_token_) rplan_ = XgmiComm::ResidentPlan();
    }
  }
  if (rplan_.grid <= 0) return false;
  Rec rec;
  rec.out = resident_out(static_cast<size_t>(n * es), &rec.exported);
  if (!rec.out) return false;
  rec.round = round;
  rec.epoch = cfg_.epoch;
  rec.cold = cold;
  rec.round_epoch = epoch_of(round);
  if (!cold) rec.input = input;  // held until the round completed
  {
    std::unique_lock<std::mutex> lk(mu_);
    rec.slot = take_slot(lk);
  }
  int32_t* slot_dev = ring_dev_ + static_cast<size_t>(rec.slot) * ring_stride_;
  ResidentDoor e{};
  e.in = reinterpret_cast<uint64_t>(cold ? rec.out.get() : in_ptr);
  e.out = reinterpret_cast<uint64_t>(rec.out.get());
  e.counts = reinterpret_cast<uint64_t>(cnt_vram_ + static_cast<size_t>(rec.slot) * ring_stride_);
  e.counts_host = reinterpret_cast<uint64_t>(slot_dev);
  e.err_out = reinterpret_cast<uint64_t>(slot_dev + ring_stride_ - 1);
  e.done_out = reinterpret_cast<uint64_t>(slot_dev + ring_stride_ - 2);
  e.epoch = rec.round_epoch;
  e.cmd = cold ? kResCold : kResRound;
  {
    TraceScope span("plane", [&] {
      return std::make_pair(std::string(cold ? "resident cold round " : "resident round ") + std::to_string(round),
                            "{\"worker\":" + std::to_string(cfg_.id) + ",\"bytes\":" + std::to_string(n * es) + "}");
    });
    const uint32_t seq = res_seq_;
    bool taken = false;
    try {
      taken = res_on_ && post_door(e);
    } catch (...) {
      std::lock_guard<std::mutex> g(mu_);
      free_slots_.push_back(rec.slot);
      throw;
    }
    if (!taken) {
      // no kernel (first resident round, or it left after an idle spell): launch one that
      // starts at this entry
      if (!res_on_) {
        ResidentDoor* d = door_ + seq % kResidentDoors;
        *d = e;
        d->check = door_check(reinterpret_cast<const uint32_t*>(&e), seq);
        __atomic_store_n(&d->seq, seq, __ATOMIC_RELEASE);
        res_seq_ = seq + 1;
      }
      rstate_[1] = seq - 1u;
      rstate_[0] = kResRunning;
      __atomic_thread_fence(__ATOMIC_SEQ_CST);
      try {
        comm_->launch_resident(rplan_, door_dev_, rstate_dev_, rdm_, seq, g_res_gen.fetch_add(1) + 1u,
                               static_cast<uint64_t>(o_.resident_idle_us * 100.0), stream_);
      } catch (...) {
        std::lock_guard<std::mutex> g(mu_);
        free_slots_.push_back(rec.slot);
        throw;
      }
      res_on_ = true;
      st_.resident_launches++;
    }
  }
  std::unique_lock<std::mutex> lk(mu_);
  last_round_ = round;
  st_.launches++;
  st_.resident_rounds++;
  if (cold) st_.cold++;
  st_.bytes += static_cast<uint64_t>(n * es);
  q_.push_back(std::move(rec));
  q_len_.fetch_add(1, std::memory_order_release);
  lk.unlock();
  // the completion thread is polling for it unless it went to sleep (a futex wake costs the
  // launch path microseconds)
  if (comp_sleeping_.load(std::memory_order_seq_cst)) cv_.notify_all();
  return true;
}

void XgmiRoundPlane::launch(int round, const Payload& input, bool cold) {
  if (!configured_) throw ProtocolError("xgmi plane: launch before configure (InitWorkers)");
  if (orphaned_) throw ProtocolError("xgmi plane: its round memory was handed to a group kernel that never left");
  if (round != last_round_ + 1) throw ProtocolError("xgmi plane: rounds must be launched in order");
  hip_check(hipSetDevice(o_.device), "hipSetDevice");
  if (group_) {
    launch_group(round, input, cold);
    return;
  }
  if (launch_resident(round, input, cold)) return;
  park_resident();
  const int64_t n = cfg_.dataSize;
  const int64_t es = static_cast<int64_t>(dtype_size(o_.dtype));
  const int dcode = static_cast<int>(o_.dtype);
  Rec rec;
  rec.round = round;
  rec.epoch = cfg_.epoch;
  rec.cold = cold;
  flush_releases();
  rec.out = out_buffer(static_cast<size_t>(n * es), &rec.exported);
  {
    std::unique_lock<std::mutex> lk(mu_);
    rec.slot = take_slot(lk);
  }
  int32_t* slot_dev = ring_dev_ + static_cast<size_t>(rec.slot) * ring_stride_;
  const void* in_ptr = rec.out.get();  // a cold round reads no input
  if (!cold) {
    if (!input || static_cast<int64_t>(input->size()) != n) throw ProtocolError("xgmi plane: input must hold dataSize elements");
    auto* dp = dynamic_cast<const DevicePayload*>(input.get());
    if (dp != nullptr && dp->device() == o_.device) {
      if (dp->ready()) hip_check(hipStreamWaitEvent(stream_, static_cast<hipEvent_t>(dp->ready().get()), 0), "hipStreamWaitEvent");
      else if (dp->stream() && dp->stream() != stream_) hip_check(hipStreamSynchronize(dp->stream()), "hipStreamSynchronize");
      in_ptr = dp->bytes();  // any element alignment: the kernel takes unaligned units element-wise
      if (dp->dtype() != dcode) {  // cast into the plane's dtype on the device
        rec.staging = buffer(static_cast<size_t>(n * es));
        launch_cast(dp->bytes(), static_cast<DType>(dp->dtype()), rec.staging.get(), o_.dtype, n, stream_);
        in_ptr = rec.staging.get();
      }
      rec.input = input;  // held until the round completed
    } else {  // host (or other-device) float32 payload: upload, cast into the plane's dtype
      const std::vector<float> h = input->to_host();
      auto up = buffer(static_cast<size_t>(n * 4));
      hip_check(hipMemcpyAsync(up.get(), h.data(), n * 4, hipMemcpyHostToDevice, stream_), "hipMemcpyAsync H2D");
      hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");  // h is pageable and local
      if (o_.dtype == DType::F32) {
        rec.staging = up;
      } else {
        rec.staging = buffer(static_cast<size_t>(n * es));
        launch_cast(up.get(), DType::F32, rec.staging.get(), o_.dtype, n, stream_);
        rec.input = std::make_shared<DevicePayload>(up, 0, static_cast<size_t>(n), o_.device, nullptr);  // keep alive
      }
      in_ptr = rec.staging.get();
    }
  }
  XgmiComm::RoundSpec spec;
  spec.epoch = epoch_of(round);
  rec.round_epoch = spec.epoch;
  spec.block = block_;
  spec.chunk = chunk_;
  spec.cold = cold;
  spec.order_ref = o_.order_ref;
  spec.host_force = hforce_dev_;
  spec.lag_wait_us = o_.lag_wait_us;
  spec.host_abort = hforce_dev_ + 1;
  spec.err_out = reinterpret_cast<uint32_t*>(slot_dev + ring_stride_ - 1);
  spec.done_out = reinterpret_cast<uint32_t*>(slot_dev + ring_stride_ - 2);
  spec.counts_host = slot_dev;  // the kernel counts into HBM and copies once, at round end
  if (o_.split) {
    spec.split_scratch = split_mem_;
    spec.split_bytes = split_bytes_;
  }
  int32_t* cnt_dev = cnt_vram_ + static_cast<size_t>(rec.slot) * ring_stride_;
  {
    TraceScope span("plane", [&] {
      return std::make_pair(std::string(cold ? "cold round " : "round ") + std::to_string(round),
                            "{\"worker\":" + std::to_string(cfg_.id) + ",\"bytes\":" + std::to_string(n * es) + "}");
    });
    try {
      comm_->round(in_ptr, rec.out.get(), n, o_.dtype, stream_, cfg_.thReduce, cfg_.thComplete, cnt_dev, spec,
                   1.f);
    } catch (...) {
      std::lock_guard<std::mutex> g(mu_);
      free_slots_.push_back(rec.slot);
      throw;
    }
  }
  std::unique_lock<std::mutex> lk(mu_);
  rec.ev = events_[rec.slot];
  last_round_ = round;
  st_.launches++;
  if (cold) st_.cold++;
  st_.bytes += static_cast<uint64_t>(n * es);
  q_.push_back(std::move(rec));
  q_len_.fetch_add(1, std::memory_order_release);
  lk.unlock();
  // the completion thread is polling for it unless it went to sleep (a futex wake costs the
  // launch path microseconds)
  if (comp_sleeping_.load(std::memory_order_seq_cst)) cv_.notify_all();
}

void XgmiRoundPlane::force(int round) {
  if (!configured_ || round < cfg_.startRound) return;
  const int r = std::min(round, std::max(last_round_, cfg_.startRound));
  const uint32_t e = epoch_of(r);
  volatile uint32_t* w = hforce_;
  if (static_cast<int32_t>(e - *w) > 0) {
    *w = e;  // the kernel polls it (system-scope loads of coherent pinned memory)
    st_.forced++;
  }
}

void XgmiRoundPlane::abort(int round) {
  force(round);
  if (!configured_ || round < cfg_.startRound) return;
  const int r = std::min(round, std::max(last_round_, cfg_.startRound));
  const uint32_t e = epoch_of(r);
  volatile uint32_t* w = hforce_ + 1;
  if (static_cast<int32_t>(e - *w) > 0) *w = e;  // the kernel polls it at its lag gate
  // a grouped worker's posted rounds must run to be abandoned: with a co-located worker still
  // to join, no group kernel may be running - start one without it
  if (group_ && static_cast<int32_t>(res_seq_ - 1u - rstate_[1]) > 0) {
    try {
      group_->ensure(this, gidx_, true, o_.timeout_s);
    } catch (const std::exception& ex) {
      MXAR_LOG(ERROR, "plane", "abandoning rounds: " << ex.what());
    }
  }
}

void XgmiRoundPlane::drain() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_idle_.wait(lk, [&] { return q_.empty(); });
}

void XgmiRoundPlane::completion_loop() {
  // Past its spin budget this thread polls the done word with 20 us sleeps; the default 50 us
  // timer slack would stretch each one to ~70 us (Linux), i.e. a long round's completion seen
  // up to that much late.
  (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
  for (;;) {
    Rec rec;
    {
      // the next round is usually launched within microseconds: poll for it (the spin budget)
      // before sleeping on the condition variable
      const auto t_idle = std::chrono::steady_clock::now();
      const auto idle_budget = std::chrono::microseconds(o_.spin_us);
      for (unsigned i = 0; q_len_.load(std::memory_order_acquire) == 0; ++i) {
        if ((i & 63) == 0 && (stop_flag_.load(std::memory_order_relaxed) ||
                              std::chrono::steady_clock::now() - t_idle > idle_budget))
          break;
        __builtin_ia32_pause();
      }
      std::unique_lock<std::mutex> lk(mu_);
      comp_sleeping_.store(true, std::memory_order_seq_cst);
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      comp_sleeping_.store(false, std::memory_order_relaxed);
      if (q_.empty()) return;
      rec = q_.front();  // stays queued until its callback ran (drain waits for that)
    }
    hipError_t e;
    {
      TraceScope span("plane", [&] { return std::make_pair("wait r" + std::to_string(rec.round), std::string()); });
      // The kernel's last workgroup sets the slot's pinned done word to the round epoch once
      // every workgroup drained its stores (output, counts) and passed its ticket
      // (xgmi_threshold.hip, round end): that word IS the completion. Reading it is a plain
      // load of host memory - no runtime call, so this thread does not contend with the
      // workers' launches for the HIP runtime's locks, and no event is recorded per round.
      // The output's consumers are device work on this GPU, which reads the drained stores
      // through L2. Poll first (a blocking wait sleeps on an interrupt whose wake-up costs
      // tens of microseconds), then poll with short sleeps: the kernel bounds its own waits
      // (timeout_s), so a round that never writes the word is a lost kernel - reported as an
      // error after twice that long.
      const auto t0 = std::chrono::steady_clock::now();
      const auto budget = std::chrono::microseconds(o_.spin_us);
      const volatile uint32_t* done = reinterpret_cast<const volatile uint32_t*>(
          ring_ + static_cast<size_t>(rec.slot) * ring_stride_ + ring_stride_ - 2);
      const uint32_t want = static_cast<uint32_t>(rec.round_epoch);
      while (*done != want && std::chrono::steady_clock::now() - t0 < budget) {
        for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
      }
      e = hipSuccess;
      {  // (round 2 confirmed with a per-round event: +2-3 us of hipEventRecord per launch,
         // profiles/round3/api_cost.json; the pinned done word replaced it)
        const auto lost = std::chrono::microseconds(static_cast<int64_t>(2e6 * o_.timeout_s) + 5000000);
        while (*done != want) {
          if (std::chrono::steady_clock::now() - t0 > lost) {
            MXAR_LOG(ERROR, "plane", "round " << rec.round << " never signalled its completion word");
            e = hipErrorLaunchTimeOut;
            break;
          }
          std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        std::atomic_thread_fence(std::memory_order_acquire);  // counts / error word after the done word
      }
    }
    if (Tracer::get().enabled())
      trace_instant("plane", "done r" + std::to_string(rec.round), "{\"worker\":" + std::to_string(cfg_.id) + "}");
    RoundResult res;
    res.epoch = rec.epoch;
    res.round = rec.round;
    res.cold = rec.cold;
    const volatile int32_t* host = ring_ + static_cast<size_t>(rec.slot) * ring_stride_;
    const size_t nc = static_cast<size_t>(cfg_.peers) * nch_;
    // The kernel writes the counts and the error word after its last release, each tagged
    // with the round epoch (xgmi_threshold.hip host_tag), so they may land after the done
    // word: wait for every tag (PCIe writes in flight: microseconds at most).
    const uint32_t tag = static_cast<uint32_t>(rec.round_epoch) & 0xffffffu;
    auto tagged = [&](size_t i) { return (static_cast<uint32_t>(host[i]) >> 8) == tag; };
    if (e == hipSuccess) {
      const auto t_tag = std::chrono::steady_clock::now();
      for (size_t i = 0; i < nc || !tagged(ring_stride_ - 1);) {
        if (i < nc && tagged(i)) {
          ++i;
          continue;
        }
        if (std::chrono::steady_clock::now() - t_tag > std::chrono::seconds(1)) {
          MXAR_LOG(ERROR, "plane", "round " << rec.round << ": counts / error word never arrived");
          e = hipErrorLaunchTimeOut;
          break;
        }
        __builtin_ia32_pause();
      }
      std::atomic_thread_fence(std::memory_order_acquire);
    }
    auto cnt = [&](size_t i) { return static_cast<int32_t>(static_cast<uint32_t>(host[i]) & 0xffu); };
    if (coarse_ == 1) {
      res.count.resize(nc);
      for (size_t i = 0; i < nc; ++i) res.count[i] = cnt(i);
    } else {  // coarsened at thresholds 1: every reference chunk of a kernel chunk shares its count
      res.count.resize(static_cast<size_t>(cfg_.peers) * nch_ref_);
      for (int j = 0; j < cfg_.peers; ++j)
        for (int c = 0; c < nch_ref_; ++c)
          res.count[static_cast<size_t>(j) * nch_ref_ + c] = cnt(static_cast<size_t>(j) * nch_ + c / coarse_);
    }
    const uint32_t err = static_cast<uint32_t>(host[ring_stride_ - 1]) & 0xffu;
    res.error = (err & ~err_seen_) | (e != hipSuccess ? 0x80000000u : 0u);
    err_seen_ |= err;
    {
      auto dp = std::make_shared<DevicePayload>(rec.out, 0, static_cast<size_t>(cfg_.dataSize), o_.device, nullptr,
                                                nullptr, static_cast<int>(o_.dtype));
      dp->set_export_flag(rec.exported);
      res.data = std::move(dp);
    }
    rec.input.reset();
    rec.staging.reset();
    {
      std::lock_guard<std::mutex> g(done_mu_);
      if (done_) done_(std::move(res));
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      free_slots_.push_back(rec.slot);
      q_.pop_front();
      q_len_.fetch_sub(1, std::memory_order_relaxed);
      st_.completed++;
    }
    cv_idle_.notify_all();
  }
}

std::shared_ptr<XgmiRoundPlane> make_xgmi_plane(const XgmiPlaneOptions& o) {
  return std::make_shared<XgmiRoundPlane>(o);
}

}  // namespace mxar
