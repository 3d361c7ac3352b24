// XgmiRoundPlane: the MI355X data plane of the round-granular protocol engine
// (PlaneWorkerActor, csrc/runtime/plane_worker.h). One persistent threshold-kernel launch
// per allreduce round (csrc/hip/xgmi_threshold.hip) replaces the reference's per-chunk
// ScatterBlock / ReduceBlock messages (AllreduceWorker.scala:194-251) with direct xGMI
// peer stores into the owners' HBM slots.
//
//   * Arena: at construction the worker allocates ONE fine-grained HBM arena big enough for
//     any membership up to `max_peers` workers and `max_lag` (the largest slab layout of
//     XgmiComm over those), zeroes it once and exports it with hipIpcGetMemHandle. The
//     handle travels in the worker's registration (MemberUp.meta -> the master ->
//     InitWorkers.planes), so a worker maps its peers from InitWorkers alone.
//     Workers of one process find each other's arenas through a process-local registry
//     (IPC handles cannot be opened by their own process).
//   * configure (InitWorkers): the reference's block ranges (step = ceil(N / P), float32)
//     and maxChunkSize chunks; an XgmiComm is laid out over the arena (rows = maxLag + 1)
//     and connected to the peers' mapped arenas (mappings are kept across epochs).
//   * launch (StartAllreduce): input ordered after its producer (ready event, no host
//     sync), one threshold launch with the round's explicit epoch
//     (roundBase + r - startRound + 1), per-chunk counts and the error word copied to
//     pinned host memory, a completion event; a completion thread hands each finished
//     round to the worker in launch order.
//   * resident rounds (<= 4 MiB, XgmiPlaneOptions::resident_max): instead of one launch per
//     round, the round is written to a pinned door ring that a resident threshold kernel
//     polls (XgmiComm::launch_resident); the kernel leaves after an idle spell or when the
//     plane needs its stream (re-initialisation, an input that must be staged on the stream)
//     and the next round launches it again. Same round semantics, same done word.
//   * force (catch-up): raises a pinned host word the kernel polls; rounds <= it complete
//     with what has arrived. Peers ahead by more than maxLag force us through our slab.
//   * co-located workers (several workers of one job in this process on this GPU, e.g. a
//     PlaneJob): they form a PlaneGroup and every round of every one of them runs in ONE
//     resident kernel, a slice of workgroups per worker fed from that worker's door
//     (xgmi_threshold.hip threshold_group_resident_kernel). Each worker's rounds still run on
//     their own schedule (a straggler's slice lags, the others run ahead), and no worker's
//     round can wait in a hardware queue behind a co-located peer's spinning round - any number
//     of workers at any GPU_MAX_HW_QUEUES (>= 2).
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/round_plane.h"
#include "device_plane.h"
#include "xgmi_comm.h"

namespace mxar {

struct XgmiPlaneOptions {
  int device = 0;
  DType dtype = DType::F32;
  int64_t capacity = 0;  // elements per round (>= the job's dataSize)
  int max_peers = 8;     // largest membership the arena is sized for
  int max_lag = 4;       // largest maxLag the arena is sized for
  int grid = 0;          // workgroups per launch (0: 2 per CU; split when planes share a GPU)
  double timeout_s = 60.0;
  bool order_ref = true;  // the reference's arrival-order accounting (threshold kernel doc)
  int ring = 64;          // rounds in flight at most (pinned count / error slots)
  bool high_priority = true;  // plane stream priority (see XgmiRoundPlane ctor)
  bool order_release = true;  // a round output's release waits for the default stream (buffer())
  int spin_us = 1000;         // completion thread polls a round's event this long before blocking
  bool split = true;          // chunks fewer than workgroups are split over several (threshold kernel)
  // Smallest maxChunkSize (elements) that keeps one flag word, count and threshold decision
  // per reference chunk (DataBuffer.scala:12,28-29,69-75); 0 = 1 KiB of data per flag. Finer
  // chunks cost flag-table memory (3 x rows x P words per chunk). A job with a finer
  // maxChunkSize runs at thresholds 1 with chunks coarsened to the flag granularity (counts
  // reported per reference chunk), and is refused at thresholds < 1 (ProtocolError).
  int64_t min_chunk = 0;
  // Resident rounds of a lone worker (XgmiComm::launch_resident; co-located workers run every
  // round on their group kernel instead): rounds of at most this many bytes are posted
  // to a kernel that stays on the plane stream between rounds instead of one launch each
  // (0 = off; MXAR_PLANE_RESIDENT). The kernel leaves after `resident_idle_us` without a
  // round (MXAR_PLANE_RESIDENT_IDLE_US) and is launched again by the next one. Rounds whose
  // geometry needs more than 64 workgroups (MXAR_PLANE_RESIDENT_GRID) or split chunks are
  // launched. 2 workers, th 1, bench geometry: 256 KiB 38-47 -> 32-34 us, 1 MiB 44-45 ->
  // 34-40, 4 MiB 46-52 -> 42-47 per round (profiles/round4/resident_grid_ab.jsonl).
  int64_t resident_max = 4 << 20;
  // Lag skip (XgmiComm::RoundSpec::lag_wait_us): a round waits at most this long at its lag
  // gate for a peer still inside the round that last used the row, then runs without it
  // (writes nothing to it, forces it). < 0: wait for the peer - a straggler then holds every
  // fast worker within maxLag + 1 rounds of itself (bounded buffers). Applies only where
  // the thresholds let a round complete without one peer.
  double lag_wait_us = -1.0;
  // The owner reserved this plane's group-kernel workgroups in the device residency budget
  // (residency.h) already - PlaneJob does, for all its co-located planes at once, so a job that
  // cannot fit fails at construction. false: the group reserves them itself when it forms.
  bool residency_external = false;
  int resident_grid = 64;
  double resident_idle_us = 1000.0;
};

struct XgmiPlaneStats {
  uint64_t launches = 0, cold = 0, forced = 0, bytes = 0, completed = 0, coarsened = 0, peer_maps = 0;
  uint64_t pool_grown = 0;  // round outputs the pool had to allocate (none after warm-up in steady state)
  uint64_t resident_pool_misses = 0;  // resident-size rounds launched instead: pool growth not ready in time
  uint64_t resident_rounds = 0, resident_launches = 0, resident_parks = 0;
  uint64_t group_rounds = 0;   // rounds run by the co-located workers' group kernel
  uint64_t group_launches = 0;  // group kernels this worker launched
  int group_size = 0;          // co-located workers in the current membership (0: none / alone)
};

struct PlaneGroup;

class XgmiRoundPlane final : public RoundPlane {
 public:
  explicit XgmiRoundPlane(const XgmiPlaneOptions& o);
  ~XgmiRoundPlane() override;
  const char* name() const override { return "xgmi"; }
  std::string descriptor() const override { return desc_; }
  void set_done(DoneFn fn) override;
  void configure(const PlaneConfig& cfg) override;
  void launch(int round, const Payload& input, bool cold) override;
  void force(int round) override;
  void abort(int round) override;
  void drain() override;
  // chunks per block as the reference counts them (ceil(block / maxChunkSize)): the length of
  // an output's counts is peers x chunks()
  int chunks() const override { return nch_ref_; }

  const XgmiPlaneOptions& options() const { return o_; }
  const XgmiPlaneStats& stats() const { return st_; }
  hipStream_t stream() const { return stream_; }
  int64_t arena_bytes() const { return arena_bytes_; }
  int64_t chunk_elems() const { return chunk_; }
  int64_t block_elems() const { return block_; }
  XgmiComm* comm() const { return comm_.get(); }
  // Diagnostics (blocking copies of device words - never on a hot path): the door / resident
  // words, the group's state, the device go word and control words.
  std::string debug_state() const;
  // Phase-stamp buffer for this plane's round kernels (study knob, XgmiComm::set_phase_stamps);
  // kept across re-initialisations. Call between rounds.
  void set_phase_stamps(uint64_t* buf, int64_t slots) {
    park_resident();  // a resident kernel holds the old launch arguments
    rplan_tried_ = false;
    stamps_ = buf;
    stamp_slots_ = buf ? slots : 0;
    if (comm_) comm_->set_phase_stamps(stamps_, stamp_slots_);
  }

 private:
  bool coarsen_full_ = true;    // MXAR_PLANE_COARSEN=0: kernel chunks = maxChunkSize at thresholds 1
  int wg_chunks_ = 1;           // at thresholds 1: kernel chunks per workgroup at most (0: no cap)
  struct Rec {
    int round = 0;
    int64_t epoch = 0;
    std::shared_ptr<void> out, staging;
    std::shared_ptr<std::atomic<bool>> exported;  // the output's export flag (out_buffer)
    uint32_t round_epoch = 0;                      // the kernel's round epoch (done word)
    Payload input;
    hipEvent_t ev = nullptr;
    int slot = 0;
    bool cold = false;
  };
  uint32_t epoch_of(int round) const {
    return cfg_.roundBase + static_cast<uint32_t>(round - cfg_.startRound) + 1u;
  }
  char* map_peer(const std::string& desc);
  // Stream-ordered device buffer (hipMallocAsync on the plane stream, hipFreeAsync when the
  // last holder drops it): the launch path never calls a device-synchronising allocator
  // while a peer's kernel may be spinning on this worker's next launch.
  std::shared_ptr<void> buffer(size_t bytes, bool user_visible = false);
  // A round output from the plane's pool (no allocator call on the round path): released
  // to the pool directly, or - once exported to another stream (DevicePayload::
  // mark_exported) - at the next launch behind the default stream (flush_releases).
  std::shared_ptr<void> out_buffer(size_t bytes, std::shared_ptr<std::atomic<bool>>* exported);
  void reset_pool(size_t bytes);
  int take_slot(std::unique_lock<std::mutex>& lk);
  void completion_loop();
  // Resident rounds: post the round to the resident kernel (launching it if none runs);
  // false = the round needs the launch path (park_resident first).
  bool launch_resident(int round, const Payload& input, bool cold);
  // Writes door entry res_seq_ and hands it to the kernel; false = the kernel had exited
  // before it took the entry (nothing runs it). state: the kernel's state word (the group's
  // for a grouped worker; null = this plane's own).
  bool post_door(const ResidentDoor& e, const volatile uint32_t* state = nullptr);
  // Stops the resident kernel (a STOP entry behind the posted rounds) and waits for it to leave.
  void park_resident();
  // Co-located workers (PlaneGroup): join the group of this membership (configure), post a
  // round to the group kernel (every round of a grouped worker), leave the group (a STOP entry
  // for this worker's slice; configure / destruction).
  void join_group(const PlaneConfig& cfg);
  void launch_group(int round, const Payload& input, bool cold);
  void leave_group();
  friend struct PlaneGroup;
  // the workers of this membership in this process on this device: (rank, arena id)
  std::vector<std::pair<int, uint64_t>> colocated(const PlaneConfig& cfg) const;
  bool grouped_ = false;  // this membership has co-located workers (configure)
  // the group kernel never took this worker's STOP: its round memory went to the group
  // (PlaneGroup::orphans) and the plane can run no further round
  bool orphaned_ = false;
  // where configure() is (debug_state): 0 idle, 1 abandoning the old epoch's rounds, 2 draining
  // them, 3 leaving the old group (31-35: leave_group's steps), 4 parking a solo kernel, 5
  // mapping peers, 6 the new communicator and published progress, 7 joining the new group
  std::atomic<int> cfg_stage_{0};
  std::shared_ptr<PlaneGroup> group_;
  int gidx_ = -1;                      // this worker's index in the group
  XgmiComm::ResidentPlan gplan_;       // the group kernel's geometry for this membership

  XgmiPlaneOptions o_;
  char* arena_ = nullptr;
  int64_t arena_bytes_ = 0;
  int64_t flag_bytes_ = 0;  // flag table reserved at its largest size (every layout the same)
  int64_t flag_gran_ = 0;   // slot bytes per flag word (XgmiComm flag_gran)
  uint64_t arena_id_ = 0;
  std::string desc_;
  uint32_t* hforce_ = nullptr;      // pinned host words the engine raises: [0] force, [1] abort
  uint32_t* hforce_dev_ = nullptr;  // their device-visible address
  hipStream_t stream_ = nullptr;
  hipStream_t alloc_stream_ = nullptr;  // idle stream for resident-round output growth (resident_out)
  std::unique_ptr<XgmiComm> comm_;
  std::map<std::string, char*> mapped_;  // peer IPC handle -> mapping (kept across epochs)
  PlaneConfig cfg_;
  bool configured_ = false;
  int64_t block_ = 0, chunk_ = 0;
  int nch_ = 0;       // chunks per block the kernel runs
  int nch_ref_ = 0;   // reference chunks per block (= nch_ unless coarsened at thresholds 1)
  int coarse_ = 1;    // reference chunks per kernel chunk
  int last_round_ = -1;  // last launched round of this epoch
  // pinned ring: per slot P x nch counts + the error word
  int32_t* ring_ = nullptr;
  int32_t* ring_dev_ = nullptr;  // the ring's device-visible address
  uint32_t* ctl_mem_ = nullptr;  // the communicator's control words, kept across epochs
  void* split_mem_ = nullptr;    // split-chunk scratch, zeroed per membership
  size_t split_bytes_ = 16;
  int32_t* cnt_vram_ = nullptr;  // per-slot counts the workgroups write (HBM); copied into the ring at round end
  size_t ring_stride_ = 0;  // int32 per slot
  std::vector<int> free_slots_;
  uint32_t err_seen_ = 0;

  std::mutex mu_;
  std::condition_variable cv_, cv_idle_;
  std::deque<Rec> q_;
  std::atomic<int> q_len_{0};              // q_.size(), polled without the lock by the completion thread
  std::atomic<bool> comp_sleeping_{false};  // the completion thread waits on cv_ (launch must notify)
  std::atomic<bool> stop_flag_{false};
  bool stop_ = false;
  std::vector<hipEvent_t> events_;
  std::mutex done_mu_;
  DoneFn done_;
  std::thread th_;
  XgmiPlaneStats st_;
  uint64_t* stamps_ = nullptr;
  int64_t stamp_slots_ = 0;
  // Round outputs the sinks dropped, freed at the next launch behind one default-stream event
  // (work a sink queued on torch's default stream may still read them; see buffer()).
  struct ReleaseQ {
    std::mutex mu;
    std::vector<void*> ptrs;  // released after an export: reusable once behind the default stream
    std::vector<void*> free;  // reusable now (ordered on the plane stream)
    size_t bytes = 0;         // size of the pooled output buffers
  };
  std::shared_ptr<ReleaseQ> rel_ = std::make_shared<ReleaseQ>();
  hipEvent_t rel_ev_ = nullptr;
  void flush_releases();
  std::shared_ptr<bool> alive_ = std::make_shared<bool>(true);
  // resident rounds
  ResidentDoor* door_ = nullptr;       // pinned door ring (kResidentDoors entries)
  ResidentDoor* door_dev_ = nullptr;   // its device-visible address
  volatile uint32_t* rstate_ = nullptr;  // pinned: [0] kernel state, [1] last entry it consumed
  uint32_t* rstate_dev_ = nullptr;
  uint32_t* rdm_ = nullptr;            // the kernel's device words
  XgmiComm::ResidentPlan rplan_;
  bool rplan_tried_ = false;
  std::shared_ptr<void> res_token_;    // the resident kernel's share of the residency budget
  bool res_on_ = false;                // a resident kernel was launched and may still run
  uint32_t res_seq_ = 1;               // next door entry
  // exported outputs released while a resident kernel holds the plane stream: reusable once
  // an event recorded on the default stream behind them has completed (host query)
  std::deque<std::pair<hipEvent_t, std::vector<void*>>> rel_pend_;
  std::vector<hipEvent_t> rel_spare_;
  // a pooled round output for a resident round (grown with hipMalloc: nothing may queue on
  // the plane stream behind the resident kernel)
  // (wait: a grouped worker has no launch path - it waits for the pool's growth)
  std::shared_ptr<void> resident_out(size_t bytes, std::shared_ptr<std::atomic<bool>>* exported, bool wait = false);
};

std::shared_ptr<XgmiRoundPlane> make_xgmi_plane(const XgmiPlaneOptions& o);

}  // namespace mxar
