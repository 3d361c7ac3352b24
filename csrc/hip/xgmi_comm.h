// XgmiComm: one-process-per-GPU allreduce over directly mapped peer HBM (xGMI).
//
// This is the MI355X data plane of the reference's scatter/reduce/broadcast protocol
// (AllreduceWorker.scala:194-209 scatter, :240-251 reduce, :230-238 broadcast): a
// *direct* (one-hop, fully connected) reduce-scatter + all-gather, which on an 8-GPU
// xGMI mesh drives all 7 links of every GPU at once, where a ring drives 2.
//
//   ScatterBlock(chunk c of block j)  == rank r stores input[j][c] straight into rank j's
//                                        receive slot S_j[r][c] over xGMI, then sets
//                                        flag F1_j[r][c] = epoch
//   count == minRequired (th = 1)      == rank j sees F1_j[s][c] == epoch for every s
//   reduce + ReduceBlock broadcast     == rank j sums the P contributions in fp32 and
//                                        stores the result into every R_k[j][c], then
//                                        sets F2_k[j][c]
//   CompleteAllreduce / flush          == rank k waits on F2_k[*][c] and copies R_k into
//                                        the output (its own block is written directly)
//
// All three phases run inside ONE persistent launch per segment (no host round trip per
// chunk), every spin is bounded by a deadline, and epochs live in device memory so a
// launch can be captured into a hipGraph. Slabs are fine-grained device memory exported
// with hipIpcGetMemHandle; peers map them with hipIpcOpenMemHandle.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>
#include <memory>
#include <vector>

namespace mxar {

enum class DType : int { F32 = 0, BF16 = 1, F16 = 2 };
inline size_t dtype_size(DType d) { return d == DType::F32 ? 4 : 2; }

// Ring: fp32 partials on the reduce-scatter hops (rounded once); RingNative: partials in the
// element type (half the RS wire bytes for 16-bit types, one rounding per hop).
enum class Algo : int { Auto = 0, TwoShot = 1, OneShot = 2, Ring = 3, LL = 4, RingNative = 5 };

// The reference's two allreduce phases as collectives of their own (xgmi_coll.hip).
enum class Coll : int { AllToAll = 0, AllGather = 1, ReduceScatter = 2 };

// AdamW hyper-parameters of one fused step (PyTorch AdamW semantics; step counts from 1).
struct AdamW {
  float lr = 1e-3f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, weight_decay = 0.f;
  int step = 1;
};
// Per-rank fp32 shard state for the fused step: master params, exp_avg, exp_avg_sq, each
// holding the rank's own block (block r of the flat tensor, ceil(n / P) rounded to 16 B).
struct AdamShard {
  float* param = nullptr;
  float* exp_avg = nullptr;
  float* exp_avg_sq = nullptr;
};

constexpr int kMaxRanks = 16;
// threshold kernel one-shot body: ranks at most (its per-source registers; larger memberships
// take the two-shot body)
constexpr int kOneshotRanks = 8;
// Threshold kernel: gather units (chunk x peer) one workgroup may own (its pending bitmap in
// LDS), and reduce chunks per workgroup with a launch snapshot (reference arrival order).
constexpr int kThresholdGatherUnits = 4096;
constexpr int kThresholdSnapChunks = 2048;
constexpr int kCommThreads = 256;

// Resident rounds (xgmi_threshold.hip threshold_resident_kernel; xgmi_plane.cc): the host
// posts each round as one 64-B entry of a door ring in pinned host memory, the sequence word
// written last; a kernel that stays on the GPU between rounds runs them.
struct ResidentDoor {
  uint64_t in, out, counts, counts_host, err_out, done_out;  // device-visible addresses
  uint32_t epoch;
  int32_t cmd;  // kResRound / kResCold / kResStop
  uint32_t seq;
  uint32_t check;  // door_check(entry): the kernel reads the whole entry in one 64-B load and
                   // takes it only when the check matches (no second read after the sequence word)
};
constexpr int kResidentDoors = 64;
// A mix of the entry's words and its sequence number (host and device compute the same).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t door_check(const uint32_t* w14, uint32_t seq) {
  uint32_t h = seq * 0x9E3779B1u + 0x7F4A7C15u;
  for (int i = 0; i < 14; ++i) {
    h = (h ^ w14[i]) * 0x85EBCA6Bu;
    h ^= h >> 13;
  }
  return h ^ (h >> 16);
}
enum : int32_t { kResRound = 0, kResCold = 1, kResStop = 2 };
// host state words the kernel writes: [0] kResRunning / kResExiting / kResExited, [1] the
// last entry it consumed (its door slot may be reused)
enum : uint32_t { kResRunning = 0, kResExiting = 1, kResExited = 2 };

// Group resident rounds (xgmi_threshold.hip threshold_group_resident_kernel; xgmi_plane.cc
// PlaneGroup): the co-located workers of one job share ONE resident kernel, a slice of
// workgroups per worker, each fed from that worker's own door ring by a dispatcher wave.
struct GroupResidentMember {
  const ResidentDoor* door;  // the worker's pinned door ring (device-visible address)
  uint32_t* hstate;          // its pinned words: [1] the last entry consumed
  uint64_t* dm;              // its device words: [0] go, [2..9] the entry handed to its slice
  const uint32_t* hforce;    // its pinned force / abort words
  const uint32_t* habort;
  uint64_t* stamps;          // its phase-stamp buffer (study knob; null = off)
  uint64_t* split_dec;       // its split-chunk scratch (RoundSpec::split_scratch; null = unsplit)
  uint32_t* split_ctr;
  uint32_t* split_early;
  uint32_t seq0;             // the first entry this launch takes
  int rank;
};

// The launch-size grid rule (XgmiComm::launch_grid; profiles/round4/README.md section 9):
// workgroups for a launch moving `bytes` of input over all its ranks at device grid `grid`.
// Two-shot style: one per 64 KiB, 64..`cap`, the full grid from `full_at`; one-shot: every
// rank reads all `world` inputs, so one per 64 KiB of world x bytes, 64..the full grid.
inline int size_grid_rule(int64_t bytes, int grid, int world, bool oneshot, int64_t full_at = int64_t{512} << 20,
                          int64_t cap = 256) {
  if (oneshot) bytes *= (world > 1 ? world : 1);
  else if (bytes >= full_at) return grid;
  int64_t g = bytes / (int64_t{64} << 10);
  const int64_t hi = oneshot ? grid : cap;
  g = g < 64 ? 64 : (g > hi ? hi : g);
  return static_cast<int>(g < grid ? g : grid);
}

// Workgroups per rank at most when `ranks_here` logical ranks share one launch at the default
// grid (XgmiComm::shared_launch_cap): a quarter of that grid, half the CUs. 0 = no cap.
inline int shared_launch_rule(int ranks_here, int default_grid) {
  return ranks_here <= 1 ? 0 : (default_grid / 4 > 1 ? default_grid / 4 : 1);
}

struct CommStats {
  uint64_t calls = 0, launches = 0, bytes = 0, oneshot = 0, twoshot = 0, ring = 0, threshold = 0, ll = 0, coll = 0,
           adamw = 0, stream_switches = 0;
};

class XgmiComm {
 public:
  // slot_bytes: capacity of one receive slot (one block of one peer). A two-shot launch
  // reduces up to world * slot_bytes bytes, a one-shot launch up to slot_bytes bytes;
  // larger tensors are processed in segments. Memory per GPU ~ 2 * world * slot_bytes.
  // threshold_rows: depth of the lag ring of S/R slots used by allreduce_threshold
  // (maxLag + 1; 0 = threshold rounds disabled). The other algorithms use row 0.
  // Memory per GPU ~ 2 * (1 + threshold_rows) * world * slot_bytes.
  // external_slab: lay the communicator out over an arena the caller allocated (fine-grained,
  // zeroed once, >= layout(...).slab_bytes; xgmi_plane.cc) instead of allocating one.
  // min_flag_bytes: reserve at least this much for the flag table (an arena reused by
  // layouts of different sizes keeps its flags at the same place: data never lands on a flag).
  // external_slab / external_ctl: an arena and 256 B of control words owned by the caller
  // (xgmi_plane.cc). With both, construction and destruction make NO device-synchronising
  // call (no hipMalloc / hipFree / hipMemset / hipDeviceSynchronize): a plane re-lays its
  // arena out while a peer's round kernel may be spinning on this worker; the caller
  // resets the control words stream-ordered (hipMemsetAsync) before the first launch.
  // flag_gran: slot bytes per flag word (0 = min_chunk_bytes(), 1 KiB). The protocol plane
  // passes its maxChunkSize in bytes when chunks are finer, so that every reference chunk
  // keeps a flag, a count and a threshold decision of its own (xgmi_plane.cc).
  XgmiComm(int rank, int world, int device, int64_t slot_bytes, int grid = 0, double timeout_s = 20.0,
           int threshold_rows = 0, char* external_slab = nullptr, int64_t external_bytes = 0,
           int64_t min_flag_bytes = 0, uint32_t* external_ctl = nullptr, int64_t flag_gran = 0);
  ~XgmiComm();
  XgmiComm(const XgmiComm&) = delete;
  XgmiComm& operator=(const XgmiComm&) = delete;

  // 64-byte hipIpcMemHandle of this rank's slab.
  std::string ipc_handle() const;
  // handles[k] = ipc_handle() of rank k (own entry ignored).
  void connect(const std::vector<std::string>& handles);
  // Single-process mode: all "ranks" are this process (tests / P logical ranks).
  void connect_local(const std::vector<XgmiComm*>& comms);
  // Peer slab bases already mapped by the caller (the protocol plane keeps its own IPC
  // mappings across re-initialisations); own entry ignored.
  void connect_ptrs(const std::vector<char*>& bases);

  // Slab geometry for (world, slot_bytes, threshold_rows), without allocating.
  struct Layout {
    int64_t slot_bytes = 0, slot_stride = 0, maxch = 0, off_S = 0, off_R = 0, off_LL = 0, ll_max = 0, ll_slot = 0;
    int64_t slab_bytes = 0, alloc_bytes = 0;
  };
  static Layout layout(int world, int64_t slot_bytes, int threshold_rows, int64_t min_flag_bytes = 0,
                       int64_t flag_gran = 0);
  // Bytes of the flag table alone (the part of off_S before its 64 KiB rounding).
  static int64_t flag_bytes(int world, int64_t slot_bytes, int threshold_rows, int64_t flag_gran = 0);
  // Tell every peer that this rank has finished every threshold round up to `value`
  // (progress words; enqueued on `stream`). The protocol plane publishes its round base
  // after draining an old membership epoch, which opens the peers' lag gates for the new
  // epoch's first rounds only once no old-epoch round of this rank can still write.
  void publish_progress(uint32_t value, hipStream_t stream);
  // An allocation size hipIpcOpenMemHandle can map on this ROCm stack (see the constructor).
  static int64_t ipc_safe_bytes(int64_t bytes);

  // out = scale * sum over ranks of in (n elements of dtype); in == out allowed (in-place).
  // The scale is applied to the fp32 sum before the single rounding (scale = 1/P: mean).
  // Pointers must be 16-byte aligned. Enqueued on `stream`; returns immediately.
  void allreduce(const void* in, void* out, int64_t n, DType dt, hipStream_t stream, Algo algo = Algo::Auto,
                 float scale = 1.f);
  // The kernel a call of `algo` (Auto included) over n elements runs - the one place the
  // automatic dispatch is decided (allreduce() and the bench's latency table both use it).
  // ranks_in_launch: logical ranks of this device served by one launch (LocalCluster).
  Algo resolve(int64_t n, DType dt, Algo algo, int ranks_in_launch = 1) const;
  // Straggler-tolerant round (xgmi_threshold.hip): a chunk is reduced once
  // f32((th_reduce * P)) contributions are in, the round completes once
  // f32(th_complete * P * nch) reduced chunks are in (missing ones -> zeros, count 0), and
  // ranks run at most rows-1 rounds apart. counts (optional, int32 [P][nch], device) receives
  // the number of contributions summed per output chunk. The tensor must fit one launch
  // (n * dtype <= world * slot_bytes); nch = threshold_chunks(n, dt). rescale: a chunk
  // reduced from cnt < P contributions is multiplied by P / cnt before the rounding, i.e.
  // the sum is extrapolated from the contributions that made it (with scale = 1/P: the mean
  // over the contributors) - the reference leaves partial sums unscaled.
  void allreduce_threshold(const void* in, void* out, int64_t n, DType dt, hipStream_t stream, float th_reduce,
                           float th_complete, int32_t* counts = nullptr, float scale = 1.f, bool rescale = false);
  static void allreduce_threshold_local(const std::vector<XgmiComm*>& comms, const std::vector<const void*>& ins,
                                        const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream,
                                        float th_reduce, float th_complete, int32_t* counts = nullptr,
                                        float scale = 1.f, bool rescale = false);
  // One round of the protocol engine (xgmi_plane.cc) on the threshold kernel: explicit round
  // epoch and geometry (the reference's block ranges and maxChunkSize), the reference's
  // arrival-order accounting, a cold (force-completed, never started) round, and the pinned
  // host word the engine raises to force-complete rounds on a catch-up.
  struct RoundSpec {
    uint32_t epoch = 0;            // 0: this communicator's own threshold-round count + 1
    int64_t block = 0, chunk = 0;  // elements; 0: the kernel's own geometry
    bool cold = false;
    bool order_ref = false;
    const uint32_t* host_force = nullptr;  // device-visible pinned host word (may be null)
    const uint32_t* host_abort = nullptr;  // rounds <= this epoch are abandoned (may be null)
    uint32_t* err_out = nullptr;           // device-visible word the round's error word is copied to
    // device-visible pinned word the round's last workgroup sets to the round epoch once every
    // workgroup is done (a completion HINT for the host: it still confirms with the event)
    uint32_t* done_out = nullptr;
    int32_t* counts_host = nullptr;        // device-visible pinned copy of `counts`, written at round end
    // the rank's scratch for split chunks (zeroed per membership; split_scratch_bytes(P));
    // null: one workgroup per chunk
    void* split_scratch = nullptr;
    size_t split_bytes = 0;
    // lag skip (CommArgs::lag_skip): wait at most this long at the lag gate for a peer, then
    // skip it for the round; < 0 = wait for it. Taken only where it is safe and useful: unsplit
    // chunks and thresholds that let a round complete without one peer.
    double lag_wait_us = -1.0;
  };
  // Scratch a round of P ranks needs to split its chunks over several workgroups.
  static size_t split_scratch_bytes(int P, int64_t maxch) {
    return static_cast<size_t>(maxch) * (static_cast<size_t>(P + 1) * 12 + static_cast<size_t>(P) * 4);
  }
  int64_t max_chunks() const { return maxch_; }
  uintptr_t slab_address() const { return reinterpret_cast<uintptr_t>(slab_); }  // study: placement
  // Launch-size grids at the default grid (launch_grid); false: the full grid ("algo@full").
  bool size_grid() const { return size_grid_; }
  void set_size_grid(bool on) { size_grid_ = on; }
  // Resident rounds: round()'s geometry for n elements computed once (plan_resident; grid 0
  // = the round does not fit a resident kernel: chunks split over workgroups, or more than
  // `max_grid` workgroups), and a kernel on `stream` that runs the rounds posted to `door`
  // from entry `seq` on (launch_resident; hstate / dm: the state words above, and 32 device
  // words of scratch). Per-round operands come from the entries, not from `spec`.
  struct ResidentPlan {
    std::shared_ptr<void> args;  // the kernel's CommArgs
    int grid = 0;
    DType dt = DType::F32;
    int64_t n = 0;
  };
  // allow_split: a plane group's kernel also runs geometries that split their chunks (a lone
  // worker launches those)
  ResidentPlan plan_resident(int64_t n, DType dt, float th_reduce, float th_complete, const RoundSpec& spec,
                             int max_grid, bool allow_split = false) const;
  void launch_resident(const ResidentPlan& p, const ResidentDoor* door, uint32_t* hstate, uint32_t* dm,
                       uint32_t seq, uint32_t gen, uint64_t idle_ticks, hipStream_t stream);
  void round(const void* in, void* out, int64_t n, DType dt, hipStream_t stream, float th_reduce, float th_complete,
             int32_t* counts, const RoundSpec& spec, float scale = 1.f);
  // A plane group's resident kernel (xgmi_threshold.hip threshold_group_resident_kernel): ONE
  // launch serves the co-located workers `comms` (their plan_resident plans, one geometry),
  // members[k] = worker k's door, words and first entry; gstate: the group's pinned state
  // word, gdm: 8 device words of the group.
  static void launch_group_resident(const std::vector<XgmiComm*>& comms, const std::vector<const ResidentPlan*>& plans,
                                    const std::vector<GroupResidentMember>& members, uint32_t* gstate, uint64_t* gdm,
                                    uint32_t gen, uint64_t idle_ticks, hipStream_t stream);
  // Workgroups a round launch of `nch` chunks per block uses (counts / geometry checks).
  int round_grid(int nch) const;
  // Workgroups per rank at most when several ranks share one launch (default grid only).
  int shared_launch_cap(int ranks_here) const;
  // Chunks per block the threshold kernel uses for n elements (size of `counts` = P * this).
  int threshold_chunks(int64_t n, DType dt, int ranks_in_launch = 1) const;
  // Test knob: rank `rank` idles `us` microseconds at the start of each threshold launch.
  void set_straggler(int rank, double us) {
    delay_rank_ = rank;
    delay_us_ = us;
  }
  // Test knob: rank `rank` idles `us` microseconds before the slab-reading phase of every
  // one-shot / two-shot / collective launch (a slow reader for the slot-reuse guard tests).
  void set_read_delay(int rank, double us) {
    rdelay_rank_ = rank;
    rdelay_us_ = us;
  }
  // Test knob: rank `rank` idles `us` microseconds before the ring's last all-gather forward
  // of every ring launch (its late flag races the next kernel's flags: flag-ownership test).
  void set_forward_delay(int rank, double us) {
    fdelay_rank_ = rank;
    fdelay_us_ = us;
  }
  // Device-side barrier over all ranks (enqueued on `stream`).
  void barrier(hipStream_t stream);

  // xGMI bring-up probes (xgmi_probe.hip; bench.py `xgmi_links`), for collective quiet points
  // only (every rank idle). probe_push: `bytes` of `src` written through into the S slot (row
  // 0, column rank()) of every peer in `peer_mask`, one launch, `grid` workgroups per peer -
  // the scatter's store path, no flags. probe_pingpong: `iters` flag round trips with `peer`
  // (both ranks call it concurrently with the same iters / nonce; the lower rank leads and
  // writes the elapsed 100 MHz ticks to out[0], 0 on timeout); `fenced` adds the kernels'
  // release / acquire around each hand-off.
  // mode 0: the write-through pushes above; 1: plain stores into the peers' COARSE-grained
  // probe buffers (probe_coarse_handle / probe_coarse_connect) and one system release per
  // workgroup at the end - the other memory kind and store path a two-shot could use; 2: PULL,
  // this rank loading the peers' S slots (fine-grained, remote loads) into `src` (scratch).
  int64_t probe_max_bytes() const;
  void probe_push(const void* src, int64_t bytes, uint32_t peer_mask, int grid, hipStream_t stream, int mode = 0);
  // the coarse-grained probe buffer (probe_max_bytes, allocated on the first call): IPC handle
  // for the peers, and the peers' handles (collective, like connect)
  std::string probe_coarse_handle();
  void probe_coarse_connect(const std::vector<std::string>& handles);
  void probe_pingpong(int peer, int iters, uint32_t nonce, bool fenced, uint64_t* out, hipStream_t stream);

  // Fused data-parallel step (xgmi_adam.hip): grads [n] of every rank are reduce-scattered
  // (x scale, fp32), the owner applies AdamW to its shard state, and the updated parameters
  // are all-gathered into `params` [n] (identical on every rank). One launch; n * dtype must
  // fit one segment (<= world * slot_bytes). shard_len() = elements of this rank's block.
  void step_adamw(const void* grads, void* params, int64_t n, DType dt, hipStream_t stream, const AdamShard& st,
                  const AdamW& h, float scale);
  static void step_adamw_local(const std::vector<XgmiComm*>& comms, const std::vector<const void*>& grads,
                               const std::vector<void*>& params, int64_t n, DType dt, hipStream_t stream,
                               const std::vector<AdamShard>& st, const AdamW& h, float scale);
  int64_t block_elems(int64_t n, DType dt) const;

  // Collectives on [P][m] buffers (m elements per block, m * dtype a multiple of 16 B):
  //   AllToAll      in[P][m] -> out[P][m]   out_r[s] = in_s[r]
  //   AllGather     in[m]    -> out[P][m]   out_r[s] = in_s
  //   ReduceScatter in[P][m] -> out[m]      out_r = scale * sum_s in_s[r]
  // in and out must not overlap. One launch per segment of slot_bytes per block.
  void collective(Coll op, const void* in, void* out, int64_t m, DType dt, hipStream_t stream, float scale = 1.f);
  static void collective_local(const std::vector<XgmiComm*>& comms, Coll op, const std::vector<const void*>& ins,
                               const std::vector<void*>& outs, int64_t m, DType dt, hipStream_t stream,
                               float scale = 1.f);

  // Single-process cluster: ONE launch on `stream` runs every rank of `comms` (all on
  // one device, consecutive ranks, connected with connect_local); blockIdx.y = rank.
  static void allreduce_local(const std::vector<XgmiComm*>& comms, const std::vector<const void*>& ins,
                              const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream,
                              Algo algo = Algo::Auto, float scale = 1.f);
  static void barrier_group(const std::vector<XgmiComm*>& comms, hipStream_t stream);

  // Sticky device error word (ORed codes, see device_common.h); 0 = healthy.
  uint32_t error() const;
  // diagnostics: the control words ([0] launch epoch, [1] ticket, [2] error, [4] threshold
  // round epoch, ...), read with a blocking copy - for error reports, never on a hot path
  std::vector<uint32_t> ctl_words() const;
  void clear_error();
  // Zero this rank's flags, LL slots and counters (recovery after CommError; collective use
  // only, with every rank idle - see XgmiCommunicator.reset).
  void reset_local();
  // One-rank traffic rehearsal (benchmarks/sections.py dp_overlap): mark every flag word peers
  // would write into THIS rank's slab as reached for the next 2^30 epochs, so this rank's
  // two-shot runs alone - reading its input, pushing into the (local, never launched) peers'
  // slots, reducing its own S slots and gathering its own R slots - and moves exactly one
  // rank's HBM bytes of a real P-rank two-shot without waiting. Never for real collectives.
  void arm_solo_rehearsal();

  int rank() const { return rank_; }
  int threshold_rows() const { return rows_ - 1; }
  int world() const { return world_; }
  int device() const { return device_; }
  int grid() const { return grid_; }
  int64_t slot_bytes() const { return slot_bytes_; }
  int64_t oneshot_max_bytes() const { return oneshot_max_; }
  void set_oneshot_max_bytes(int64_t b) { oneshot_max_ = b; }
  int64_t ll_auto_max_bytes() const { return ll_auto_max_; }
  void set_ll_auto_max_bytes(int64_t b) { ll_auto_max_ = b; }
  // Largest tensor (bytes) one low-latency launch carries (Algo::LL; larger ones run in
  // segments). Fixed at construction: the LL slots are sized for it (MXAR_LL_MAX).
  int64_t ll_max_bytes() const { return ll_max_; }
  void set_grid(int g);
  void set_timeout(double s) { timeout_s_ = s; }
  // bit0: system-scope release fence (buffer_wbl2 sc0 sc1) before each flag store,
  // bit1: system-scope acquire after each wait. Default 3 (memory-model correct). A
  // drained write-through store is only known to have reached the producer's L2; without
  // the release the flag can reach memory first through another L2 channel (observed on
  // MI355X: stale slab reads). All kernel stores are write-through, so the release finds
  // no dirty lines and stays cheap. 2 exists only to measure the fence's cost.
  int fence() const { return fence_; }
  int units_per_wg() const { return units_per_wg_; }
  void set_units_per_wg(int u) { units_per_wg_ = u > 0 ? u : 0; }
  int ring_depth() const { return ring_depth_; }
  void set_ring_depth(int d) { ring_depth_ = d > 0 ? d : 1; }
  void set_fence(int f) { fence_ = f & 3; }
  // Study knob: per-workgroup phase stamps of the two-shot / ring kernels (xgmi_device.h
  // PhaseStamps) into `buf` (device, >= slots x 8 u64; slots = workgroups x ranks in the
  // launch); nullptr turns it off. Only the first rank of a grouped launch's buffer counts.
  void set_phase_stamps(uint64_t* buf, int64_t slots) {
    stamps_ = buf;
    stamp_slots_ = buf ? slots : 0;
  }
  bool connected() const { return connected_; }
  const CommStats& stats() const { return stats_; }
  char* slab() const { return slab_; }
  uint32_t* ctl_ptr() const { return ctl_; }  // device control words ([2] = error word)
  int64_t slab_bytes() const { return slab_bytes_; }
  int64_t alloc_bytes() const { return alloc_bytes_; }
  static int64_t min_chunk_bytes() { return 1024; }

 private:
  // Stream safety: every launch of a communicator reads its epoch / slab rows from device
  // state the previous launch left behind, so launches must run one after the other even
  // when callers use different streams (e.g. the DP reducer's comm stream and user code on
  // the default stream). When `s` differs from the stream of this communicator's previous
  // launch, an event recorded on that stream NOW (it covers the previous launch) is waited
  // on by `s`. Same stream: nothing to do, no per-call event.
  static void order_group(const std::vector<XgmiComm*>& group, hipStream_t s);
  void order_after_last(hipStream_t s);

  static void run(const std::vector<XgmiComm*>& group, const std::vector<const void*>& ins,
                  const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream, Algo algo, float scale);
  static void launch_segment(const std::vector<XgmiComm*>& group, const char* const* ins, char* const* outs,
                             int64_t n, DType dt, hipStream_t stream, Algo kind, float scale,
                             const std::vector<AdamShard>* adam_state = nullptr, const AdamW* adam = nullptr);

  static void run_coll(const std::vector<XgmiComm*>& group, Coll op, const std::vector<const void*>& ins,
                       const std::vector<void*>& outs, int64_t m, DType dt, hipStream_t stream, float scale);
  // run_threshold's launch arguments and grid (no launch); false: nothing to do (n <= 0)
  static bool threshold_args(const std::vector<XgmiComm*>& group, const std::vector<const void*>& ins,
                             const std::vector<void*>& outs, int64_t n, DType dt, float thr, float thc,
                             int32_t* counts, float scale, bool rescale, const RoundSpec* spec, void* args, int* gx);
  static void run_threshold(const std::vector<XgmiComm*>& group, const std::vector<const void*>& ins,
                            const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream, float thr,
                            float thc, int32_t* counts, float scale, bool rescale, const RoundSpec* spec = nullptr);
  void geometry_threshold(int64_t n, DType dt, int ranks_here, int64_t* block, int64_t* chunk, int* nch,
                          int* gx) const;

  int rank_, world_, device_, grid_, rows_;
  char* probe_coarse_ = nullptr;  // this rank's coarse-grained probe buffer (xgmi_probe.hip)
  std::vector<char*> probe_peers_;  // the peers' coarse probe buffers, IPC-mapped
  int64_t slot_bytes_, slot_stride_, maxch_, off_S_, off_R_, off_B_, slab_bytes_;
  int64_t ll_max_ = 0, ll_slot_ = 0, off_LL_ = 0;
  int64_t alloc_bytes_ = 0;  // slab_bytes_ padded around the IPC size bug (constructor)
  int delay_rank_ = -1;
  double delay_us_ = 0;
  int rdelay_rank_ = -1;
  double rdelay_us_ = 0;
  int fdelay_rank_ = -1;
  double fdelay_us_ = 0;
  int64_t oneshot_max_;
  int64_t ll_auto_max_ = 0;  // Auto picks the low-latency one-shot up to this many bytes
  double timeout_s_;
  int fence_ = 3;
  uint64_t* stamps_ = nullptr;  // phase-stamp buffer (study knob, set_phase_stamps)
  int64_t stamp_slots_ = 0;
  int units_per_wg_ = 0;  // two-shot scatter units per workgroup; 0 = by block size (launch_segment)
  int sub_max_ = 0;       // two-shot: most reduce pieces per chunk; 0 = by block size
  int ring_depth_ = 1;    // ring: chunks per workgroup, walked step-major (MXAR_RING_DEPTH)
  int ring_grid_ = 256;
  // The device-default grid, and whether a launch at the default grid sizes it by its bytes
  // (launch_grid; MXAR_SIZE_GRID=0: always the full grid). An explicit grid (set_grid(g),
  // tune()'s "algo@g" labels) is always used as given.
  int default_grid_ = 0;
  bool size_grid_ = true;
  int launch_grid(int64_t bytes_in_launch, bool oneshot, int64_t full_at = int64_t{512} << 20) const;
  char* slab_ = nullptr;            // own fine-grained slab (flags | S | R | LL)
  uint32_t* ctl_ = nullptr;         // [0] epoch, [1] ticket, [2] sticky error (device memory)
  char* peers_[kMaxRanks] = {};     // slab base of every rank (own included)
  bool ipc_opened_[kMaxRanks] = {};
  bool connected_ = false;
  bool own_slab_ = true;           // false: laid out over a caller's arena
  bool own_ctl_ = true;            // false: control words owned by the caller
  bool noguard_ = false;           // MXAR_SLOT_GUARD=0 (study / negative control only)
  bool no_gate_shortcut_ = false;  // MXAR_STUDY=1 MXAR_GATE_SHORTCUT=0: threshold lag gate always polled (A/B)
  // full-threshold rounds of at most this many bytes per rank run the one-shot body
  // (xgmi_threshold.hip; MXAR_STUDY=1 MXAR_TH_ONESHOT_MAX=bytes, 0 = off): 1.1-1.8x faster
  // than the two-shot body at 64-256 KiB (profiles/round6 section 12). The multi-process
  // failures of a first 256 KiB default came from workgroups past the fast pass; the host now
  // sizes the grid for it or takes the two-shot body (threshold_args)
  int64_t th_oneshot_max_ = 256 << 10;
  bool ring_hop_rows_ = false;     // negative control: the two-writer ring flag layout (MXAR_RING_FLAGS=hop)
  int geom_ = -1;                  // two-shot geometry: -1 by block size, 0 coarse, 1 fine, 2 flat (MXAR_TWOSHOT_GEOM)
  int64_t flat_min_ = int64_t{2} << 20;  // blocks of at least this many bytes use the flat geometry (MXAR_TWOSHOT_FLAT_MIN)
  bool launched_ = false;          // a launch has been enqueued (last_stream_ valid)
  hipStream_t last_stream_ = nullptr;
  hipEvent_t switch_ev_ = nullptr;  // recorded on last_stream_ when the stream changes
  CommStats stats_;
};

// Standalone data-plane kernels (csrc/hip/kernels.hip).
// out[i] = sum_{p < nslots} slots[p * slot_stride + i], fp32 accumulate; i < n.
void launch_reduce_slots(const void* slots, int64_t slot_stride_elems, int nslots, void* out, int64_t n, DType dt,
                         float scale, hipStream_t stream);
// dst[i] = (float)(i + offset) (reference data source AllreduceWorker.scala:285-291)
void launch_fill_iota(void* dst, int64_t n, double offset, DType dt, hipStream_t stream);
// dst[i] = slope * i + offset (iota: slope 1; a constant: slope 0)
void launch_fill_affine(void* dst, int64_t n, double slope, double offset, DType dt, hipStream_t stream);
void launch_clock_probe(uint64_t* out, int samples, uint64_t interval_ticks, hipStream_t stream);
// dst[i] = uniform(-1, 1) from a counter-based hash of (seed, i)
void launch_fill_uniform(void* dst, int64_t n, uint64_t seed, DType dt, hipStream_t stream);
// dst[0:bytes) = src[0:bytes) as a kernel (16-B aligned)
void launch_copy(const void* src, void* dst, int64_t bytes, hipStream_t stream);
// true when a kernel on `b` runs while a kernel on `a` spins (the streams sit on different
// hardware queues); kernels.hip
bool streams_independent(hipStream_t a, hipStream_t b, double timeout_ms = 50.0);
void set_copy_variant(int v);  // study knob: 0..3, -1 default
void set_reduce_variant(int v);  // study knob: 0 runtime-P loop, 1..4 static-P (U, NT), -1 default
// dst (dt_out) = src (dt_in), n elements
void launch_cast(const void* src, DType dt_in, void* dst, DType dt_out, int64_t n, hipStream_t stream);
// flat bucket pack/unpack: copy `count` tensors (ptr, numel) into / out of a contiguous bucket
void launch_bucket_copy(const uint64_t* dev_table, int count, void* bucket, DType dt, bool pack, int64_t total,
                        hipStream_t stream);

void hip_check(hipError_t e, const char* what);

}  // namespace mxar
