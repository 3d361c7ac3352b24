// Device-side pieces shared by the fused allreduce kernels (xgmi_comm.hip: two-shot,
// one-shot, ring, barrier; xgmi_threshold.hip: threshold / bounded-staleness two-shot):
// launch arguments, slab flag addressing, slab copy / reduce loops, launch epochs.
#pragma once

#include <hip/hip_runtime.h>

#include "device_common.h"
#include "xgmi_comm.h"

namespace mxar {
using namespace dev;

// One launch serves one rank (one process per GPU: gridDim.y == 1, rank = rank0) or all
// P logical ranks of a single-process cluster on one device (gridDim.y == P, rank =
// rank0 + blockIdx.y): every rank's workgroups are then co-resident in ONE dispatch, so
// no rank can be starved behind another on a shared hardware queue.
struct CommArgs {
  const char* in[kMaxRanks];
  char* out[kMaxRanks];
  // per rank: [0] epoch [1] ticket [2] error; threshold rounds: [3] completion / late-ticket
  // counter [4] round count [5] early arrivals [6] snapshot barrier [7] early tickets
  uint32_t* ctl[kMaxRanks];
  int64_t n;      // elements in this segment
  int64_t block;  // elements per block (two-shot) / whole segment (one-shot)
  int64_t chunk;  // elements per chunk (scatter / gather work unit)
  int64_t subchunk;  // elements per reduce work unit (chunk split `sub` ways)
  int nch;        // chunks per block
  int sub;        // reduce units per chunk
  int P;
  int rank0;
  int fence;      // bit0: system release before flags, bit1: system acquire after waits
  float scale;    // applied to the fp32 sum before rounding (1 = sum, 1/P = mean)
  int64_t maxch;
  int64_t off_S, off_R, slot_bytes;  // slot_bytes: the slot STRIDE in the slab (capacity + pad)
  int64_t slot_cap;                   // usable bytes per slot
  uint64_t timeout;
  char* base[kMaxRanks];
  // threshold kernel (xgmi_threshold.hip); rows = 1 for the other kernels
  int rows;            // S/R slot rows in the slab: row 0 (lock-step kernels) + trows
  int trows;           // threshold lag ring: rows 1..trows (maxLag + 1; 0 = not allocated)
  int full;            // thReduce = thComplete = 1: every contribution and chunk is taken
  int min_reduce;      // contributions per chunk that complete a reduce (thReduce)
  int64_t min_complete;  // reduced chunks that complete the round (thComplete)
  int32_t* counts;     // optional [P][nch] contributions per output chunk (0 = missing)
  int rescale;         // scale a chunk reduced from cnt contributions by P / cnt
  // protocol-engine rounds (xgmi_plane.cc, RoundSpec): explicit round epoch (0 = ctl[4] + 1),
  // forced-cold round (no own contribution, nothing waited for), the reference's
  // arrival-order accounting, and the pinned host word the engine raises on a catch-up
  uint32_t epoch_set;
  int cold;
  int order_ref;
  const uint32_t* hforce;
  const uint32_t* habort;  // pinned host word: rounds <= this epoch are abandoned (threshold kernel)
  uint32_t* err_out;  // optional: the round's error word, written by the last workgroup (pinned host)
  uint32_t* done_out;  // optional: set to the epoch by the last workgroup after its release (pinned host)
  // optional: where the last workgroup copies `counts` (P x nch int32, pinned host) once the
  // round is done - every workgroup writes its counts to device memory (`counts`), so no
  // unit waits on a PCIe write acknowledgement
  int32_t* counts_host;
  // low-latency one-shot (xgmi_ll.hip): slots [parity][src] of ll_slot bytes at off_LL
  int64_t off_LL, ll_slot;
  // fused reduce-scatter + AdamW + all-gather (xgmi_adam.hip): per rank fp32 shard state
  float* opt_p[kMaxRanks];
  float* opt_m[kMaxRanks];
  float* opt_v[kMaxRanks];
  float lr, beta1, beta2, eps, wd, c1, c2_sqrt;  // c1 = 1 - beta1^t, c2_sqrt = sqrt(1 - beta2^t)
  // phase profile (MXAR study knob, XgmiComm::set_phase_stamps): per (rank y, workgroup x)
  // kPhaseSlots s_memrealtime values - see PhaseStamps below
  uint64_t* stamps;
  uint64_t delay;      // test knob: ticks rank `delay_rank` idles before phase 1
  int delay_rank;
  // test knob (XgmiComm::set_read_delay): ticks rank `rdelay_rank` idles before the phase that
  // reads what peers pushed - holds a slow reader inside its launch (slot-reuse tests)
  uint64_t rdelay;
  int rdelay_rank;
  // test knob (XgmiComm::set_forward_delay): ticks rank `fdelay_rank` idles before the ring's
  // LAST all-gather forward (its late flag then races the next kernel's flags - the flag
  // ownership test, tests/test_comm_gpu.py)
  uint64_t fdelay;
  int fdelay_rank;
  int noguard;  // MXAR_SLOT_GUARD=0: skip entry_guard (A/B of its cost and negative control only)
  int ring_hop_rows;  // study only (MXAR_RING_FLAGS=hop): the pre-fix ring flag layout, row = hop index
  // threshold kernel with sub > 1 (chunks split into `sub` slices of `subchunk` elements,
  // one workgroup each): the rank's own scratch, zeroed when the membership is configured.
  // split_dec: 64-bit decision words, [c] own reduce chunk c, [maxch + j * maxch + c] gather
  // unit (j, c); split_ctr: slice counters, [c] reduce, [maxch + j * maxch + c] scatter;
  // split_early: [j * maxch + c] = epoch when gather unit (j, c) was in at launch
  int sgroup;  // threshold kernel, unsplit chunks: chunks per scatter unit (one copy, one release)
  // threshold kernel: the lag gate of round e may be taken as open when this rank's round e - 1
  // was clean (it gathered every peer's reduced chunk of e - 1, so every peer had finished
  // e - 2). Set by the host when that proof holds: trows >= 2 and every rank's block holds at
  // least one chunk or the thresholds are full (XgmiComm::threshold_args).
  int gate_shortcut;
  // threshold kernel, protocol rounds with thresholds that tolerate a missing peer (unsplit
  // chunks only): a peer still inside the round that last used this round's row after
  // `lag_wait` ticks at the lag gate is SKIPPED for the round - nothing is written into its
  // slab (its FORCE request still is), so a straggler never holds the fast ranks back. The
  // laggard's late writes land in its own slots of our slab under older epochs, which no
  // round of ours takes (xgmi_threshold.hip, lag gate). 0 = wait (the bounded-buffer gate).
  int lag_skip;
  uint64_t lag_wait;
  // threshold kernel, full thresholds: the one-shot body (xgmi_threshold.hip) - every rank
  // pushes its whole input as low-latency units and reduces every chunk itself (small rounds)
  int oneshot;
  uint64_t* split_dec;
  uint32_t* split_ctr;
  uint32_t* split_early;
};

// A plane group's resident kernel (threshold_group_resident_kernel): y = 0 is the dispatcher
// row, y = 1 + k worker k's slice.
struct GroupResArgs {
  GroupResidentMember m[kMaxRanks];
  uint32_t* gstate;  // pinned: [0] kResRunning / kResExiting / kResExited (the group's kernel)
  uint64_t* gdm;     // device: [0] the dispatcher's heartbeat (100 MHz ticks)
  uint64_t idle;     // ticks without a round before the kernel leaves
  uint32_t gen;      // launch generation (the go words of a relaunched kernel differ)
  int Y;             // workers
};
static_assert(sizeof(CommArgs) + sizeof(GroupResArgs) <= 4096, "threshold_group_resident_kernel arguments exceed 4 KiB");

// Phase stamps of one workgroup (100 MHz s_memrealtime ticks): [0] start, [1] scatter done,
// [2] ticks spent waiting in the reduce phase, [3] reduce phase done, [4] ticks spent
// waiting in the gather phase, [5] end, [6] units reduced, [7] units gathered. Thread 0
// writes them; a null buffer (the default) costs one scalar compare per phase.
constexpr int kPhaseSlots = 8;
struct PhaseStamps {
  uint64_t* out;  // this workgroup's slots in the buffer, or null (uniform)
  uint64_t* lds;  // kPhaseSlots u64 of LDS (thread 0 updates them)
  __device__ __forceinline__ PhaseStamps(const CommArgs& a, uint64_t* sh)
      : PhaseStamps(a.stamps == nullptr
                        ? nullptr
                        : a.stamps + (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * kPhaseSlots,
                    sh) {}
  // this workgroup's slots given (a plane group's slice: its worker's own buffer)
  __device__ __forceinline__ PhaseStamps(uint64_t* slots, uint64_t* sh) : out(slots), lds(sh) {
    if (out != nullptr && threadIdx.x == 0) {
      for (int i = 0; i < kPhaseSlots; ++i) lds[i] = 0;
      lds[0] = wall_ticks();
    }
  }
  __device__ __forceinline__ void mark(int i) {
    if (out != nullptr && threadIdx.x == 0) lds[i] = wall_ticks();
  }
  __device__ __forceinline__ uint64_t now() const { return out != nullptr ? wall_ticks() : 0; }
  __device__ __forceinline__ void add(int i, uint64_t t0) {
    if (out != nullptr && threadIdx.x == 0) lds[i] += wall_ticks() - t0;
  }
  __device__ __forceinline__ void count(int i) {
    if (out != nullptr && threadIdx.x == 0) lds[i] += 1;
  }
  __device__ __forceinline__ void flush() {
    if (out != nullptr && threadIdx.x == 0)
      for (int i = 0; i < kPhaseSlots; ++i) out[i] = lds[i];
  }
};

__device__ __forceinline__ uint32_t* f1(const CommArgs& a, int k, int s, int c) {
  return reinterpret_cast<uint32_t*>(a.base[k]) + static_cast<int64_t>(s) * a.maxch + c;
}
__device__ __forceinline__ uint32_t* f2(const CommArgs& a, int k, int s, int c) {
  return reinterpret_cast<uint32_t*>(a.base[k]) + static_cast<int64_t>(a.rows * a.P + s) * a.maxch + c;
}
__device__ __forceinline__ uint32_t* fb(const CommArgs& a, int k, int s) {
  return reinterpret_cast<uint32_t*>(a.base[k]) + static_cast<int64_t>(2 * a.rows * a.P) * a.maxch + s;
}
__device__ __forceinline__ int64_t clamp_len(int64_t avail, int64_t cap) {
  return avail <= 0 ? 0 : (avail < cap ? avail : cap);
}

// Device-side bounds guard of one work unit: the bytes [off, off + bytes) of
// a slot and the flag index `flag` must lie inside the slab geometry. The host derives the
// geometry so this never fires; if it does (a geometry bug), the unit moves no data, the
// error word gets ERR_BAD_ARGS (CommError on the host) and the flags are still published,
// so no peer hangs and nothing is written out of bounds. Wave-uniform scalar compares.
__device__ __forceinline__ bool unit_in_bounds(const CommArgs& a, int64_t off, int64_t bytes, int64_t flag,
                                               uint32_t* err) {
  const bool ok = off >= 0 && bytes >= 0 && off + bytes <= a.slot_cap && flag >= 0 && flag < a.maxch;
  if (!ok && threadIdx.x == 0) __hip_atomic_fetch_or(err, ERR_BAD_ARGS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return ok;
}

// Push len elements from ordinary memory into a (peer's) slab with write-through stores,
// 16 B per lane, 4 packs in flight per lane.
// Packs in flight per lane in the slab copies (scatter / gather phases). The persistent
// grids run 2 workgroups per CU, so bytes in flight come from this unroll.
#ifndef MXAR_COPY_U
#define MXAR_COPY_U 8
#endif
constexpr int kCopyU = MXAR_COPY_U;

template <class E>
__device__ __forceinline__ void copy_to_slab(char* slab_dst, const char* src, int64_t len) {
  const int64_t npk = len / E::ELEMS;
  const __amdgpu_buffer_rsrc_t rs = slab_rsrc(src);  // the input stream: nt loads (device_common.h)
  const __amdgpu_buffer_rsrc_t rd = slab_rsrc(slab_dst);
  int64_t i = threadIdx.x;
  constexpr int U = kCopyU;
  for (; i + (U - 1) * kCommThreads < npk; i += U * kCommThreads) {
    Pack16 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16_nt(rs, static_cast<uint32_t>((i + u * kCommThreads) * 16));
#pragma unroll
    for (int u = 0; u < U; ++u) st16_wt(rd, static_cast<uint32_t>((i + u * kCommThreads) * 16), v[u]);
  }
  for (; i < npk; i += kCommThreads) st16_wt(rd, static_cast<uint32_t>(i * 16), ld16_nt(rs, static_cast<uint32_t>(i * 16)));
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len) copy_scalar_wt<E>(rd, src, t);
}

// Copy len elements out of a (fine-grained) slab with nt loads - after the caller's
// acquire - 4 packs in flight per lane.
template <class E>
__device__ __forceinline__ void copy_from_slab(char* dst, const char* slab_src, int64_t len) {
  const int64_t npk = len / E::ELEMS;
  const __amdgpu_buffer_rsrc_t rs = slab_rsrc(slab_src);
  const __amdgpu_buffer_rsrc_t rd = slab_rsrc(dst);
  int64_t i = threadIdx.x;
  constexpr int U = kCopyU;
  for (; i + (U - 1) * kCommThreads < npk; i += U * kCommThreads) {
    Pack16 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16_nt(rs, static_cast<uint32_t>((i + u * kCommThreads) * 16));
#pragma unroll
    for (int u = 0; u < U; ++u) st16_wt(rd, static_cast<uint32_t>((i + u * kCommThreads) * 16), v[u]);
  }
  for (; i < npk; i += kCommThreads) st16_wt(rd, static_cast<uint32_t>(i * 16), ld16_nt(rs, static_cast<uint32_t>(i * 16)));
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len) st_scalar_wt<E>(rd, t, ld_scalar_nt<E>(rs, t));
}

// Reduction sources: source s is at slab0 + s * stride, except source `own` (if >= 0),
// which is the rank's own input. Every source is read with nt buffer loads through a
// descriptor chosen by a scalar select, so the P loads of a pack issue back to back
// with no per-source branch (and the own input is simply L1-bypassing).
struct RedSrc {
  const char* own_ptr;
  const char* slab0;
  int64_t stride;
  int own;
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(int s) const {
    return slab_rsrc(s == own ? own_ptr : slab0 + s * stride);
  }
};

// Sum P sources (fixed order s = 0..P-1, fp32) and store the result to up to P
// destinations. src(s) / dst(k) return byte pointers to element 0 of the chunk.
// Destinations of a reduced chunk: every peer slab is written through (sc0 sc1); the
// rank's own output (k == own) too when `wt_out`, so it leaves no dirty L2 lines for the
// next release fence to write back.
template <class E, int PT, class DstF>
__device__ __forceinline__ void reduce_to(int P, const RedSrc& src, int ndst, int own_dst, DstF dst, int64_t len,
                                          float scale, bool wt_out) {
  const int64_t npk = len / E::ELEMS;
  constexpr int U = 2;
  int64_t i = threadIdx.x;
  if constexpr (PT > 0) {
    __amdgpu_buffer_rsrc_t rs[PT];
#pragma unroll
    for (int s = 0; s < PT; ++s) rs[s] = src.rsrc(s);
    for (; i + (U - 1) * kCommThreads < npk; i += U * kCommThreads) {
      Pack16 v[PT][U];
#pragma unroll
      for (int s = 0; s < PT; ++s)
#pragma unroll
        for (int u = 0; u < U; ++u) v[s][u] = ld16_nt(rs[s], static_cast<uint32_t>((i + u * kCommThreads) * 16));
      Acc<E> acc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u].zero();
#pragma unroll
      for (int s = 0; s < PT; ++s)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u].add(v[s][u]);
      if (scale != 1.f) {
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u].scale(scale);
      }
      Pack16 o[U];
#pragma unroll
      for (int u = 0; u < U; ++u) o[u] = acc[u].pack();
      for (int k = 0; k < ndst; ++k) {
        char* d = dst(k);
        if (d == nullptr) continue;
        if (k == own_dst && !wt_out) {
#pragma unroll
          for (int u = 0; u < U; ++u) st16(d + (i + u * kCommThreads) * 16, o[u]);
        } else {
          const __amdgpu_buffer_rsrc_t rd = slab_rsrc(d);
#pragma unroll
          for (int u = 0; u < U; ++u) st16_wt(rd, static_cast<uint32_t>((i + u * kCommThreads) * 16), o[u]);
        }
      }
    }
  }
  // runtime P (and the tail of a static-P launch): the sources' packs load in batches of 8
  // before their adds (one memory latency per batch, not one per source); a source past P
  // loads nothing and adds +0, exact (acc starts at +0 and is never -0)
  auto store_all = [&](int64_t at, const Pack16& o) {
    for (int k = 0; k < ndst; ++k) {
      char* d = dst(k);
      if (d == nullptr) continue;
      if (k == own_dst && !wt_out)
        st16(d + at * 16, o);
      else
        st16_wt(slab_rsrc(d), static_cast<uint32_t>(at * 16), o);
    }
  };
  for (; i < npk; i += U * kCommThreads) {
    const int nu = i + kCommThreads < npk ? 2 : 1;
    Acc<E> acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u].zero();
    for (int s0 = 0; s0 < P; s0 += 8) {
      Pack16 v[8][U];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int s = s0 + q;
        const __amdgpu_buffer_rsrc_t rs = src.rsrc(s < P ? s : 0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (s < P && u < nu) {
            v[q][u] = ld16_nt(rs, static_cast<uint32_t>((i + u * kCommThreads) * 16));
          } else {
            v[q][u][0] = v[q][u][1] = v[q][u][2] = v[q][u][3] = 0u;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u].add(v[q][u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= nu) break;
      if (scale != 1.f) acc[u].scale(scale);
      store_all(i + u * kCommThreads, acc[u].pack());
    }
  }
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len) {
    float acc = 0.f;
    for (int s = 0; s < P; ++s) acc += ld_scalar_nt<E>(src.rsrc(s), t);
    acc *= scale;
    for (int k = 0; k < ndst; ++k) {
      char* d = dst(k);
      if (d == nullptr) continue;
      if (k == own_dst && !wt_out)
        Scalar<E>::store(d, t, acc);
      else
        st_scalar_wt<E>(slab_rsrc(d), t, acc);
    }
  }
}

// The rank's last workgroup to finish publishes the epoch for the next launch.
__device__ __forceinline__ void finish_launch(uint32_t* ctl, uint32_t epoch) {
  __syncthreads();
  if (threadIdx.x == 0) {
    // relaxed: only the count matters. The next launch of this communicator is ordered
    // after this one - same stream, or XgmiComm::order_after_last makes the new stream
    // wait - and kernel end publishes ctl[0]; no peer learns anything from this ticket
    // (slot reuse is guarded by entry_guard / finish_launch_done below). An acq_rel at agent
    // scope would be a `buffer_wbl2` per workgroup, writing back the XCD's dirty L2 lines
    // mid-kernel (e.g. AdamW state). Kernels whose last workgroup DOES tell peers that all
    // reads are done take a relaxed ticket too (finish_launch_done: every slab load fed a
    // store before it; xgmi_threshold.hip progress words: every wave drains first).
    const uint32_t t = __hip_atomic_fetch_add(&ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(&ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctl[0], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ uint32_t launch_epoch(const uint32_t* ctl) {
  return __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
}

// ---------------------------------------------------------------------------------
// Slot reuse across launches. A launch pushes into its peers' S / R slots in its first
// phase, before it has heard from those peers in this launch - while a slower peer may
// still be READING the same slots in the previous launch: a one-shot's reduce of S after
// the fast rank's next one-shot push, a two-shot's gather of R after the fast rank's next
// all-gather push, a ring hop into a neighbour that is still forwarding. A kernel whose
// slot reads can still be pending at peers once it has completed locally records the
// region(s) in ctl[12] (S) / ctl[13] (R) as its epoch and, from its last workgroup, writes
// "launch e done" into every peer's FB word once every workgroup's loads have returned.
// A launch that pushes into a region whose reads were left by the PREVIOUS launch first
// waits until the target peers' FB words reached that epoch (normally already true: one
// local load per peer). Every rank runs the same launch sequence, so the local words name
// the peers' epochs too. Two-shot chains record only R (their S reads end before any rank
// can complete) and push S first, and one-shot launches alternate between the S and R
// regions by epoch parity, so back-to-back two-shot or one-shot launches never poll.
// The low-latency kernel keeps its own parity slots and takes no part; the threshold kernel
// has its own progress-word gate (xgmi_threshold.hip).
enum : uint32_t { kHazS = 1u, kHazR = 2u };

__device__ __forceinline__ uint32_t later_epoch(uint32_t x, uint32_t y) {
  if (x == 0) return y;
  if (y == 0) return x;
  return static_cast<int32_t>(y - x) > 0 ? y : x;
}

// All threads call. `only` >= 0 waits for that peer alone (ring: the only rank it writes).
// Only the PREVIOUS launch's reads can still be pending: every kernel waits for flags of its
// own epoch from every peer before it can complete (the ring transitively, through its hops),
// so a peer whose flags this rank saw in launch e-1 had finished every launch before it
// (stream order). A hazard older than e-1 costs the two control-word loads (beside the
// epoch load, same line) and nothing else.
__device__ __forceinline__ void entry_guard(const CommArgs& a, const uint32_t* ctl, int r, uint32_t epoch,
                                            uint32_t regions, int only, uint64_t deadline, uint32_t* err) {
  if (a.noguard) return;  // uniform
  const uint32_t hs = (regions & kHazS) ? __hip_atomic_load(&ctl[12], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  const uint32_t hr = (regions & kHazR) ? __hip_atomic_load(&ctl[13], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  const uint32_t h = later_epoch(hs, hr);
  if (h == 0 || h != epoch - 1u) return;  // uniform: every thread loaded the same words
  if (threadIdx.x < 64) {
    const int k = static_cast<int>(threadIdx.x);
    const bool mine = k < a.P && k != r && (only < 0 || k == only);
    const uint32_t* f = mine ? fb(a, r, k) : nullptr;
    bool ok = f == nullptr || reached(ld_flag(f), h);
    while (!__all(ok)) {
      __builtin_amdgcn_s_sleep(1);
      if (!ok) ok = reached(ld_flag(f), h);
      if (wall_ticks() > deadline) break;
    }
    if (!__all(ok) && k == 0) __hip_atomic_fetch_or(err, ERR_TIMEOUT_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // write-after-read: the pushes below issue only after the poll returned - no acquire
  __syncthreads();
}

// Flag-ownership test knob: rank `fdelay_rank` idles before the ring's last forward.
__device__ __forceinline__ void forward_delay(const CommArgs& a, int r) {
  if (a.fdelay && r == a.fdelay_rank) {
    const uint64_t until = wall_ticks() + a.fdelay;
    while (wall_ticks() < until) __builtin_amdgcn_s_sleep(8);
  }
}

// Slot-reuse test knob: rank `rdelay_rank` idles before its slab reads (one scalar compare).
__device__ __forceinline__ void read_delay(const CommArgs& a, int r) {
  if (a.rdelay && r == a.rdelay_rank) {
    const uint64_t until = wall_ticks() + a.rdelay;
    while (wall_ticks() < until) __builtin_amdgcn_s_sleep(8);
  }
}

// finish_launch for kernels whose slot reads may outlive their local completion: the last
// workgroup tells every peer "launch `epoch` done" (FB word), records the regions' hazard
// epoch and advances ctl[0]. No drain: every slab load of a workgroup feeds a store (reduce,
// copy, forward) issued before this point, so it has returned - the barrier extends that to
// every wave and the ticket to every workgroup. (A vmcnt(0) drain here also waited for the
// write-through stores and cost ~0.5 us per launch.)
__device__ __forceinline__ void finish_launch_done(const CommArgs& a, uint32_t* ctl, uint32_t epoch, int r,
                                                   uint32_t regions) {
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(&ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x - 1 ? 1 : 0;
  }
  __syncthreads();
  if (!last) return;
  const int k = static_cast<int>(threadIdx.x);
  if (k < a.P && k != r) st_flag(fb(a, k, r), epoch);
  if (threadIdx.x == 0) {
    if (regions & kHazS) __hip_atomic_store(&ctl[12], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (regions & kHazR) __hip_atomic_store(&ctl[13], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ctl[0], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


// Host entry of the threshold kernel (xgmi_threshold.hip).
void launch_threshold(const CommArgs& a, dim3 grid, hipStream_t s, DType dt);
// A plane group's resident kernel: dim3(grid, workers + 1) (xgmi_threshold.hip).
void launch_threshold_group_resident(const CommArgs& a, const GroupResArgs& g, int grid, hipStream_t s, DType dt);
// Resident rounds (xgmi_threshold.hip; XgmiComm::launch_resident).
void launch_threshold_resident(const CommArgs& a, int grid, hipStream_t s, DType dt, const ResidentDoor* door,
                               uint32_t* hstate, uint32_t* dm, uint32_t seq, uint32_t gen, uint64_t idle_ticks);
// Progress words = value in every peer's slab (xgmi_threshold.hip; XgmiComm::publish_progress).
void launch_publish_progress(const CommArgs& a, uint32_t value, hipStream_t s);
// Host entry of the low-latency one-shot (xgmi_ll.hip).
void launch_ll(const CommArgs& a, dim3 grid, hipStream_t s, DType dt);
// Host entry of the fused reduce-scatter + AdamW + all-gather (xgmi_adam.hip).
void launch_adamw(const CommArgs& a, dim3 grid, hipStream_t s, DType dt);
// Host entry of all-to-all (mode 0) / all-gather (1) / reduce-scatter (2) (xgmi_coll.hip).
void launch_coll(const CommArgs& a, dim3 grid, hipStream_t s, DType dt, int mode);

}  // namespace mxar
