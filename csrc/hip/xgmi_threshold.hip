// Threshold (straggler-tolerant, bounded-staleness) fused allreduce over xGMI (gfx950).
//
// The reference's round semantics on the GPU hot path, in one persistent launch per round:
//   thReduce   - a chunk of rank r's block is reduced as soon as `min_reduce` of the P
//                contributions (own included) have arrived (AllreduceWorker.scala:116-121,
//                DataBuffer reachThreshold :31-33). Missing contributions count as zeros.
//   thComplete - the round completes once `min_complete` of the P x nch reduced chunks are
//                in; chunks still missing then are output as zeros with count 0
//                (AllreduceWorker.scala:143-145, reachRoundThreshold DataBuffer.scala:69-75).
//   maxLag     - the S/R slots and their flags form a ring of `trows` = maxLag + 1 rows
//                (slab rows 1..trows; row 0 belongs to the lock-step kernels), indexed by
//                the round epoch (the worker's lag ring, AllreduceWorker.scala:59-73).
//                Before writing row e % rows a rank waits until every peer has finished
//                the round that last used it (progress words), so a row is never
//                overwritten while a lagging peer still reads it.
//   catch-up   - a rank held at that gate by a laggard does not just wait: it writes a
//                FORCE request (the round the laggard must finish) into the laggard's slab,
//                and the laggard's round stops waiting for contributions and reduced chunks
//                and completes with what has arrived (zeros, count 0 elsewhere) - the
//                reference's forced catch-up (AllreduceWorker.scala:91-97), triggered by
//                the fast rank's traffic as in the reference (a future-round message makes
//                the laggard StartAllreduce, :123-126). The protocol engine raises the same
//                condition from the host (pinned `hforce` word) when StartAllreduce(r)
//                arrives with r - maxLag > round; a `cold` round (never started before it
//                became stale) contributes nothing and waits for nothing.
//   count      - per output chunk, how many contributions were summed (ReduceBlock.count,
//                AllreduceMessage.scala:19); 0 marks a chunk that was not completed.
//
// Two accountings of "what arrived first":
//   greedy (DP communicator) - a chunk's reduce sums everything present when the count
//                first reaches min_reduce (own input always present); the round keeps every
//                reduced chunk that arrived before it gave up. Most data per round.
//   reference (protocol engine, order_ref) - the reference's actor order: what was already
//                queued when StartAllreduce was processed comes first (snapshot at launch,
//                S0 per chunk / R0 for the round), then the worker's own scatter (it sends
//                to itself first, :194-209, but behind the queued messages), then later
//                arrivals. A reduce sums exactly the first min_reduce contributions of that
//                order, and the round output holds exactly the first min_complete reduced
//                chunks (tickets); own chunks reduced under a forced completion are flushed
//                after it (outdated), as in the reference. Same outputs and counts as the
//                host WorkerCore for the same arrival order.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "xgmi_device.h"

namespace mxar {

namespace {

constexpr int kMaxGatherUnits = kThresholdGatherUnits;  // gather units per workgroup (host geometry guarantees)
constexpr int kGatherWords = kMaxGatherUnits / 64;
constexpr int kMaxSnapChunks = kThresholdSnapChunks;    // reduce chunks per workgroup with an S0 snapshot

__device__ __forceinline__ uint32_t* prog(const CommArgs& a, int k, int s) {
  return reinterpret_cast<uint32_t*>(a.base[k]) + static_cast<int64_t>(2 * a.rows * a.P) * a.maxch + a.P + s;
}
__device__ __forceinline__ uint32_t* f2c(const CommArgs& a, int k, int rs, int c) {  // rs = row * P + src
  return reinterpret_cast<uint32_t*>(a.base[k]) + static_cast<int64_t>(2 * a.rows * a.P) * a.maxch + 2 * a.P +
         static_cast<int64_t>(rs) * a.maxch + c;
}
// FORCE[s] in rank k's slab: rank s asks k to complete every round <= this epoch now.
__device__ __forceinline__ uint32_t* forcew(const CommArgs& a, int k, int s) {
  return reinterpret_cast<uint32_t*>(a.base[k]) + static_cast<int64_t>(3 * a.rows * a.P) * a.maxch + 2 * a.P + s;
}
// FORCE requests only ever move forward (a later, lower request must not un-force a round):
// an atomic max on the peer's word, over xGMI on fine-grained memory.
__device__ __forceinline__ void force_max(uint32_t* w, uint32_t v) {
  __hip_atomic_fetch_max(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The engine's pinned host words, [0] force and [1] abort: ONE PCIe read when they are
// adjacent (the plane's layout). Returns "forced" (an abandoned round is forced too) and
// sets *aborted.
__device__ __forceinline__ bool host_forced(const uint32_t* hforce, const uint32_t* habort, uint32_t epoch,
                                            bool* aborted) {
  *aborted = false;
  if (hforce == nullptr) return false;
  uint32_t fw, aw = epoch - 1u;
  if (habort == hforce + 1) {
    const uint64_t w = __hip_atomic_load(reinterpret_cast<const uint64_t*>(hforce), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
    fw = static_cast<uint32_t>(w);
    aw = static_cast<uint32_t>(w >> 32);
  } else {
    fw = __hip_atomic_load(const_cast<uint32_t*>(hforce), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (habort != nullptr)
      aw = __hip_atomic_load(const_cast<uint32_t*>(habort), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  *aborted = reached(aw, epoch);
  return *aborted || reached(fw, epoch);
}

// Wave 0 only: is round `epoch` forced? Lane s < P reads FORCE[s] of the own slab (peer s
// waits at its lag gate for this rank); lane 63 reads the engine's pinned host words when
// `host` (a PCIe read: callers rate-limit it). Wave-uniform.
// (out of line - see copy_in below; it takes plain values, not the kernel's CommArgs, which an
// out-of-line callee would have copied to scratch)
__device__ __attribute__((noinline)) bool wave_forced_words(const uint32_t* own_force, int P, int r, uint32_t epoch,
                                                            const uint32_t* hforce, const uint32_t* habort) {
  // lane, not thread: every wave of a one-shot workgroup polls (xgmi_threshold.hip one-shot
  // body); with threadIdx.x only wave 0 could ever see a force and the others waited for the
  // deadline
  const int s = static_cast<int>(threadIdx.x & 63u);
  bool f = false;
  if (s < P && s != r) f = reached(ld_flag(own_force + s), epoch);
  if (hforce != nullptr && s == 63) {
    uint32_t fw, aw = epoch - 1u;
    if (habort == hforce + 1) {
      const uint64_t w = __hip_atomic_load(reinterpret_cast<const uint64_t*>(hforce), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
      fw = static_cast<uint32_t>(w);
      aw = static_cast<uint32_t>(w >> 32);
    } else {
      fw = __hip_atomic_load(const_cast<uint32_t*>(hforce), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (habort != nullptr) aw = __hip_atomic_load(const_cast<uint32_t*>(habort), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    f = reached(aw, epoch) || reached(fw, epoch);
  }
  return __any(f);
}
// lag skip: on-time rounds in a row after which a skipped peer is waited for again
constexpr uint32_t kHintRounds = 16;

__device__ __forceinline__ bool wave_forced(const CommArgs& a, const uint32_t* hforce, const uint32_t* habort, int r,
                                            uint32_t epoch, bool host) {
  return wave_forced_words(forcew(a, r, 0), a.P, r, epoch, host ? hforce : nullptr, habort);
}

// Host-word polls at most every 100 us per workgroup, the first one 100 us after the kernel
// started: every poll is a PCIe read that stalls the polling wave for microseconds, and at
// 512 workgroups x 2 planes a 20 us interval put ~50 M reads/s on the link, slowing the
// rounds themselves (same-box A/B, profiles/round2/README.md). A forced round is exceptional;
// learning of it within 100 us is enough.
struct HostPoll {
  uint64_t next;
  __device__ __forceinline__ explicit HostPoll(uint64_t now) : next(now + 10000) {}
  __device__ __forceinline__ bool due(uint64_t t) {
    if (t < next) return false;
    next = t + 10000;
    return true;
  }
  __device__ __forceinline__ bool due() { return due(wall_ticks()); }
};

// The slab's FORCE words (a peer waiting at its lag gate for this rank) are polled at most
// every 5 us, the first time 5 us after the round started: checked on every spin they doubled the period of the
// flag polls beside them (two dependent loads per iteration), and a catch-up noticed a few
// microseconds later costs nothing.
struct SlabPoll {
  // the first poll 5 us in too: a wait that ends sooner (the common case) never pays the
  // fine-grained load of P FORCE words on its critical path
  uint64_t next;
  __device__ __forceinline__ explicit SlabPoll(uint64_t now) : next(now + 500) {}
  __device__ __forceinline__ bool due(uint64_t t) {
    if (t < next) return false;
    next = t + 500;
    return true;
  }
};

// The first k set bits of `mask` in the order start, start+1, ... (mod P): the reference's
// rotated peer order (AllreduceWorker.scala:196) as the tie-break among simultaneous arrivals.
__device__ __forceinline__ uint32_t first_k(uint32_t mask, int k, int start, int P) {
  uint32_t out = 0;
  for (int i = 0; i < P && k > 0; ++i) {
    const int s = (start + i) % P;
    if ((mask >> s) & 1u) {
      out |= 1u << s;
      --k;
    }
  }
  return out;
}

__device__ __forceinline__ bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Protocol geometry (maxChunkSize elements, reference block ranges) need not be 16-B
// aligned: such a unit takes an element-wise path (wave-uniform branch).
// Code size matters for the small rounds: a round's code is fetched into the instruction
// cache of every CU it lands on, from L2, on the round's critical path (the full-threshold
// kernel went 19.3 -> 16.5 us at 8 logical ranks x 4 KiB when its code shrank from 51 to 26 KB,
// profiles/round5/README.md). Paths a round rarely takes - element-wise copies of unaligned
// protocol geometry, zero fills of given-up chunks, FORCE polls - are out-of-line functions, so
// the hot path stays dense.
template <class E>
__device__ __attribute__((noinline)) void copy_in_scalar(char* slab_dst, const char* src, int64_t len) {
  const __amdgpu_buffer_rsrc_t rd = slab_rsrc(slab_dst);
  for (int64_t t = threadIdx.x; t < len; t += kCommThreads) copy_scalar_wt<E>(rd, src, t);
}
template <class E>
__device__ __forceinline__ void copy_in(char* slab_dst, const char* src, int64_t len) {
  if (al16(slab_dst) && al16(src))
    copy_to_slab<E>(slab_dst, src, len);
  else
    copy_in_scalar<E>(slab_dst, src, len);
}

template <class E>
__device__ __attribute__((noinline)) void copy_out_scalar(char* dst, const char* slab_src, int64_t len) {
  const __amdgpu_buffer_rsrc_t rs = slab_rsrc(slab_src);
  const __amdgpu_buffer_rsrc_t rd = slab_rsrc(dst);
  for (int64_t t = threadIdx.x; t < len; t += kCommThreads) st_scalar_wt<E>(rd, t, ld_scalar_nt<E>(rs, t));
}
template <class E>
__device__ __forceinline__ void copy_out(char* dst, const char* slab_src, int64_t len) {
  if (al16(dst) && al16(slab_src))
    copy_from_slab<E>(dst, slab_src, len);
  else
    copy_out_scalar<E>(dst, slab_src, len);
}

// Zeros for a given-up chunk of the output. Write-through (sc0 sc1) like every other output
// store of this kernel when the host takes the round's completion from the done word
// (`done_out`): the output is then handed on before the kernel ends, so no store may sit in
// this XCD's L2 waiting for the end-of-kernel writeback.
template <class E>
__device__ __attribute__((noinline)) void zero_fill(char* dst, int64_t len) {
  const __amdgpu_buffer_rsrc_t rd = slab_rsrc(dst);
  if (al16(dst)) {
    const int64_t npk = len / E::ELEMS;
    Pack16 z;
    z[0] = z[1] = z[2] = z[3] = 0u;
    for (int64_t i = threadIdx.x; i < npk; i += kCommThreads) st16_wt(rd, static_cast<uint32_t>(i * 16), z);
    const int64_t t = npk * E::ELEMS + threadIdx.x;
    if (t < len) st_scalar_wt<E>(rd, t, 0.f);
    return;
  }
  for (int64_t t = threadIdx.x; t < len; t += kCommThreads) st_scalar_wt<E>(rd, t, 0.f);
}

// reduce_masked for unaligned protocol geometry: element by element (inline: an out-of-line
// function taking the kernel's CommArgs would copy them to scratch)
template <class E>
__device__ __forceinline__ void reduce_masked_scalar(const CommArgs& a, int P, int r, uint32_t mask,
                                                             const char* own_in, const char* S, int64_t slot,
                                                             char* own_out, int64_t roff, int64_t len, float scale,
                                                             uint32_t skip) {
  for (int64_t t = threadIdx.x; t < len; t += kCommThreads) {
    // every source's load issues before the first add (one memory latency per 8 sources,
    // not one per source); the fixed order s = 0..P-1 keeps the sum bit-exact (+0.f for a
    // source outside the mask is an identity: acc starts at +0 and is never -0)
    float acc = 0.f;
    for (int s0 = 0; s0 < P; s0 += 8) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int s = s0 + q;
        v[q] = (s < P && ((mask >> s) & 1u)) ? ld_scalar_nt<E>(slab_rsrc(s == r ? own_in : S + s * slot), t) : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) acc += v[q];
    }
    acc *= scale;
    for (int k = 0; k < P; ++k) {
      if (k == r) {
        if (own_out != nullptr) st_scalar_wt<E>(slab_rsrc(own_out), t, acc);
      } else if (!((skip >> k) & 1u)) {
        st_scalar_wt<E>(slab_rsrc(a.base[k] + roff), t, acc);
      }
    }
  }
}

// Sum the sources in `mask` (fixed order s = 0..P-1, fp32), store to the own output (when
// own_out != nullptr) and to the R slot of every peer not in `skip` (lagging peers, lag skip).
// Source r is the rank's own input.
template <class E>
__device__ __forceinline__ void reduce_masked(const CommArgs& a, int P, int r, uint32_t mask, const char* own_in,
                                              const char* S, int64_t slot, char* own_out, int64_t roff,
                                              int64_t len, bool wt_out, float scale, uint32_t skip) {
  const bool vec = al16(own_in) && al16(S) && (own_out == nullptr || al16(own_out)) && (roff & 15) == 0;
  if (!vec) {
    reduce_masked_scalar<E>(a, P, r, mask, own_in, S, slot, own_out, roff, len, scale, skip);
    return;
  }
  // Every source's pack is loaded before the first add: a batch of B sources x U packs issues
  // back to back (one memory latency per batch, not one per source - the per-source
  // load-then-add loop cost ~1 us of fine-grained-memory latency per peer at small rounds).
  // Sources outside the mask (or past P) load
  // nothing and add +0, which is exact (acc starts at +0 and is never -0), so the fixed order
  // s = 0..P-1 keeps the sum bit-exact.
  const int64_t npk = len / E::ELEMS;
  // Batches of B sources x U packs per lane: 2 sources x 8 (16 packs in flight), 3-4 x 2 and
  // more x 2 in batches of 8. Three instantiations, one call site each, so the kernel's code
  // stays small enough to fetch quickly on a cold CU. At 2 ranks the former 4 x 2 form kept
  // only 4 packs of real sources in flight and its reduce phase ran at ~4.5 TB/s against the
  // two-shot's 5.6 (phase stamps); 4 x 4 at 4 ranks measured 2 % slower than 4 x 2 at 64 MiB
  // (same-box A/B, profiles/round6 section 11).
  auto run = [&](auto bt) {
    constexpr int B = decltype(bt)::value;
    constexpr int U = B == 2 ? 8 : 2;
    for (int64_t i = threadIdx.x; i < npk; i += U * kCommThreads) {
      const int64_t left = (npk - i + kCommThreads - 1) / kCommThreads;
      const int nu = left < U ? static_cast<int>(left) : U;
      Acc<E> acc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u].zero();
      for (int s0 = 0; s0 < P; s0 += B) {
        Pack16 v[B][U];
#pragma unroll
        for (int q = 0; q < B; ++q) {
          const int s = s0 + q;
          const bool on = s < P && ((mask >> s) & 1u);
          const __amdgpu_buffer_rsrc_t rs = slab_rsrc(s == r ? own_in : S + (on ? s : 0) * slot);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (on && u < nu) {
              v[q][u] = ld16_nt(rs, static_cast<uint32_t>((i + u * kCommThreads) * 16));
            } else {
              v[q][u][0] = v[q][u][1] = v[q][u][2] = v[q][u][3] = 0u;
            }
          }
        }
#pragma unroll
        for (int q = 0; q < B; ++q)
#pragma unroll
          for (int u = 0; u < U; ++u) acc[u].add(v[q][u]);
      }
      Pack16 o[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (scale != 1.f) acc[u].scale(scale);
        o[u] = acc[u].pack();
      }
      for (int k = 0; k < P; ++k) {
        char* d = k == r ? own_out : ((skip >> k) & 1u) ? nullptr : a.base[k] + roff;
        if (d == nullptr) continue;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (u < nu) {
            const int64_t at = i + u * kCommThreads;
            if (k == r && !wt_out)
              st16(d + at * 16, o[u]);
            else
              st16_wt(slab_rsrc(d), static_cast<uint32_t>(at * 16), o[u]);
          }
        }
      }
    }
  };
  if (P <= 2)
    run(std::integral_constant<int, 2>{});
  else if (P <= 4)
    run(std::integral_constant<int, 4>{});
  else
    run(std::integral_constant<int, 8>{});
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len) {
    float acc = 0.f;
    for (int s = 0; s < P; ++s)
      if ((mask >> s) & 1u) acc += ld_scalar_nt<E>(slab_rsrc(s == r ? own_in : S + s * slot), t);
    acc *= scale;
    for (int k = 0; k < P; ++k) {
      char* d = k == r ? own_out : ((skip >> k) & 1u) ? nullptr : a.base[k] + roff;
      if (d == nullptr) continue;
      if (k == r && !wt_out)
        Scalar<E>::store(d, t, acc);
      else
        st_scalar_wt<E>(slab_rsrc(d), t, acc);
    }
  }
}

__device__ __forceinline__ uint32_t ld_ctl(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t add_ctl(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Split chunks (a.sub = S > 1). A protocol chunk is ONE decision (which contributions its
// reduce sums, whether the round takes it, its count) but S workgroups move its data, one
// slice each, so a few big chunks still spread over the whole grid. The slices agree on the
// decision through one epoch-tagged word per unit: the first slice ready to decide claims
// it (CAS), decides exactly as an unsplit unit would (tickets included) and publishes;
// every other slice adopts that decision. The decider never waits for anything after its
// claim, so a slice waiting for a decision always gets one.
constexpr uint64_t kDecided = 1ull << 31, kDecTake = 1ull << 30, kDecVal = (1ull << 30) - 1;

__device__ __forceinline__ uint64_t dec_load(uint64_t* w) {
  return __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool dec_this_epoch(uint64_t d, uint32_t epoch) {
  return static_cast<uint32_t>(d >> 32) == epoch;
}
// One lane. True: the caller decides and must dec_publish. False: *out is the decision of
// this epoch (0 with ERR_TIMEOUT_REDUCE if the decider never published before the deadline).
__device__ __forceinline__ bool dec_claim(uint64_t* w, uint32_t epoch, uint64_t deadline, uint32_t* err,
                                          uint64_t* out) {
  uint64_t d = dec_load(w);
  if (!dec_this_epoch(d, epoch)) {
    if (__hip_atomic_compare_exchange_strong(w, &d, static_cast<uint64_t>(epoch) << 32, __ATOMIC_ACQ_REL,
                                             __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT))
      return true;
  }
  while (!(d & kDecided)) {  // claimed by another slice: its decision is instructions away
    __builtin_amdgcn_s_sleep(1);
    d = dec_load(w);
    if (wall_ticks() > deadline) {
      __hip_atomic_fetch_or(err, ERR_TIMEOUT_REDUCE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      d = 0;
      break;
    }
  }
  *out = d;
  return false;
}
__device__ __forceinline__ void dec_publish(uint64_t* w, uint32_t epoch, bool take, uint32_t val) {
  __hip_atomic_store(w, (static_cast<uint64_t>(epoch) << 32) | kDecided | (take ? kDecTake : 0ull) | val,
                     __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// All threads. Every slice of a unit counts once per round; true (uniform) in the workgroup
// that counted last, which then publishes the unit's flags. Each slice releases its stores
// (system scope: they went to peer slabs) before it counts, so the last one's flags follow
// every slice's data. The last one resets the counter for the next round of this unit.
__device__ __forceinline__ bool last_slice(uint32_t* ctr, int S, int* sh) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    // relaxed: the system release above already ordered this slice's stores, and the last
    // slice reads nothing of the others' (it only publishes flags, behind its own release)
    const uint32_t t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = t == static_cast<uint32_t>(S) - 1u;
    if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sh = last ? 1 : 0;
  }
  __syncthreads();
  return *sh != 0;
}

}  // namespace

// A per-chunk count: a `sc1` store (leaves this XCD's L2), read back by the round's last
// workgroup with `sc1` loads after the ticket count - no release / acquire needed.
// A host word of round `epoch` (xgmi_plane.cc reads them): value in the low 8 bits (counts
// <= 32, error bits < 256), the epoch's low 24 bits above.
__device__ __forceinline__ uint32_t host_tag(uint32_t epoch, uint32_t v) { return (epoch << 8) | (v & 0xffu); }

__device__ __forceinline__ void put_count(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One-shot body (CommArgs::oneshot): the low-latency unit of xgmi_ll.hip - a 16-B store of two
// {4 payload bytes, tag} words, each delivered whole - tagged per round epoch. The tag mixes the
// epoch so that stale data in a slot (an older round's units, or plain two-shot data of a
// round of another size) matches it with probability 2^-64 per unit; never 0 (a fresh slab).
__device__ __forceinline__ uint32_t ll_tag(uint32_t epoch) {
  const uint32_t t = (epoch * 0x9E3779B1u) ^ 0x7F4A7C15u;
  return t ? t : 1u;
}
typedef unsigned int U32x2 __attribute__((ext_vector_type(2)));
constexpr int kAuxSysLd = 17;  // sc0 | sc1: loads that see the peers' xGMI stores in HBM
// 8 bytes of a byte range at unit i (zero past its end; the range is a whole number of 4-B words)
__device__ __forceinline__ uint2 load_unit8(const char* p, int64_t i, int64_t nbytes) {
  const int64_t off = i * 8;
  if (off + 8 <= nbytes) return *reinterpret_cast<const uint2*>(p + off);
  return make_uint2(off + 4 <= nbytes ? *reinterpret_cast<const uint32_t*>(p + off) : 0u, 0u);
}

// The per-round operands of threshold_round: a launch's own (CommArgs, threshold_kernel) or
// the ones a resident kernel read from the host's door (threshold_resident_kernel).
// The rank's own words come with them too (its control words, pinned host words and split
// scratch): a plane group's resident kernel (threshold_group_resident_kernel) runs several
// workers' rounds, each with its own set, under one CommArgs of shared geometry.
struct RoundVars {
  const char* in;
  char* out;
  int32_t* counts;       // this rank's [P][nch] (already offset)
  int32_t* counts_host;  // this rank's pinned copy (already offset)
  uint32_t* err_out;
  uint32_t* done_out;
  uint32_t epoch;  // 0: ctl[4] + 1
  int cold;
  // the lag gate is known open: every peer finished round epoch - trows (a resident kernel
  // whose previous round gathered every peer's chunks of epoch - 1, threshold_resident_kernel)
  int gate_open;
  // run by a resident kernel: its workgroups start the next round once ctl[4] names this
  // one, so the round end orders its counter resets before that store
  int resident;
  int rank;
  uint32_t* ctl;
  const uint32_t* hforce;
  const uint32_t* habort;
  uint64_t* split_dec;
  uint32_t* split_ctr;
  uint32_t* split_early;
  uint64_t* stamps;  // this workgroup's phase-stamp slots (null = off)
};

// A launch's own round of rank a.rank0 + y (threshold_kernel; the resident kernel: y = 0).
__device__ __forceinline__ RoundVars launch_vars(const CommArgs& a, int y, const char* in, char* out, int32_t* counts,
                                                 int32_t* counts_host, uint32_t* err_out, uint32_t* done_out,
                                                 uint32_t epoch, int cold, int gate_open, int resident) {
  const int64_t cy = static_cast<int64_t>(y) * a.P * a.nch;
  return RoundVars{in, out, counts ? counts + cy : nullptr, counts_host ? counts_host + cy : nullptr, err_out, done_out,
                   epoch, cold, gate_open, resident, a.rank0 + y, a.ctl[y], a.hforce, a.habort, a.split_dec,
                   a.split_ctr, a.split_early,
                   a.stamps == nullptr
                       ? nullptr
                       : a.stamps + (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * kPhaseSlots};
}

// One round of rank a.rank0 + blockIdx.y by the whole grid.
// Returns true when this workgroup's round took every peer's reduced chunk it gathers, with
// nothing forced, cold or given up (the resident kernel's lag-gate shortcut).
// FULL: a compile-time full-threshold round (thReduce = thComplete = 1, unsplit chunks - the
// DP communicator's exact lag-tolerant allreduce and most protocol rounds).
// Snapshot, tickets and split-chunk agreement fold away: less than half
// the code of the general kernel, whose instruction fetch a small round otherwise pays from
// L2 on every cold CU (51 KB of code vs 21 KB for the 8-rank two-shot).
// ONESHOT: the one-shot body of a small full-threshold round (CommArgs::oneshot, below).
template <class E, bool FULL, bool ONESHOT = false>
__device__ __forceinline__ bool threshold_round(const CommArgs& a, const RoundVars& rv) {
  constexpr int es = 16 / E::ELEMS;
  __shared__ uint32_t sh_mask;
  __shared__ int sh_flag;
  __shared__ int sh_last;
  __shared__ uint32_t sh_u32;
  __shared__ uint64_t sh_arr;
  __shared__ uint64_t pend[kGatherWords];
  __shared__ uint64_t early[kGatherWords];
  __shared__ uint32_t s0[kMaxSnapChunks];
  __shared__ uint64_t ps_lds[kPhaseSlots];
  // phase stamps (threshold layout): [0] start, [1] snapshot + lag gate done, [2] ticks
  // waiting for contributions + reduce bodies, [3] scatter + reduce done, [4] ticks waiting
  // in the gather + gather copies,
  // [5] end, [6] scatter done, [7] units gathered
  PhaseStamps ps(rv.stamps, ps_lds);
  const int P = a.P;
  const int r = rv.rank;
  const char* const in = rv.in;
  char* const out = rv.out;
  uint32_t* const ctl = rv.ctl;
  // threshold rounds count separately (ctl[4]); the protocol engine passes its round epochs.
  // ctl[14] = the last round of this rank that was clean (every workgroup gathered every
  // peer's reduced chunks): loaded beside ctl[4], same line, no extra latency
  const uint32_t clean_prev = rv.epoch ? 0u : ld_ctl(&ctl[14]);
  const uint32_t epoch = rv.epoch ? rv.epoch : ld_ctl(&ctl[4]) + 1u;
  const int row = 1 + static_cast<int>(epoch % static_cast<uint32_t>(a.trows));
  const int G = gridDim.x;
  const int64_t slot = a.slot_bytes;
  const int64_t rowS = a.off_S + static_cast<int64_t>(row) * P * slot;
  const int64_t rowR = a.off_R + static_cast<int64_t>(row) * P * slot;
  uint32_t* err = &ctl[2];
  const bool rel = a.fence & 1, acq = a.fence & 2;
  const int Pm1 = P > 1 ? P - 1 : 1;
  int32_t* const counts = rv.counts;
  const bool cold = rv.cold != 0;
  const bool ref = a.order_ref != 0;
  // Full thresholds (thReduce = thComplete = 1): every contribution and every chunk is taken
  // whatever the arrival order, so neither the launch snapshot (a grid-wide barrier) nor the
  // output tickets (one device-scope atomic per unit) change the result: both are skipped.
  // Forced rounds still exclude their own force-reduced chunks (reference order).
  const bool full = FULL || a.full != 0;
  const bool snap = ref && !cold && !full;  // cold rounds are forced from the start: no snapshot
  const bool tickets = !full;
  // work units: S slices per chunk (S = 1: a unit is a chunk). Scatter / gather unit
  // u = ((c * (P-1) + peer) * S + slice); reduce unit v = c * S + slice.
  const int S = (!FULL && a.sub > 1) ? a.sub : 1;
  const bool split = S > 1;
  const int nu = (P - 1) * a.nch * S;
  const int nr = a.nch * S;
  const int64_t sub = split ? a.subchunk : a.chunk;
  const int mine = blockIdx.x < static_cast<unsigned>(nu) ? (nu - 1 - static_cast<int>(blockIdx.x)) / G + 1 : 0;
  // Chunk c of block j exists: the last block may have fewer chunks than nch (uneven blocks,
  // SURVEY Q9). A chunk that does not exist is never a reduced chunk of the round: no ticket,
  // count 0 - the host WorkerCore counts only the chunks that exist.
  auto exists = [&](int j, int c) -> bool {
    return clamp_len(clamp_len(a.n - static_cast<int64_t>(j) * a.block, a.block) - static_cast<int64_t>(c) * a.chunk,
                     a.chunk) > 0;
  };
  const int nwords = (mine + 63) / 64;
  // ONE clock read for the round's prologue (each s_memrealtime is a scalar-memory round trip)
  const uint64_t t_start = wall_ticks();
  HostPoll hp(t_start);
  SlabPoll sp(t_start);
  bool clean = !cold;
  // One workgroup (then nch = 1, P <= 2): it also keeps its counts in LDS, so the round end
  // does not read them back from HBM.
  __shared__ int32_t sh_cnt[2];
  const bool counts_lds = G == 1 && P <= 2 && a.nch == 1;
  auto cput = [&](int64_t i, int32_t v) {
    put_count(counts + i, v);
    if (counts_lds) sh_cnt[i] = v;
  };

  uint64_t deadline = t_start + a.timeout;
  if (a.delay && r == a.delay_rank) {  // straggler simulation (tests)
    const uint64_t until = wall_ticks() + a.delay;
    while (wall_ticks() < until) __builtin_amdgcn_s_sleep(8);
    deadline = wall_ticks() + a.timeout;
  }

  // Reference order: what had arrived when the round started (S0 per own chunk, R0 for the
  // round) comes before the own scatter. One grid-wide count of R0 (every workgroup is
  // resident) decides how many later arrivals the round still takes.
  uint32_t etotal = 0;
  if (snap) {
    if (threadIdx.x < 64) {
      const int lane = static_cast<int>(threadIdx.x);
      int k = 0;
      for (int v = blockIdx.x; v < nr && k < kMaxSnapChunks; v += G, ++k) {
        const int c = v / S;
        const bool in_ = lane < P && lane != r && reached(ld_flag(f1(a, r, row * P + lane, c)), epoch);
        const uint32_t m = static_cast<uint32_t>(__ballot(in_));
        if (lane == 0) s0[k] = m;
      }
      uint32_t cnt = 0;
      for (int w = 0; w < nwords; ++w) {
        const int idx = w * 64 + lane;
        bool arr = false, first = false;
        if (idx < mine) {
          const int u = blockIdx.x + idx * G;
          const int b = u / S;
          const int c = b / Pm1;
          const int j = (r + 1 + b % Pm1) % P;
          arr = exists(j, c) && reached(ld_flag(f2(a, r, row * P + j, c)), epoch);
          first = u - b * S == 0;  // a split chunk's early arrival is decided by its slice 0
          if (split && first && arr)
            __hip_atomic_store(&rv.split_early[static_cast<int64_t>(j) * a.maxch + c], epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint64_t m = __ballot(arr);
        if (lane == 0) early[w] = m;
        cnt += static_cast<uint32_t>(__popcll(__ballot(arr && first)));
      }
      if (lane == 0) {
        if (cnt) add_ctl(&ctl[5], cnt);
        __hip_atomic_fetch_add(&ctl[6], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        // relaxed spin, ONE acquire after it: an acquire per poll would invalidate this
        // XCD's L2 on every iteration of every workgroup
        while (ld_ctl(&ctl[6]) < static_cast<uint32_t>(G)) {
          __builtin_amdgcn_s_sleep(1);
          if (wall_ticks() > deadline) {
            __hip_atomic_fetch_or(err, ERR_TIMEOUT_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        sh_u32 = ld_ctl(&ctl[5]);
      }
    }
    __syncthreads();
    etotal = sh_u32;
    if (split) {  // every slice of a chunk takes slice 0's early bit (written before the barrier)
      if (threadIdx.x < 64) {
        const int lane = static_cast<int>(threadIdx.x);
        for (int w = 0; w < nwords; ++w) {
          const int idx = w * 64 + lane;
          bool arr = false;
          if (idx < mine) {
            const int b = (static_cast<int>(blockIdx.x) + idx * G) / S;
            const int c = b / Pm1;
            const int j = (r + 1 + b % Pm1) % P;
            arr = ld_ctl(&rv.split_early[static_cast<int64_t>(j) * a.maxch + c]) == epoch;
          }
          const uint64_t m = __ballot(arr);
          if (lane == 0) early[w] = m;
        }
      }
      __syncthreads();
    }
  } else {
    for (int w = static_cast<int>(threadIdx.x); w < nwords; w += kCommThreads) early[w] = 0;
  }

  // Lag gate: every peer has finished the round that last used row `row` of its slab
  // (progress words live in OUR slab, written by the peers at the end of each round). A
  // peer that is not there yet gets a FORCE request: it completes that round with what
  // has arrived instead of waiting (catch-up), so this wait ends as soon as the laggard
  // runs. Only a laggard that never runs again (a dead process) turns into ERR_TIMEOUT_LAG -
  // unless the engine abandons the round meanwhile (host abort word: re-initialisation or
  // shutdown): an abandoned round that has not passed its gate writes nothing anywhere.
  // Shortcut (a.gate_shortcut, trows >= 2): this rank's round e - 1 was clean - every peer
  // published its reduced chunks of e - 1, which it does only after its round e - 2 ended
  // (rounds of a rank run in order; a launched round's kernel starts after the previous one
  // ended, a resident workgroup after its previous round's last workgroup), so every peer is
  // past e - 2 >= e - trows: P fine-grained progress-word loads (~2 us at 4 KiB rounds,
  // profiles/round4/README.md section 4) are skipped. The resident kernel proves it itself
  // (rv.gate_open); a launched round reads ctl[14], written by its predecessor's last
  // workgroup when every workgroup of that round was clean.
  // Lag skip (a.lag_skip, unsplit thresholds < 1): a peer still short of the gate after
  // a.lag_wait ticks is skipped for this round - its FORCE request is written, nothing else of
  // this round goes into its slab (scatter units, reduced chunks, counts). The reference's
  // fast workers never wait for a straggler either: their messages queue in its mailbox and
  // come out outdated (AllreduceWorker.scala:113-114,137-138). Each workgroup decides for its
  // own units, and both outcomes are safe: a peer that reached the gate may be written, one
  // that did not is not; the laggard's own late writes go to its slots of our slab with an
  // older epoch, which no later round of ours takes, and its rounds in order mean its newer
  // data always follows its older data.
  // One-shot body: this thread's unit of the fast pass and its input word, loaded BEFORE the
  // lag gate so the input load overlaps the gate's progress-word loads (both are latency)
  [[maybe_unused]] int64_t tot = 0, my_u = -1, my_b0 = 0, my_b1 = 0;
  [[maybe_unused]] uint2 own_unit = make_uint2(0u, 0u);
  if constexpr (ONESHOT) {
    const int nq = P * a.nch;
    auto chunk_span = [&](int q, int64_t* b0, int64_t* b1) __attribute__((always_inline)) -> bool {  // bytes of chunk q (false: none)
      const int j = q / a.nch;
      const int c = q - j * a.nch;
      const int64_t blen = clamp_len(a.n - static_cast<int64_t>(j) * a.block, a.block);
      const int64_t clen = clamp_len(blen - static_cast<int64_t>(c) * a.chunk, a.chunk);
      *b0 = (static_cast<int64_t>(j) * a.block + static_cast<int64_t>(c) * a.chunk) * es;
      *b1 = *b0 + clen * es;
      return clen > 0;
    };
    // the fast pass's mapping (below): thread t of this workgroup owns flat unit t of the
    // workgroup's chunks q = blockIdx.x + i * G
    for (int q = blockIdx.x; q < nq; q += G) {
      int64_t b0, b1;
      if (!chunk_span(q, &b0, &b1)) continue;
      const int64_t u0 = b0 / 8, u1 = (b1 + 7) / 8;
      const int64_t t = static_cast<int64_t>(threadIdx.x) - tot;
      if (t >= 0 && t < u1 - u0) {
        my_u = u0 + t;
        my_b0 = b0;
        my_b1 = b1;
      }
      tot += u1 - u0;
    }
    if (!cold && tot <= kCommThreads && my_u >= 0) own_unit = load_unit8(in, my_u, a.n * es);
  }
  __shared__ uint32_t sh_skip;
  const bool gate_open = a.gate_shortcut &&
                         (rv.gate_open || (rv.epoch == 0 && clean_prev != 0u && clean_prev == epoch - 1u));
  if (gate_open) {
    if (threadIdx.x == 0) {
      sh_flag = 0;
      sh_skip = 0;
    }
  } else if (threadIdx.x < 64) {
    const int k = static_cast<int>(threadIdx.x);
    const uint32_t target = epoch - static_cast<uint32_t>(a.trows);
    const uint32_t* f = (k < P && k != r) ? prog(a, r, k) : nullptr;
    bool ok = f == nullptr || reached(ld_flag(f), target);
    bool asked = false, aborted = false;
    // lag skip: a peer this rank skipped last round (ctl[15], sticky while it lags) is skipped
    // at once; any other after lag_wait - a peer momentarily late is waited for
    const uint64_t skip_at =
        !a.lag_skip ? ~0ull : t_start + ((k < 32 && ((ld_ctl(&ctl[15]) >> k) & 1u)) ? 0ull : a.lag_wait);
    bool give = false;
    while (!__all(ok || give)) {
      if (!ok && !asked && blockIdx.x == 0) {
        force_max(forcew(a, k, r), target);
        asked = true;
      }
      give = !ok && wall_ticks() >= skip_at;
      if (__all(ok || give)) break;
      __builtin_amdgcn_s_sleep(2);
      if (!ok) ok = reached(ld_flag(f), target);
      if (rv.habort != nullptr && hp.due()) {
        bool ab = false;
        if (k == 0) (void)host_forced(rv.hforce, rv.habort, epoch, &ab);
        if (__any(ab)) {
          aborted = true;
          break;
        }
      }
      if (wall_ticks() > deadline) {
        if (k == 0) __hip_atomic_fetch_or(err, ERR_TIMEOUT_LAG, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    const uint32_t lag = a.lag_skip ? static_cast<uint32_t>(__ballot(!ok)) : 0u;
    // a skipped peer gets nothing of this round, so its round `epoch` can only end forced:
    // force it now (up to this round), not only up to epoch - trows - it then completes its
    // stale rounds at once with what it has and is back at the gate in time, instead of
    // waiting trows rounds for the force and staying skipped (a one-off late peer would
    // otherwise turn into a permanent laggard). The sticky hint skips it at once next round.
    if (a.lag_skip && blockIdx.x == 0) {
      // (k < P first: a 32-bit shift by k >= 32 wraps on the hardware - lane 32 + j would
      // alias peer j and write through base[32 + j], past the peer table)
      if (k < P && ((lag >> k) & 1u)) force_max(forcew(a, k, r), epoch);
      // The sticky hint keeps a skipped peer until it has been at the gate on time for
      // kHintRounds rounds in a row (ctl[16 + k] counts them; a skip restarts the count). A
      // straggler that catches up in bursts - forced and cold rounds complete at once - is at
      // the gate now and then; clearing the hint on each such round made the fast ranks wait
      // lag_wait for it every few rounds (4.5x their period with a 0.2 ms straggler at 40 B,
      // profiles/round6/README.md section 6).
      const uint32_t hint = ld_ctl(&ctl[15]);
      const bool lagged = k < P && ((lag >> k) & 1u);
      bool clear = false;
      if (k < P && k != r && (lagged || (k < 32 && ((hint >> k) & 1u)))) {
        uint32_t streak = lagged ? 0u : ld_ctl(&ctl[16 + k]) + 1u;
        if (streak >= kHintRounds) {
          clear = true;
          streak = 0u;
        }
        __hip_atomic_store(&ctl[16 + k], streak, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const uint32_t up = static_cast<uint32_t>(__ballot(clear));
      if (k == 0) __hip_atomic_store(&ctl[15], (hint & ~up) | lag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (k == 0) {
      sh_flag = aborted ? 1 : 0;
      sh_skip = lag;
    }
    // No acquire here: the gate orders this round's STORES into the peers' rows after the
    // peers' reads of those rows (write-after-read - the progress word was published after
    // them, and our stores issue only once the poll has returned: the wait below + the
    // barrier). Nothing peer-written is LOADED before phase 2's and phase 3's own acquires
    // (flag / force / decision words are sc1 loads). A system-scope acquire here cost every
    // workgroup an L1 + L2 invalidate on the round's critical path.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const bool void_round = sh_flag != 0;  // abandoned before the exchange: no peer writes
  if (void_round) clean = false;
  const uint32_t skip = sh_skip;  // peers this workgroup writes nothing to (lag skip)
  ps.mark(1);

  if constexpr (ONESHOT) {
    // One-shot body (a.oneshot: full thresholds, unsplit, at most a few KiB per rank, chunk
    // boundaries on 4-B words, the LL-encoded input fits a slot): every rank pushes its WHOLE
    // input into its S slot of this row in every peer's slab as low-latency units (the tag is
    // the flag: no release, no flag store), then reduces EVERY chunk itself once each source's
    // words carry this round's tag. One xGMI hop and no fenced hand-off, where the two-shot
    // body below takes five on the round's critical path (scatter -> flag -> reduce ->
    // broadcast -> flag -> gather); same sums (fixed order s = 0..P-1 in fp32, one rounding)
    // and counts (P per chunk). The lag gate above guards the row exactly as for the two-shot:
    // a peer still reading its slot of this row (epoch - trows) is never overwritten. A chunk
    // that is forced, cold or timed out sums exactly the sources whose every word of the chunk
    // arrived, and reports that count - the two-shot's "reduce what has arrived".
    const uint32_t tag = ll_tag(epoch);
    const int64_t nbytes = a.n * es;
    static_assert(kOneshotRanks <= kMaxRanks, "one-shot sources beyond the peer table");
    const int64_t units = (nbytes + 7) / 8;
    const int64_t gstride = static_cast<int64_t>(G) * kCommThreads;
    const int nq = P * a.nch;
    auto chunk_span = [&](int q, int64_t* b0, int64_t* b1) __attribute__((always_inline)) -> bool {
      const int j = q / a.nch;
      const int c = q - j * a.nch;
      const int64_t blen = clamp_len(a.n - static_cast<int64_t>(j) * a.block, a.block);
      const int64_t clen = clamp_len(blen - static_cast<int64_t>(c) * a.chunk, a.chunk);
      *b0 = (static_cast<int64_t>(j) * a.block + static_cast<int64_t>(c) * a.chunk) * es;
      *b1 = *b0 + clen * es;
      return clen > 0;
    };
    const bool fast = !cold && !void_round && tot <= kCommThreads;  // uniform
    if (fast) {
      // each thread pushes the unit it will sum (loaded before the gate): the workgroups'
      // chunks together cover the input (a unit shared by two chunks goes twice, identical)
      if (my_u >= 0) {
        const Pack16 v{own_unit.x, tag, own_unit.y, tag};
        for (int k = 0; k < P; ++k)
          if (k != r)
            st16_wt(slab_rsrc(a.base[k] + rowS + static_cast<int64_t>(r) * slot), static_cast<uint32_t>(my_u * 16), v);
      }
    } else if (!cold && !void_round) {
      // the units of this workgroup's OWN chunks, as the fast pass does: `fast` is uniform per
      // workgroup, not over the grid (a workgroup with more chunks may exceed the fast pass
      // while the others do not), so a grid-stride walk here left the units whose stride owner
      // took the fast pass unpushed - their chunks waited out the deadline (MXAR_GRID=64, 8 x
      // 128 KiB; the 2- and 4-process stress tests at 64 KiB, profiles/round6 section 12)
      for (int q = blockIdx.x; q < nq; q += G) {
        int64_t b0, b1;
        if (!chunk_span(q, &b0, &b1)) continue;
        const int64_t u1 = (b1 + 7) / 8;
        for (int64_t i = b0 / 8 + threadIdx.x; i < u1; i += kCommThreads) {
          const uint2 d = load_unit8(in, i, nbytes);
          Pack16 v;
          v[0] = d.x;
          v[1] = tag;
          v[2] = d.y;
          v[3] = tag;
          for (int k = 0; k < P; ++k)
            if (k != r) st16_wt(slab_rsrc(a.base[k] + rowS + static_cast<int64_t>(r) * slot), static_cast<uint32_t>(i * 16), v);
        }
      }
    }
    ps.mark(6);
    const char* const mine_s = a.base[r] + rowS;  // source s's units at mine_s + s * slot
    const __amdgpu_buffer_rsrc_t ro = slab_rsrc(out);
    __shared__ uint32_t sh_miss;
    auto poll_unit = [&](int64_t u, bool act, bool h0, bool h1, Pack16* v, bool& stop) __attribute__((always_inline)) -> uint32_t {
      uint32_t want = 0;  // sources whose words of this unit are not in yet
#pragma unroll
      for (int s = 0; s < kOneshotRanks; ++s) {
        if (s < P && s != r && act) {
          v[s] = __builtin_amdgcn_raw_buffer_load_b128(slab_rsrc(mine_s + static_cast<int64_t>(s) * slot),
                                                        static_cast<int>(u * 16), 0, kAuxSysLd);
          want |= 1u << s;
        }
      }
      auto in_now = [&](const Pack16& w) { return (!h0 || w[1] == tag) && (!h1 || w[3] == tag); };
#pragma unroll
      for (int s = 0; s < kOneshotRanks; ++s)
        if (((want >> s) & 1u) && in_now(v[s])) want &= ~(1u << s);
      const uint64_t tw = ps.now();
      while (__any(want != 0) && !stop) {
        __builtin_amdgcn_s_sleep(1);
        // every missing source's load in flight first, then the tag checks: a check right after
        // each load waited for it before the next was issued (one memory round trip per source)
#pragma unroll
        for (int s = 0; s < kOneshotRanks; ++s)
          if ((want >> s) & 1u)
            v[s] = __builtin_amdgcn_raw_buffer_load_b128(slab_rsrc(mine_s + static_cast<int64_t>(s) * slot),
                                                          static_cast<int>(u * 16), 0, kAuxSysLd);
#pragma unroll
        for (int s = 0; s < kOneshotRanks; ++s)
          if (((want >> s) & 1u) && in_now(v[s])) want &= ~(1u << s);
        const uint64_t now = wall_ticks();
        const bool host = hp.due(now);
        const bool slab = sp.due(now);  // both polls advance unconditionally: a short-circuit
                                        // picked one of them by address (a scratch round trip)
        if ((host || slab) && wave_forced(a, rv.hforce, rv.habort, r, epoch, host)) stop = true;
        if (now > deadline) {
          if ((threadIdx.x & 63) == 0)
            __hip_atomic_fetch_or(err, ERR_TIMEOUT_SCATTER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          stop = true;
        }
      }
      ps.add(2, tw);
      return want;
    };
    // every source in: the sum in rank order (`own`: this rank's unit, already loaded)
    auto sum_unit = [&](int64_t u, bool h0, bool h1, const Pack16* v, const uint2* own) __attribute__((always_inline)) {
      Acc8<E> acc;
#pragma unroll
      for (int s = 0; s < kOneshotRanks; ++s) {
        if (s >= P) continue;
        acc.add(s == r ? (own != nullptr ? *own : load_unit8(in, u, nbytes)) : make_uint2(v[s][0], v[s][2]));
      }
      const uint2 o = acc.pack(a.scale);
      if (h0 && h1)
        __builtin_amdgcn_raw_buffer_store_b64(U32x2{o.x, o.y}, ro, static_cast<int>(u * 8), 0, kAuxWt);
      else if (h0)
        __builtin_amdgcn_raw_buffer_store_b32(o.x, ro, static_cast<int>(u * 8), 0, kAuxWt);
      else if (h1)
        __builtin_amdgcn_raw_buffer_store_b32(o.y, ro, static_cast<int>(u * 8 + 4), 0, kAuxWt);
    };
    // Fast pass: every unit of every chunk this workgroup owns at once, one per thread (the host
    // sizes the grid for it), all sources' loads in flight together - one load round trip after
    // the data lands, where a chunk-by-chunk walk pays one per chunk. It completes when every
    // word of every source arrives (the common case at full thresholds); a forced / cold /
    // void / timed-out pass falls through to the chunk-by-chunk body (arrival within a round is
    // final: it reads the slots again and reduces what arrived).
    bool done_fast = false;
    if (fast) {
      {
        const bool act = my_u >= 0;
        const bool h0 = act && my_u * 8 >= my_b0 && my_u * 8 < my_b1;
        const bool h1 = act && my_u * 8 + 4 >= my_b0 && my_u * 8 + 4 < my_b1;
        Pack16 v[kOneshotRanks];
        bool stop = false;
        const uint32_t want = poll_unit(my_u, act, h0, h1, v, stop);
        if (__syncthreads_or(want != 0u) == 0) {
          if (act) sum_unit(my_u, h0, h1, v, &own_unit);
          if (counts)
            for (int q = blockIdx.x + static_cast<int>(threadIdx.x) * G; q < nq; q += G * kCommThreads) {
              int64_t b0, b1;
              cput(static_cast<int64_t>(q), chunk_span(q, &b0, &b1) ? P : 0);
            }
          done_fast = true;
        }
      }
    }
    for (int q = blockIdx.x; q < nq && !done_fast; q += G) {
      const int j = q / a.nch;
      const int c = q - j * a.nch;
      const int64_t blen = clamp_len(a.n - static_cast<int64_t>(j) * a.block, a.block);
      const int64_t clen = clamp_len(blen - static_cast<int64_t>(c) * a.chunk, a.chunk);
      if (clen <= 0) {  // past the end of a short last block: not a chunk of the round
        if (threadIdx.x == 0 && counts) cput(static_cast<int64_t>(q), 0);
        continue;
      }
      const int64_t b0 = (static_cast<int64_t>(j) * a.block + static_cast<int64_t>(c) * a.chunk) * es;
      const int64_t b1 = b0 + clen * es;
      const int64_t u0 = b0 / 8, u1 = (b1 + 7) / 8;
      if (threadIdx.x == 0) sh_miss = 0u;
      __syncthreads();
      // a forced / timed-out wave stops waiting; a cold round waits for nothing
      bool stop = cold || void_round;
      uint32_t miss = 0;
      for (int64_t ub = u0; ub < u1; ub += kCommThreads) {
        const int64_t u = ub + threadIdx.x;
        const bool act = u < u1;
        const bool h0 = act && u * 8 >= b0 && u * 8 < b1;          // low word in this chunk
        const bool h1 = act && u * 8 + 4 >= b0 && u * 8 + 4 < b1;  // high word in this chunk
        Pack16 v[kOneshotRanks];
        const uint32_t want = poll_unit(u, act, h0, h1, v, stop);
        miss |= want;
        if (act && want == 0u && !cold) sum_unit(u, h0, h1, v, nullptr);
      }
      // the common case (every word of every source in) costs one barrier-with-reduction; only
      // a forced / cold / timed-out chunk gathers which sources it misses
      const bool any_miss = __syncthreads_or(miss != 0u) != 0;
      if (any_miss) {
        if (miss) atomicOr(&sh_miss, miss);
        __syncthreads();
      }
      const uint32_t missing = any_miss ? sh_miss : 0u;
      const bool partial = missing != 0u || cold || void_round;
      uint32_t mask = (P >= 32 ? 0xffffffffu : ((1u << P) - 1u)) & ~missing;
      if (cold) mask &= ~(1u << r);
      if (void_round) mask = 0u;  // abandoned before the exchange: zeros, count 0 (as the two-shot)
      if (partial) {
        // forced / cold / timed out: the sources whose every word of the chunk arrived (arrival
        // within a round is final), the same mask for every word of the chunk
        clean = false;
        for (int64_t u = u0 + threadIdx.x; u < u1; u += kCommThreads) {
          const bool h0 = u * 8 >= b0 && u * 8 < b1;
          const bool h1 = u * 8 + 4 >= b0 && u * 8 + 4 < b1;
          Acc8<E> acc;
          for (int s = 0; s < P; ++s) {
            if (!((mask >> s) & 1u)) continue;
            if (s == r) {
              acc.add(load_unit8(in, u, nbytes));
            } else {
              const Pack16 w = __builtin_amdgcn_raw_buffer_load_b128(slab_rsrc(mine_s + static_cast<int64_t>(s) * slot),
                                                                     static_cast<int>(u * 16), 0, kAuxSysLd);
              acc.add(make_uint2(w[0], w[2]));
            }
          }
          const uint2 o = acc.pack(a.scale);
          if (h0) __builtin_amdgcn_raw_buffer_store_b32(o.x, ro, static_cast<int>(u * 8), 0, kAuxWt);
          if (h1) __builtin_amdgcn_raw_buffer_store_b32(o.y, ro, static_cast<int>(u * 8 + 4), 0, kAuxWt);
        }
      }
      if (threadIdx.x == 0 && counts) cput(static_cast<int64_t>(j) * a.nch + c, __popc(mask));
      __syncthreads();  // sh_miss is reused by the next chunk
    }
    ps.mark(3);
  } else {
  // Phase 1 - ScatterBlock into the owners' row slots (a cold or void round sends nothing).
  // Unsplit chunks travel in groups of `sgroup` consecutive chunks of one destination block:
  // one contiguous copy and ONE release for the group, then one flag per chunk (each chunk
  // stays its own arrival for the owner's threshold decision). Small chunks otherwise cost a
  // fence each and the scatter ran at a quarter of the two-shot's rate (phase stamps,
  // profiles/round3/README.md).
  if (!cold && !void_round) {
    if (split) {
      for (int u = blockIdx.x; u < nu; u += G) {
        const int b = u / S;
        const int c = b / Pm1;
        const int j = (r + 1 + b % Pm1) % P;
        const int64_t bstart = static_cast<int64_t>(j) * a.block;
        const int64_t cstart = static_cast<int64_t>(c) * a.chunk + static_cast<int64_t>(u - b * S) * sub;
        const int64_t len = clamp_len(clamp_len(clamp_len(a.n - bstart, a.block) - c * a.chunk, a.chunk) -
                                          (cstart - c * a.chunk),
                                      sub);
        if (len > 0) copy_in<E>(a.base[j] + rowS + r * slot + cstart * es, in + (bstart + cstart) * es, len);
        if (!last_slice(&rv.split_ctr[a.maxch + static_cast<int64_t>(j) * a.maxch + c], S, &sh_last)) continue;
        publish_flags([&](int) { return f1(a, j, row * P + r, c); }, 1, epoch, rel);
      }
    } else {
      const int gs = a.sgroup > 1 ? a.sgroup : 1;
      const int ngr = (a.nch + gs - 1) / gs;
      const int nsu = Pm1 * ngr;
      for (int u = blockIdx.x; u < nsu; u += G) {
        const int cg = u / Pm1;
        const int j = (r + 1 + u % Pm1) % P;
        if ((skip >> j) & 1u) continue;  // a lagging owner: uniform per workgroup (LDS)
        const int c0 = cg * gs;
        const int ncg = a.nch - c0 < gs ? a.nch - c0 : gs;
        const int64_t bstart = static_cast<int64_t>(j) * a.block;
        const int64_t cstart = static_cast<int64_t>(c0) * a.chunk;
        const int64_t len = clamp_len(clamp_len(a.n - bstart, a.block) - cstart, static_cast<int64_t>(ncg) * a.chunk);
        if (len > 0) copy_in<E>(a.base[j] + rowS + r * slot + cstart * es, in + (bstart + cstart) * es, len);
        publish_flags([&](int i) { return f1(a, j, row * P + r, c0 + i); }, ncg, epoch, rel);
      }
    }
  }
  ps.mark(6);

  // Phase 2 - reduce own chunk c once min_reduce contributions are in
  const int64_t bstart_own = static_cast<int64_t>(r) * a.block;
  const int64_t blen_own = clamp_len(a.n - bstart_own, a.block);
  const uint32_t all = P >= 32 ? 0xffffffffu : ((1u << P) - 1u);
  const uint32_t others = all & ~(1u << r);
  const uint32_t own = cold ? 0u : (1u << r);
  int kk = 0;
  for (int v = blockIdx.x; v < nr; v += G, ++kk) {
    const int c = v / S;
    // this workgroup's slice of chunk c (the whole chunk when S = 1)
    const int64_t cstart = static_cast<int64_t>(c) * a.chunk + static_cast<int64_t>(v - c * S) * sub;
    const int64_t len = clamp_len(clamp_len(blen_own - c * a.chunk, a.chunk) - (cstart - c * a.chunk), sub);
    uint64_t* const dec = split ? &rv.split_dec[c] : nullptr;
    if (void_round) {  // nothing reduced, nothing sent
      if (len > 0) zero_fill<E>(out + (bstart_own + cstart) * es, len);
      if (threadIdx.x == 0 && counts) cput(static_cast<int64_t>(r) * a.nch + c, 0);
      continue;
    }
    if (threadIdx.x < 64) {
      const int s = static_cast<int>(threadIdx.x);
      const uint32_t* f = (s < P && s != r) ? f1(a, r, row * P + s, c) : nullptr;
      bool in_ = f != nullptr && reached(ld_flag(f), epoch);
      uint32_t present = static_cast<uint32_t>(__ballot(in_)) & others;
      bool forced = cold, timed_out = false;
      uint32_t mask = 0;
      const bool use_snap = snap && kk < kMaxSnapChunks;
      const uint32_t s0c = use_snap ? s0[kk] : present;
      if (snap && static_cast<int>(__popc(s0c)) >= a.min_reduce) {
        mask = first_k(s0c, a.min_reduce, r + 1, P);  // fired while draining the queue: no own
      } else {
        mask = (snap ? s0c : 0u) | own;
        const uint64_t tw = ps.now();
        while (!forced) {
          const uint32_t fresh = present & ~mask;
          if (snap) {
            if (fresh && static_cast<int>(__popc(mask)) < a.min_reduce)
              mask |= first_k(fresh, a.min_reduce - static_cast<int>(__popc(mask)), r + 1, P);
          } else {
            mask |= fresh;  // greedy: everything present
          }
          if (static_cast<int>(__popc(mask)) >= a.min_reduce || (mask | own) == (own | others)) break;
          // another slice of this chunk decided (or is deciding): adopt its decision
          if (split && __any(s == 0 && dec_this_epoch(dec_load(dec), epoch))) break;
          // one clock read per spin: s_memrealtime is a scalar memory round trip
          const uint64_t now = wall_ticks();
          const bool host = hp.due(now);
          const bool slab = sp.due(now);
          if ((host || slab) && wave_forced(a, rv.hforce, rv.habort, r, epoch, host)) {
            forced = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if (!in_ && f != nullptr) in_ = reached(ld_flag(f), epoch);
          present = static_cast<uint32_t>(__ballot(in_)) & others;
          if (now > deadline) {
            timed_out = true;
            break;
          }
        }
        ps.add(2, tw);
        if (forced) {  // the reference's forced reduce sums whatever the buffer holds
          if (!in_ && f != nullptr) in_ = reached(ld_flag(f), epoch);
          mask = (static_cast<uint32_t>(__ballot(in_)) & others) | own;
        }
      }
      if (threadIdx.x == 0) {
        if (forced || timed_out) clean = false;
        if (timed_out) __hip_atomic_fetch_or(err, ERR_TIMEOUT_SCATTER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        uint64_t d = 0;
        if (split && !dec_claim(dec, epoch, deadline, err, &d)) {  // adopt the chunk's decision
          sh_mask = static_cast<uint32_t>(d & kDecVal);
          sh_flag = (d & kDecTake) ? 1 : 0;
        } else {
          sh_mask = mask;
          // reference order: does the own reduced chunk make this round's output? (forced
          // reduces are flushed after the completion; a round complete at launch takes none)
          const bool real = blen_own - static_cast<int64_t>(c) * a.chunk > 0;
          int take = real ? 1 : 0;
          if (ref && real) {
            if (forced || etotal >= static_cast<uint32_t>(a.min_complete))
              take = 0;
            else if (tickets)
              take = etotal + add_ctl(&ctl[3], 1u) < static_cast<uint32_t>(a.min_complete) ? 1 : 0;
          }
          sh_flag = take;
          if (split) {
            if (acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the flags it decided on
            dec_publish(dec, epoch, take != 0, mask);
          }
        }
      }
      if (acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const uint64_t t_body = ps.now();  // stamp [2] also holds the reduce body (loads, stores, publish)
    const uint32_t mask = sh_mask;
    const bool take = sh_flag != 0;
    const int cnt = __popc(mask);
    const float sc = (a.rescale && cnt > 0) ? a.scale * static_cast<float>(P) / static_cast<float>(cnt) : a.scale;
    char* own_out = out + (bstart_own + cstart) * es;
    if (len > 0) {
      reduce_masked<E>(a, P, r, mask, in + (bstart_own + cstart) * es, a.base[r] + rowS + cstart * es, slot,
                       take ? own_out : nullptr, rowR + r * slot + cstart * es, len,
                       (a.fence & 1) || rv.done_out != nullptr, sc, skip);
      if (!take) zero_fill<E>(own_out, len);
    }
    // a split chunk is reduced once its last slice is: that workgroup publishes it
    if (split && !last_slice(&rv.split_ctr[c], S, &sh_last)) continue;
    if (threadIdx.x < static_cast<unsigned>(P) && static_cast<int>(threadIdx.x) != r && !((skip >> threadIdx.x) & 1u))
      st_flag(f2c(a, static_cast<int>(threadIdx.x), row * P + r, c), static_cast<uint32_t>(cnt));
    if (threadIdx.x == 0) {
      if (counts) cput(static_cast<int64_t>(r) * a.nch + c, take ? cnt : 0);
      if (!ref && tickets && blen_own - static_cast<int64_t>(c) * a.chunk > 0) add_ctl(&ctl[3], 1u);
    }
    publish_flags([&](int k) -> uint32_t* { return (k == r || ((skip >> k) & 1u)) ? nullptr : f2(a, k, row * P + r, c); },
                  P, epoch, rel);
    ps.add(2, t_body);
  }

  ps.mark(3);

  // Phase 3 - gather the other owners' chunks. Units of this workgroup are polled 64 at a
  // time by wave 0 and round-robin over passes, so a late chunk never blocks the count of
  // an early one. The round gives the rest up (zeros, count 0) once it has completed
  // (greedy: min_complete chunks in; reference: the ticket count reached) or is forced.
  for (int w = static_cast<int>(threadIdx.x); w < nwords; w += kCommThreads) {
    const int left = mine - w * 64;
    pend[w] = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
  }
  __syncthreads();
  bool gave_up = false;
  // full thresholds, unsplit, no counts: a gathered unit needs no decision (no ticket, no
  // count, no slice agreement) - no workgroup barrier per unit
  const bool fastg = !split && !tickets && counts == nullptr;
  // full thresholds, unsplit, with counts: still no decision, and the owners' count words of
  // the arrived units are loaded by the polling wave (one lane per unit, after the acquire)
  // instead of one dependent load plus two workgroup barriers per unit in thread 0 - at 8 x 1
  // MiB that serial walk was most of the gather (profiles/round6 section 13)
  const bool batchc = !split && !tickets && counts != nullptr;
  __shared__ uint32_t sh_gcnt[64];
  uint32_t idle = 0;  // passes since the last arrival (uniform over the workgroup)
  for (;;) {
    bool any = false, progressed = false;
    for (int w = 0; w < nwords; ++w) {
      if (pend[w] == 0) continue;
      any = true;
      if (threadIdx.x < 64) {
        const int idx = w * 64 + static_cast<int>(threadIdx.x);
        bool arr = false;
        int cj = 0, cc = 0;
        if ((pend[w] >> threadIdx.x) & 1ull) {
          const int b = (static_cast<int>(blockIdx.x) + idx * G) / S;
          cc = b / Pm1;
          cj = (r + 1 + b % Pm1) % P;
          arr = reached(ld_flag(f2(a, r, row * P + cj, cc)), epoch);
        }
        const uint64_t m = __ballot(arr);
        if (threadIdx.x == 0) sh_arr = m;
        if (m && acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (batchc && arr) sh_gcnt[threadIdx.x] = ld_flag(f2c(a, r, row * P + cj, cc));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      uint64_t m = sh_arr;
      __syncthreads();
      while (m) {
        const int i = __ffsll(static_cast<long long>(m)) - 1;
        m &= m - 1;
        const int idx = w * 64 + i;
        const int u = blockIdx.x + idx * G;
        const int b = u / S;
        const int c = b / Pm1;
        const int j = (r + 1 + b % Pm1) % P;
        uint64_t* const dec = split ? &rv.split_dec[a.maxch + static_cast<int64_t>(j) * a.maxch + c] : nullptr;
        bool take;
        if (fastg) {  // nothing to decide: every thread knows the unit is taken if it exists
          take = exists(j, c);
          if (threadIdx.x == 0) pend[w] &= ~(1ull << i);
        } else if (batchc) {  // the same, and the count the polling wave loaded
          take = exists(j, c);
          if (threadIdx.x == 0) {
            cput(static_cast<int64_t>(j) * a.nch + c, take ? static_cast<int32_t>(sh_gcnt[i]) : 0);
            pend[w] &= ~(1ull << i);
          }
        } else {
        if (threadIdx.x == 0) {
          int take = 1;
          uint64_t d = 0;
          const bool adopt = split && !dec_claim(dec, epoch, deadline, err, &d);
          if (adopt) {  // another slice of this unit decided
            take = (d & kDecTake) ? 1 : 0;
          } else if (!exists(j, c)) {
            take = 0;  // past the end of a short last block: not a chunk of the round
          } else if (!tickets) {
            // full thresholds: every reduced chunk that arrives before a force is taken
          } else if (ref) {
            if ((early[w] >> i) & 1ull)
              take = add_ctl(&ctl[7], 1u) < static_cast<uint32_t>(a.min_complete) ? 1 : 0;
            else
              take = etotal < static_cast<uint32_t>(a.min_complete) &&
                             etotal + add_ctl(&ctl[3], 1u) < static_cast<uint32_t>(a.min_complete)
                         ? 1
                         : 0;
          } else {
            add_ctl(&ctl[3], 1u);
          }
          if (!adopt) {
            if (counts)
              cput(static_cast<int64_t>(j) * a.nch + c, take ? static_cast<int32_t>(ld_flag(f2c(a, r, row * P + j, c))) : 0);
            if (split) dec_publish(dec, epoch, take != 0, 0u);
          }
          sh_flag = take;
          pend[w] &= ~(1ull << i);
        }
        __syncthreads();
        take = sh_flag != 0;
        }
        const int64_t bstart = static_cast<int64_t>(j) * a.block;
        const int64_t cstart = static_cast<int64_t>(c) * a.chunk + static_cast<int64_t>(u - b * S) * sub;
        const int64_t len = clamp_len(clamp_len(clamp_len(a.n - bstart, a.block) - c * a.chunk, a.chunk) -
                                          (cstart - c * a.chunk),
                                      sub);
        const uint64_t t_copy = ps.now();  // stamp [4] also holds the gather copies
        if (len > 0) {
          if (take)
            copy_out<E>(out + (bstart + cstart) * es, a.base[r] + rowR + j * slot + cstart * es, len);
          else
            zero_fill<E>(out + (bstart + cstart) * es, len);
        }
        ps.add(4, t_copy);
        progressed = true;
        ps.count(7);
        if (!fastg && !batchc) __syncthreads();  // sh_flag is reused by the next unit
      }
      // thread 0's pend[] updates before anyone reads pend[] again (and sh_gcnt is refilled)
      if (fastg || batchc) __syncthreads();
    }
    if (!any) break;
    if (progressed) {
      idle = 0;
      continue;
    }
    // a full round gives up only on a force (or its deadline): between arrivals the wave
    // re-polls 7 times of 8 without the give-up block (a clock read, the host / slab force
    // polls and two workgroup barriers per pass delayed the next arrival's copy)
    if (full && !cold && !void_round && (++idle & 7) != 0) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    if (threadIdx.x < 64) {
      int give = 0;
      const uint32_t done = full ? 0u : ld_ctl(&ctl[3]);  // full rounds: only a force gives up
      if (ref)
        give = (etotal >= static_cast<uint32_t>(a.min_complete) ||
                etotal + done >= static_cast<uint32_t>(a.min_complete))
                   ? 1
                   : 0;
      else
        give = done >= static_cast<uint32_t>(a.min_complete) ? 1 : 0;
      if (!give && (cold || void_round)) give = 1;
      const uint64_t now = wall_ticks();
      if (!give) {
        const bool host = hp.due(now);
        const bool slab = sp.due(now);
        if ((host || slab) && wave_forced(a, rv.hforce, rv.habort, r, epoch, host)) give = 1;
      }
      if (!give && now > deadline) {
        if (threadIdx.x == 0)
          __hip_atomic_fetch_or(err, ERR_TIMEOUT_REDUCE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        give = 1;
      }
      if (threadIdx.x == 0) sh_flag = give;
    }
    __syncthreads();
    gave_up = sh_flag != 0;
    __syncthreads();
    if (gave_up) break;
    const uint64_t tw = ps.now();
    __builtin_amdgcn_s_sleep(2);
    ps.add(4, tw);
  }
  if (gave_up) {
    clean = false;
    for (int w = 0; w < nwords; ++w) {
      uint64_t m = pend[w];
      while (m) {
        const int i = __ffsll(static_cast<long long>(m)) - 1;
        m &= m - 1;
        const int u = blockIdx.x + (w * 64 + i) * G;
        const int b = u / S;
        const int c = b / Pm1;
        const int j = (r + 1 + b % Pm1) % P;
        const int64_t bstart = static_cast<int64_t>(j) * a.block;
        const int64_t cstart = static_cast<int64_t>(c) * a.chunk + static_cast<int64_t>(u - b * S) * sub;
        const int64_t len = clamp_len(clamp_len(clamp_len(a.n - bstart, a.block) - c * a.chunk, a.chunk) -
                                          (cstart - c * a.chunk),
                                      sub);
        bool take = false;
        if (split) {  // give the unit up, unless another slice of it already took it
          uint64_t* const dec = &rv.split_dec[a.maxch + static_cast<int64_t>(j) * a.maxch + c];
          if (threadIdx.x == 0) {
            uint64_t d = 0;
            if (dec_claim(dec, epoch, deadline, err, &d)) {
              if (counts) cput(static_cast<int64_t>(j) * a.nch + c, 0);
              dec_publish(dec, epoch, false, 0u);
              sh_flag = 0;
            } else {
              sh_flag = (d & kDecTake) ? 1 : 0;
              if (sh_flag && acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the chunk it saw arrive
            }
          }
          __syncthreads();
          take = sh_flag != 0;
          __syncthreads();
        } else if (threadIdx.x == 0 && counts) {
          cput(static_cast<int64_t>(j) * a.nch + c, 0);
        }
        if (len > 0) {
          if (take)
            copy_out<E>(out + (bstart + cstart) * es, a.base[r] + rowR + j * slot + cstart * es, len);
          else
            zero_fill<E>(out + (bstart + cstart) * es, len);
        }
      }
    }
  }

  }  // two-shot body
  ps.mark(5);
  ps.flush();

  // Round end: the last workgroup resets the per-round counters, records the round and
  // tells every peer that this rank is done with row `row`. The progress word promises the
  // peers that EVERY workgroup's reads of the row are done: every wave drains its memory
  // operations before the workgroup barrier, so the ticket follows them. The ticket itself
  // is relaxed (an acq_rel one was an L2 writeback + invalidate per workgroup on the round's
  // tail): the only data the last workgroup reads back are the counts, stored `sc1`
  // (put_count) before the drain and loaded `sc1` - the guide's fence-free hand-off form.
  // the error word, loaded before the drain so its latency hides behind it (one workgroup:
  // nobody else can raise it later; with more, the last one reads it again after its ticket)
  const uint32_t errv = (threadIdx.x == 0 && rv.err_out != nullptr) ? ld_ctl(err) : 0u;
  // The drain makes every workgroup's output / count stores complete before the ticket: only
  // the host hand-off needs that (the done word, the counts copied to pinned memory). The
  // progress words promise the peers that this rank's READS of the row are done, and every
  // load of a round feeds a store or a branch that issued before this point - a launched round
  // without host words skips the store-acknowledgement wait on its tail.
  if (rv.done_out != nullptr || rv.counts_host != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bool all_clean = clean;
  if (threadIdx.x == 0) {
    // one workgroup: it is the last (no ticket - a device-scope atomic's round trip). The
    // ticket's high half counts the clean workgroups (one atomic for both)
    const uint32_t inc = 1u + (clean ? 0x10000u : 0u);
    const uint32_t t = G == 1 ? 0u : __hip_atomic_fetch_add(&ctl[1], inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool is_last = (t & 0xffffu) == static_cast<uint32_t>(G) - 1;
    sh_flag = is_last ? ((t >> 16) + (clean ? 1u : 0u) == static_cast<uint32_t>(G) ? 3 : 1) : 0;
  }
  __syncthreads();
  const bool last = sh_flag != 0;
  all_clean = sh_flag == 3;
  if (threadIdx.x == 0) {
    if (last) {
      // one workgroup at full thresholds touched none of the round counters (no ticket, no
      // completion count, no snapshot): nothing to reset, and no other workgroup waits on ctl[4]
      const bool solo = G == 1 && full;
      // the next launched round's lag-gate shortcut (self-counted epochs only)
      if (rv.epoch == 0)
        __hip_atomic_store(&ctl[14], all_clean ? epoch : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!solo) {
        __hip_atomic_store(&ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!full) {  // full thresholds touch no ticket, snapshot or early-arrival counter
          __hip_atomic_store(&ctl[3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ctl[5], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ctl[6], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ctl[7], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // a resident kernel's workgroups start the next round once ctl[4] names this one: the
        // resets land first (a launched round's successor is ordered by the kernel boundary)
        if (rv.resident) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&ctl[4], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      // the host words below follow every store of the round; a launched round without host
      // words tells only its peers (progress: reads done, no release needed) and its successor
      // (kernel boundary)
      if (rv.resident || rv.done_out != nullptr || rv.err_out != nullptr || rv.counts_host != nullptr) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // solo: only this thread reads ctl[4] (the resident loop), so the store need not be
      // drained by the release above
      if (solo) __hip_atomic_store(&ctl[4], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (last) {
    // Host words AFTER the release, each tagged with the round epoch (host_tag): the host
    // takes them once the done word and every tag name the round, so no fence waits for
    // their PCIe write acknowledgements (a release before the done word did, on the round's
    // critical path). The counts: every workgroup's sc1 stores drained before its ticket.
    if (counts != nullptr && rv.counts_host != nullptr) {
      int32_t* dst = rv.counts_host;
      for (int64_t i = threadIdx.x; i < static_cast<int64_t>(P) * a.nch; i += kCommThreads) {
        const int32_t v = counts_lds ? sh_cnt[i] : __hip_atomic_load(counts + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dst + i, static_cast<int32_t>(host_tag(epoch, static_cast<uint32_t>(v))), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (threadIdx.x == 0) {
      if (rv.err_out) __hip_atomic_store(rv.err_out, host_tag(epoch, G == 1 ? errv : ld_ctl(err)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      for (int k = 0; k < P; ++k)
        if (k != r) st_flag(prog(a, k, r), epoch);
      // the round's completion word: every workgroup has passed its ticket and every output
      // store was write-through (zero_fill, reduce_masked with wt_out) before the release
      // above, so the host may hand the output on at once, before the kernel itself ends
      if (rv.done_out) st_flag(rv.done_out, epoch);
    }
  }
  return clean;
}

template <class E, bool FULL, bool ONESHOT>
__global__ __launch_bounds__(kCommThreads) void threshold_kernel(CommArgs a) {
  const int y = blockIdx.y;
  const RoundVars rv =
      launch_vars(a, y, a.in[y], a.out[y], a.counts, a.counts_host, a.err_out, a.done_out, a.epoch_set, a.cold, 0, 0);
  (void)threshold_round<E, FULL, ONESHOT>(a, rv);
}

// ---------------------------------------------------------------------------------
// Resident rounds (XgmiComm::launch_resident, xgmi_plane.cc). A protocol round of a few KiB
// is mostly launch: the host's launch call, the dispatch, and the skew between the
// workers' kernels, each of which then waits for the other's scatter. A resident kernel
// stays on the GPU between rounds: workgroup 0 (the leader) polls the host's door ring
// (pinned host memory, one 64-B entry per round, the sequence word written last) and hands
// each entry to the other workgroups through device words (`dm`); every workgroup then runs
// the same threshold_round a launch would, and waits for the round's last workgroup to
// reset the round counters (ctl[4] = epoch) before the next entry.
//
// Exit: a STOP entry, or no entry for `idle` ticks. The idle exit cannot lose an entry the
// host posts meanwhile: the leader writes EXITING to the host state word, fences, and reads
// the door once more (the host writes the entry, fences, then reads the state word - one
// side sees the other's write): an entry found then is taken (state back to RUNNING);
// otherwise the state becomes EXITED and the host launches a new kernel for that entry.
// dm (device, 64-bit words): [0] go = (launch generation << 32) | entry sequence, [2..9] the
// entry's 8 words (word 6 = epoch | cmd << 32). The generation keeps a relaunched kernel's
// workgroups from taking the previous kernel's last go (its idle exit) for theirs. Every
// hand-off moves the 64-B entry as ONE load / store instruction of 8 lanes: a host-memory
// read is a PCIe round trip of microseconds, and reading the fields one by one cost more
// than the launch the resident kernel saves (profiles/round4/README.md).
constexpr int kDmGo = 0, kDmEntry = 2;

__device__ __forceinline__ uint32_t sys_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Leader wave (workgroup 0, wave 0): waits for entry `seq`, copies it into dm and publishes
// go (more than one workgroup). Returns the lane's entry word (lanes < 8; word 6 = epoch |
// cmd << 32, cmd kResStop = leave).
__device__ uint64_t resident_door(const ResidentDoor* door, uint32_t* hstate, uint64_t* dm, uint32_t seq,
                                  uint32_t gen, uint64_t idle, bool broadcast) {
  const int lane = static_cast<int>(threadIdx.x);
  const ResidentDoor* d = door + seq % kResidentDoors;
  const uint64_t* dw = reinterpret_cast<const uint64_t*>(d);
  // Every poll reads the whole 64-B entry (lanes 0-7, one instruction: one PCIe round trip);
  // the entry is taken when its sequence word is `seq` and its check word matches the other
  // words - a read that caught the host mid-write fails the check and is simply repeated.
  auto poll = [&](uint64_t* w) -> bool {
    *w = lane < 8 ? __hip_atomic_load(dw + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t x = __shfl(*w, i);
      v[2 * i] = static_cast<uint32_t>(x);
      v[2 * i + 1] = static_cast<uint32_t>(x >> 32);
    }
    return v[14] == seq && v[15] == door_check(v, seq);
  };
  uint64_t w = 0;
  bool found = true;
  const uint64_t t0 = wall_ticks();
  for (;;) {
    if (poll(&w)) break;
    if (wall_ticks() - t0 > idle) {
      if (lane == 0) {
        sys_st(&hstate[0], kResExiting);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // the host may have posted the entry meanwhile: one more (checked) read decides
      found = false;
      for (int i = 0; i < 4 && !found; ++i) found = poll(&w);
      if (!found && __shfl(static_cast<uint32_t>(__shfl(w, 7)), 0) == seq) {
        // the sequence word is there but the reads kept catching a write: wait for it
        while (!found) found = poll(&w);
      }
      if (lane == 0) sys_st(&hstate[0], found ? kResRunning : kResExited);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  uint64_t w6 = __shfl(w, 6);
  if (!found) w6 = static_cast<uint64_t>(static_cast<uint32_t>(kResStop)) << 32;
  if (!found && lane == 6) w = w6;
  if (broadcast) {
    if (lane < 8 && (found || lane == 6))
      __hip_atomic_store(&dm[kDmEntry + lane], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(&dm[kDmGo], (static_cast<uint64_t>(gen) << 32) | seq, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  if (lane == 0 && found && static_cast<uint32_t>(w6 >> 32) == static_cast<uint32_t>(kResStop))
    sys_st(&hstate[0], kResExited);
  return w;
}

template <class E, bool FULL, bool ONESHOT>
__global__ __launch_bounds__(kCommThreads) void threshold_resident_kernel(CommArgs a, const ResidentDoor* door,
                                                                         uint32_t* hstate, uint64_t* dm,
                                                                         uint32_t seq, uint32_t gen, uint64_t idle) {
  __shared__ uint64_t sh_ent[8];
  __shared__ int sh_clean;
  uint32_t* const ctl = a.ctl[0];
  // the lag gate of round e is open when this single workgroup's round e - 1 gathered every
  // peer's chunks of e - 1: a peer publishes round e - 1 only after it finished round e - 2
  // (its rounds run in order) and published its progress before that, so with trows >= 2
  // every peer is past e - trows. (More workgroups: a peer's workgroup may start e - 1 before
  // its last workgroup of e - 2 published progress.)
  uint32_t prev_epoch = 0;
  bool prev_clean = false;
  for (;; ++seq) {
    if (threadIdx.x < 64) {
      const int lane = static_cast<int>(threadIdx.x);
      uint64_t w = 0;
      bool ok = true;
      if (blockIdx.x == 0) {
        // one workgroup: the entry straight from the door (no device hand-off)
        w = resident_door(door, hstate, dm, seq, gen, idle, gridDim.x > 1);
      } else {
        // the leader answers within `idle` plus one round (each bounded by a.timeout)
        const uint64_t want = (static_cast<uint64_t>(gen) << 32) | seq;
        if (lane == 0) {
          const uint64_t until = wall_ticks() + idle + 2 * a.timeout + 100000000ull;
          while (__hip_atomic_load(&dm[kDmGo], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
            if (wall_ticks() > until) {
              __hip_atomic_fetch_or(&ctl[2], ERR_TIMEOUT_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              ok = false;
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
        }
        ok = __shfl(ok ? 1 : 0, 0) != 0;
        if (ok && lane < 8) w = __hip_atomic_load(&dm[kDmEntry + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!ok && lane == 6) w = static_cast<uint64_t>(static_cast<uint32_t>(kResStop)) << 32;
      }
      if (lane < 8) sh_ent[lane] = w;
      // the round's input was written by kernels that finished before the host posted it:
      // drop what this XCD's caches hold of earlier rounds
      if (lane == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    const uint32_t cmd = static_cast<uint32_t>(sh_ent[6] >> 32);
    if (cmd == static_cast<uint32_t>(kResStop)) break;  // uniform
    const RoundVars rv = launch_vars(
        a, 0, reinterpret_cast<const char*>(sh_ent[0]), reinterpret_cast<char*>(sh_ent[1]),
        reinterpret_cast<int32_t*>(sh_ent[2]), reinterpret_cast<int32_t*>(sh_ent[3]),
        reinterpret_cast<uint32_t*>(sh_ent[4]), reinterpret_cast<uint32_t*>(sh_ent[5]), static_cast<uint32_t>(sh_ent[6]),
        cmd == static_cast<uint32_t>(kResCold) ? 1 : 0,
        (prev_clean && gridDim.x == 1 && a.trows >= 2 && static_cast<uint32_t>(sh_ent[6]) == prev_epoch + 1u) ? 1 : 0,
        1);
    __syncthreads();
    const bool clean = threshold_round<E, FULL, ONESHOT>(a, rv);
    if (threadIdx.x == 0) sh_clean = clean ? 1 : 0;
    // the entry is consumed: the host may reuse its door slot (a PCIe write, kept off the
    // round's critical path - every release waits for the writes before it)
    if (blockIdx.x == 0 && threadIdx.x == 0) sys_st(&hstate[1], seq);
    __syncthreads();
    prev_clean = sh_clean != 0;
    prev_epoch = rv.epoch;
    if (threadIdx.x == 0) {  // the round's counters are reset before any workgroup starts the next
      const uint64_t until = wall_ticks() + a.timeout + 100000000ull;
      while (ld_ctl(&ctl[4]) != rv.epoch && wall_ticks() < until) __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------
// Group resident rounds (xgmi_plane.cc PlaneGroup). Co-located workers of one job (one
// process, one GPU) run their rounds in ONE resident kernel: worker k's slice is grid row
// y = 1 + k and runs k's rounds one after another, exactly as threshold_resident_kernel runs
// one worker's; the slices never wait for each other's turn, so a straggler's slice lags
// while the others run ahead (the protocol's bounded staleness), and no slice can sit in a
// hardware queue behind a co-located peer's spinning round - however many workers share the
// GPU and however few hardware queues the process has (GPU_MAX_HW_QUEUES).
//
// Row 0, workgroup 0, wave 0 is the dispatcher. It alone reads the doors: lanes 8j..8j+7
// read worker j's next 64-B entry (and worker 8 + j's in a second load), so ONE load polls up
// to eight doors. A found entry goes to the worker's slice through its device words (entry,
// then go = gen << 32 | seq) once the slice's previous round ended (its ctl[4] names that
// round's epoch: every workgroup of the slice has read the previous entry), and the door slot
// is released at once (hstate[1]). A STOP entry (the worker leaves the group) ends its slice.
//
// Exit: only the dispatcher decides it, for the whole group - no worker's rounds may be left
// to a kernel queued behind this one. After `idle` ticks with no entry and no round running
// it writes EXITING to the group's state word, fences, and polls every door once more (the
// hosts write an entry, fence, then read the state word): an entry found keeps the kernel
// (RUNNING); otherwise every slice gets STOP and the state becomes EXITED, and the next post
// launches a new kernel. Slices wait for go without a deadline of their own while the
// dispatcher's heartbeat (gdm[0]) advances.
__device__ __forceinline__ void group_dispatch(const CommArgs& a, const GroupResArgs& g) {
  const int lane = static_cast<int>(threadIdx.x);
  const int Y = g.Y;
  const int w = lane & 7;
  // lane-held state: lanes 8j..8j+7 poll worker j (bank 0) and worker 8 + j (bank 1); lane k
  // keeps worker k's control words, its running round's epoch and whether it left
  const uint64_t* dp0 = nullptr;
  const uint64_t* dp1 = nullptr;
  uint32_t nx0 = 0, nx1 = 0;
  uint32_t* myctl = nullptr;
  for (int y = 0; y < Y; ++y) {  // uniform: scalar loads of the arguments
    if ((lane >> 3) == (y & 7)) {
      if (y < 8) {
        dp0 = reinterpret_cast<const uint64_t*>(g.m[y].door);
        nx0 = g.m[y].seq0;
      } else {
        dp1 = reinterpret_cast<const uint64_t*>(g.m[y].door);
        nx1 = g.m[y].seq0;
      }
    }
    if (lane == y) myctl = a.ctl[y];
  }
  uint32_t run_epoch = 0;
  bool busy = false, gone = lane >= Y;
  const uint64_t hb_every = 50000;  // 0.5 ms
  uint64_t t_act = wall_ticks(), t_hb = 0;
  auto poll = [&](uint64_t* v0, uint64_t* v1) {
    *v0 = dp0 != nullptr ? __hip_atomic_load(dp0 + static_cast<uint64_t>(nx0 % kResidentDoors) * 8 + w,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                         : 0ull;
    *v1 = (Y > 8 && dp1 != nullptr) ? __hip_atomic_load(dp1 + static_cast<uint64_t>(nx1 % kResidentDoors) * 8 + w,
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                    : 0ull;
  };
  // worker y's entry in (v0, v1): 1 = a whole entry, 2 = its sequence word only (a read that
  // caught the host mid-write), 0 = nothing. Uniform.
  auto entry_of = [&](int y, uint64_t v0, uint64_t v1, uint32_t* e) -> int {
    const uint64_t v = y < 8 ? v0 : v1;
    const int base = (y & 7) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t x = __shfl(v, base + i);
      e[2 * i] = static_cast<uint32_t>(x);
      e[2 * i + 1] = static_cast<uint32_t>(x >> 32);
    }
    const uint32_t seq = static_cast<uint32_t>(__shfl(static_cast<int>(y < 8 ? nx0 : nx1), base));
    if (e[14] != seq) return 0;
    return e[15] == door_check(e, seq) ? 1 : 2;
  };
  // The entry words are 8-B agent-scope atomic stores (write-through, sc1) and the slices read
  // them with 8-B agent-scope loads: draining them before the go store is the whole release
  // (MI355X_MICROARCH.md, valid forms: 8-B agent atomics both sides) - no L2 write-back.
  auto go = [&](int y, uint32_t seq) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(&g.m[y].dm[kDmGo], (static_cast<uint64_t>(g.gen) << 32) | seq, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  };
  for (;;) {
    const uint64_t now = wall_ticks();
    if (now - t_hb > hb_every) {
      if (lane == 0) __hip_atomic_store(&g.gdm[0], now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t_hb = now;
    }
    uint64_t v0, v1;
    poll(&v0, &v1);  // (the PCIe reads first: the control-word read below overlaps them)
    if (busy) busy = ld_ctl(&myctl[4]) != run_epoch;  // the slice's round ended
    bool pending = false;
    for (int y = 0; y < Y; ++y) {
      if (__shfl(gone ? 1 : 0, y) != 0) continue;
      uint32_t e[16];
      const int st = entry_of(y, v0, v1, e);
      if (st == 0) continue;
      pending = true;
      if (st != 1 || __shfl(busy ? 1 : 0, y) != 0) continue;  // taken once whole / once the slice is free
      const uint32_t seq = e[14];
      const uint64_t word = __shfl(y < 8 ? v0 : v1, (y & 7) * 8 + w);
      if (lane < 8)
        __hip_atomic_store(&g.m[y].dm[kDmEntry + lane], word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      go(y, seq);
      if (lane == 0) sys_st(&g.m[y].hstate[1], seq);  // the door slot is free
      if (static_cast<int32_t>(e[13]) == kResStop) {
        if (lane == y) gone = true;
      } else if (lane == y) {
        busy = true;
        run_epoch = e[12];
      }
      if ((lane >> 3) == (y & 7)) {
        if (y < 8)
          ++nx0;
        else
          ++nx1;
      }
      t_act = now;
    }
    if (__all(gone)) {  // every worker left: nothing more to serve
      if (lane == 0) {  // after every consumed-entry word (the hosts read them once EXITED)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sys_st(&g.gstate[0], kResExited);
      }
      return;
    }
    if (!pending && !__any(busy) && wall_ticks() - t_act > g.idle) {
      if (lane == 0) {
        sys_st(&g.gstate[0], kResExiting);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      bool found = false;
      for (int i = 0; i < 4 && !found; ++i) {
        poll(&v0, &v1);
        for (int y = 0; y < Y && !found; ++y) {
          if (__shfl(gone ? 1 : 0, y) != 0) continue;
          uint32_t e[16];
          found = entry_of(y, v0, v1, e) != 0;
        }
      }
      if (found) {  // posted meanwhile: keep serving
        if (lane == 0) sys_st(&g.gstate[0], kResRunning);
        t_act = wall_ticks();
        continue;
      }
      for (int y = 0; y < Y; ++y) {  // every slice still here leaves
        if (__shfl(gone ? 1 : 0, y) != 0) continue;
        const uint32_t seq = static_cast<uint32_t>(__shfl(static_cast<int>(y < 8 ? nx0 : nx1), (y & 7) * 8));
        // word 6: STOP; word 7: the entry's sequence number (slices check it)
        if (lane == 6 || lane == 7)
          __hip_atomic_store(&g.m[y].dm[kDmEntry + lane],
                             lane == 6 ? static_cast<uint64_t>(static_cast<uint32_t>(kResStop)) << 32 : seq,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        go(y, seq);
      }
      if (lane == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sys_st(&g.gstate[0], kResExited);
      }
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

template <class E, bool FULL, bool ONESHOT>
__global__ __launch_bounds__(kCommThreads) void threshold_group_resident_kernel(CommArgs a, GroupResArgs g) {
  if (blockIdx.y == 0) {  // the dispatcher row: one wave works, the rest leave at once
    if (blockIdx.x == 0 && threadIdx.x < 64) group_dispatch(a, g);
    return;
  }
  const int y = static_cast<int>(blockIdx.y) - 1;
  const GroupResidentMember& m = g.m[y];
  uint32_t* const ctl = a.ctl[y];
  __shared__ uint64_t sh_ent[8];
  __shared__ int sh_clean;
  uint32_t prev_epoch = 0;
  bool prev_clean = false;
  const uint64_t lost = 2 * a.timeout + 100000000ull;  // the dispatcher's heartbeat stopped this long ago
  for (uint32_t seq = m.seq0;; ++seq) {
    if (threadIdx.x < 64) {
      const int lane = static_cast<int>(threadIdx.x);
      uint64_t w = 0;
      bool ok = true;
      // ONE load per poll: lanes 0-7 the entry, lane 8 the go word (the same 128-B line). The
      // entry is taken when go names this kernel's generation and entry `seq`, and the entry
      // names `seq` itself (word 7): a read that caught an older entry is simply repeated.
      const uint64_t want = (static_cast<uint64_t>(g.gen) << 32) | seq;
      // the heartbeat is judged by THIS workgroup's clock only: it counts as stopped when its
      // value has not changed for `lost` local ticks (realtime counters of different XCDs are
      // not comparable - a dispatcher clock a little ahead made `now - hb` wrap)
      uint64_t hb_seen = lane == 0 ? __hip_atomic_load(&g.gdm[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      uint64_t hb_at = wall_ticks();
      for (;;) {
        const uint64_t x = lane < 8    ? __hip_atomic_load(&m.dm[kDmEntry + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : lane == 8 ? __hip_atomic_load(&m.dm[kDmGo], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                       : 0ull;
        const uint64_t cur = __shfl(x, 8);
        if (cur == want && static_cast<uint32_t>(__shfl(x, 7)) == seq) {
          w = x;
          break;
        }
        // a newer kernel's go (generations only grow): this kernel's dispatcher has left and
        // its STOP was overwritten - leave too
        if (static_cast<int32_t>(static_cast<uint32_t>(cur >> 32) - g.gen) > 0) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        int lost_now = 0;
        if (lane == 0) {
          const uint64_t hb = __hip_atomic_load(&g.gdm[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint64_t now = wall_ticks();
          if (hb != hb_seen) {
            hb_seen = hb;
            hb_at = now;
          } else if (now - hb_at > lost) {
            __hip_atomic_fetch_or(&ctl[2], ERR_TIMEOUT_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            lost_now = 1;
          }
        }
        if (__shfl(lost_now, 0) != 0) {
          ok = false;
          break;
        }
      }
      if (!ok && lane == 6) w = static_cast<uint64_t>(static_cast<uint32_t>(kResStop)) << 32;
      if (lane < 8) sh_ent[lane] = w;
      // the round's input was written by kernels that finished before the host posted it
      if (lane == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    const uint32_t cmd = static_cast<uint32_t>(sh_ent[6] >> 32);
    if (cmd == static_cast<uint32_t>(kResStop)) break;  // uniform
    const uint32_t epoch = static_cast<uint32_t>(sh_ent[6]);
    const RoundVars rv{reinterpret_cast<const char*>(sh_ent[0]),
                       reinterpret_cast<char*>(sh_ent[1]),
                       reinterpret_cast<int32_t*>(sh_ent[2]),
                       reinterpret_cast<int32_t*>(sh_ent[3]),
                       reinterpret_cast<uint32_t*>(sh_ent[4]),
                       reinterpret_cast<uint32_t*>(sh_ent[5]),
                       epoch,
                       cmd == static_cast<uint32_t>(kResCold) ? 1 : 0,
                       (prev_clean && gridDim.x == 1 && a.trows >= 2 && epoch == prev_epoch + 1u) ? 1 : 0,
                       1,
                       m.rank,
                       ctl,
                       m.hforce,
                       m.habort,
                       m.split_dec,
                       m.split_ctr,
                       m.split_early,
                       m.stamps == nullptr ? nullptr : m.stamps + static_cast<int64_t>(blockIdx.x) * kPhaseSlots};
    __syncthreads();
    const bool clean = threshold_round<E, FULL, ONESHOT>(a, rv);
    if (threadIdx.x == 0) sh_clean = clean ? 1 : 0;
    __syncthreads();
    prev_clean = sh_clean != 0;
    prev_epoch = epoch;
    if (threadIdx.x == 0) {  // the round's counters are reset before any workgroup starts the next
      const uint64_t until = wall_ticks() + a.timeout + 100000000ull;
      while (ld_ctl(&ctl[4]) != epoch && wall_ticks() < until) __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
  }
}

// One wave: lane k < P stores this rank's progress word into peer k's slab, after a
// system-scope release (everything this rank did before is visible first).
__global__ __launch_bounds__(64) void publish_progress_kernel(CommArgs a, uint32_t value) {
  const int k = static_cast<int>(threadIdx.x);
  if (k < a.P && k != a.rank0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_flag(prog(a, k, a.rank0), value);
  }
}

// the compile-time full-threshold kernel applies (threshold_round FULL), with its one-shot body
static bool full_fast(const CommArgs& a) { return a.full != 0 && a.sub <= 1; }
static bool full_oneshot(const CommArgs& a) { return full_fast(a) && a.oneshot != 0; }

void launch_publish_progress(const CommArgs& a, uint32_t value, hipStream_t s) {
  hipLaunchKernelGGL(publish_progress_kernel, dim3(1), dim3(64), 0, s, a, value);
}

void launch_threshold_resident(const CommArgs& a, int grid, hipStream_t s, DType dt, const ResidentDoor* door,
                               uint32_t* hstate, uint32_t* dm, uint32_t seq, uint32_t gen, uint64_t idle_ticks) {
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    using E = decltype(tag);
    if (full_oneshot(a))
      hipLaunchKernelGGL((threshold_resident_kernel<E, true, true>), dim3(grid), dim3(kCommThreads), 0, s, a, door,
                         hstate, reinterpret_cast<uint64_t*>(dm), seq, gen, idle_ticks);
    else if (full_fast(a))
      hipLaunchKernelGGL((threshold_resident_kernel<E, true, false>), dim3(grid), dim3(kCommThreads), 0, s, a, door,
                         hstate, reinterpret_cast<uint64_t*>(dm), seq, gen, idle_ticks);
    else
      hipLaunchKernelGGL((threshold_resident_kernel<E, false, false>), dim3(grid), dim3(kCommThreads), 0, s, a, door,
                         hstate, reinterpret_cast<uint64_t*>(dm), seq, gen, idle_ticks);
  });
}

void launch_threshold(const CommArgs& a, dim3 grid, hipStream_t s, DType dt) {
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    using E = decltype(tag);
    if (full_oneshot(a))
      hipLaunchKernelGGL((threshold_kernel<E, true, true>), grid, dim3(kCommThreads), 0, s, a);
    else if (full_fast(a))
      hipLaunchKernelGGL((threshold_kernel<E, true, false>), grid, dim3(kCommThreads), 0, s, a);
    else
      hipLaunchKernelGGL((threshold_kernel<E, false, false>), grid, dim3(kCommThreads), 0, s, a);
  });
}

void launch_threshold_group_resident(const CommArgs& a, const GroupResArgs& g, int grid, hipStream_t s, DType dt) {
  const dim3 gd(static_cast<unsigned>(grid), static_cast<unsigned>(g.Y + 1));
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    using E = decltype(tag);
    if (full_oneshot(a))
      hipLaunchKernelGGL((threshold_group_resident_kernel<E, true, true>), gd, dim3(kCommThreads), 0, s, a, g);
    else if (full_fast(a))
      hipLaunchKernelGGL((threshold_group_resident_kernel<E, true, false>), gd, dim3(kCommThreads), 0, s, a, g);
    else
      hipLaunchKernelGGL((threshold_group_resident_kernel<E, false, false>), gd, dim3(kCommThreads), 0, s, a, g);
  });
}

}  // namespace mxar
