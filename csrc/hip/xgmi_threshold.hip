// Threshold (straggler-tolerant, bounded-staleness) fused allreduce over xGMI (gfx950).
//
// The reference's round semantics on the GPU hot path, in one persistent launch per round:
//   thReduce   - a chunk of rank r's block is reduced as soon as `min_reduce` of the P
//                contributions (own included) have arrived; contributions that arrive
//                later are not waited for (AllreduceWorker.scala:116-121, DataBuffer
//                reachThreshold :31-33). Missing contributions count as zeros.
//   thComplete - the round completes once `min_complete` of the P x nch reduced chunks are
//                in; chunks still missing then are output as zeros with count 0
//                (AllreduceWorker.scala:143-145, reachRoundThreshold DataBuffer.scala:69-75).
//   maxLag     - the S/R slots and their flags form a ring of `trows` = maxLag + 1 rows
//                (slab rows 1..trows; row 0 belongs to the lock-step kernels, so a fast
//                rank that moves on to another algorithm never touches a row a lagging
//                rank still reads), indexed by the threshold-round counter ctl[4]; a rank
//                may run up to maxLag rounds ahead of the slowest
//                peer (the worker's lag ring, AllreduceWorker.scala:59-73). Before
//                writing row e % rows a rank waits until every peer has finished the
//                round that last used it (progress words), so a row is never overwritten
//                while a lagging peer still reads it.
//   count      - per output chunk, how many contributions were summed (ReduceBlock.count,
//                AllreduceMessage.scala:19); 0 marks a chunk that was not completed.
// Decisions are made per chunk from a snapshot of the arrival flags taken when the count
// first reaches the threshold (all contributions present at that instant are summed).
#include <hip/hip_runtime.h>

#include "xgmi_device.h"

namespace mxar {

namespace {

__device__ __forceinline__ uint32_t* prog(const CommArgs& a, int k, int s) {
  return reinterpret_cast<uint32_t*>(a.base[k]) + static_cast<int64_t>(2 * a.rows * a.P) * a.maxch + a.P + s;
}
__device__ __forceinline__ uint32_t* f2c(const CommArgs& a, int k, int rs, int c) {  // rs = row * P + src
  return reinterpret_cast<uint32_t*>(a.base[k]) + static_cast<int64_t>(2 * a.rows * a.P) * a.maxch + 2 * a.P +
         static_cast<int64_t>(rs) * a.maxch + c;
}

// Sum the sources in `mask` (fixed order s = 0..P-1, fp32), store to own output and to
// every peer's R slot. Source r is the rank's own input. The mask is wave-uniform.
template <class E>
__device__ __forceinline__ void reduce_masked(const CommArgs& a, int P, int r, uint32_t mask, const char* own_in,
                                              const char* S, int64_t slot, char* own_out, int64_t roff,
                                              int64_t len, bool wt_out, float scale) {
  const int64_t npk = len / E::ELEMS;
  constexpr int U = 2;
  int64_t i = threadIdx.x;
  for (; i + (U - 1) * kCommThreads < npk; i += U * kCommThreads) {
    Acc<E> acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u].zero();
    for (int s = 0; s < P; ++s) {
      if (!((mask >> s) & 1u)) continue;
      const __amdgpu_buffer_rsrc_t rs = slab_rsrc(s == r ? own_in : S + s * slot);
      Pack16 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld16_sc1(rs, static_cast<uint32_t>((i + u * kCommThreads) * 16));
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u].add(v[u]);
    }
    Pack16 o[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (scale != 1.f) acc[u].scale(scale);
      o[u] = acc[u].pack();
    }
    for (int k = 0; k < P; ++k) {
      char* d = k == r ? own_out : a.base[k] + roff;
      if (k == r && !wt_out) {
#pragma unroll
        for (int u = 0; u < U; ++u) st16(d + (i + u * kCommThreads) * 16, o[u]);
      } else {
        const __amdgpu_buffer_rsrc_t rd = slab_rsrc(d);
#pragma unroll
        for (int u = 0; u < U; ++u) st16_wt(rd, static_cast<uint32_t>((i + u * kCommThreads) * 16), o[u]);
      }
    }
  }
  for (; i < npk; i += kCommThreads) {
    Acc<E> acc;
    acc.zero();
    for (int s = 0; s < P; ++s)
      if ((mask >> s) & 1u) acc.add(ld16_sc1(slab_rsrc(s == r ? own_in : S + s * slot), static_cast<uint32_t>(i * 16)));
    if (scale != 1.f) acc.scale(scale);
    const Pack16 o = acc.pack();
    for (int k = 0; k < P; ++k) {
      char* d = k == r ? own_out : a.base[k] + roff;
      if (k == r && !wt_out)
        st16(d + i * 16, o);
      else
        st16_wt(slab_rsrc(d), static_cast<uint32_t>(i * 16), o);
    }
  }
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len) {
    float acc = 0.f;
    for (int s = 0; s < P; ++s)
      if ((mask >> s) & 1u) acc += ld_scalar_sc1<E>(slab_rsrc(s == r ? own_in : S + s * slot), t);
    acc *= scale;
    for (int k = 0; k < P; ++k) {
      char* d = k == r ? own_out : a.base[k] + roff;
      if (k == r && !wt_out)
        Scalar<E>::store(d, t, acc);
      else
        st_scalar_wt<E>(slab_rsrc(d), t, acc);
    }
  }
}

template <class E>
__device__ __forceinline__ void zero_fill(char* dst, int64_t len) {
  const int64_t npk = len / E::ELEMS;
  Pack16 z;
  z[0] = z[1] = z[2] = z[3] = 0u;
  for (int64_t i = threadIdx.x; i < npk; i += kCommThreads) st16(dst + i * 16, z);
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len) Scalar<E>::store(dst, t, 0.f);
}

}  // namespace

template <class E>
__global__ __launch_bounds__(kCommThreads) void threshold_kernel(CommArgs a) {
  constexpr int es = 16 / E::ELEMS;
  __shared__ uint32_t sh_mask;
  __shared__ int sh_flag;
  const int P = a.P;
  const int y = blockIdx.y;
  const int r = a.rank0 + y;
  const char* const in = a.in[y];
  char* const out = a.out[y];
  uint32_t* const ctl = a.ctl[y];
  // threshold rounds count separately (ctl[4]); flags and progress words carry this count
  const uint32_t epoch = __hip_atomic_load(&ctl[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int row = 1 + static_cast<int>(epoch % static_cast<uint32_t>(a.trows));
  const int G = gridDim.x;
  const int64_t slot = a.slot_bytes;
  const int64_t rowS = a.off_S + static_cast<int64_t>(row) * P * slot;
  const int64_t rowR = a.off_R + static_cast<int64_t>(row) * P * slot;
  uint32_t* err = &ctl[2];
  const bool rel = a.fence & 1, acq = a.fence & 2;
  const int Pm1 = P > 1 ? P - 1 : 1;
  int32_t* const counts = a.counts ? a.counts + static_cast<int64_t>(y) * P * a.nch : nullptr;

  if (a.delay && r == a.delay_rank) {  // straggler simulation (tests)
    const uint64_t until = wall_ticks() + a.delay;
    while (wall_ticks() < until) __builtin_amdgcn_s_sleep(8);
  }
  const uint64_t deadline = wall_ticks() + a.timeout;

  // Lag gate: every peer has finished the round that last used row `row` of its slab
  // (progress words live in OUR slab, written by the peers at the end of each round).
  wait_flags([&](int k) -> const uint32_t* { return k == r ? nullptr : prog(a, r, k); }, P,
             epoch - static_cast<uint32_t>(a.trows), deadline, err, ERR_TIMEOUT_LAG, acq);

  // Phase 1 - ScatterBlock into the owners' row slots
  const int nu = (P - 1) * a.nch;
  for (int u = blockIdx.x; u < nu; u += G) {
    const int c = u / Pm1;
    const int j = (r + 1 + u % Pm1) % P;
    const int64_t bstart = static_cast<int64_t>(j) * a.block;
    const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
    const int64_t len = clamp_len(clamp_len(a.n - bstart, a.block) - cstart, a.chunk);
    if (len > 0) copy_to_slab<E>(a.base[j] + rowS + r * slot + cstart * es, in + (bstart + cstart) * es, len);
    publish_flags([&](int) { return f1(a, j, row * P + r, c); }, 1, epoch, rel);
  }

  // Phase 2 - reduce own chunk c once min_reduce contributions are in (own one included)
  const int64_t bstart_own = static_cast<int64_t>(r) * a.block;
  const int64_t blen_own = clamp_len(a.n - bstart_own, a.block);
  const uint32_t all = P >= 32 ? 0xffffffffu : ((1u << P) - 1u);
  for (int c = blockIdx.x; c < a.nch; c += G) {
    const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
    const int64_t len = clamp_len(blen_own - cstart, a.chunk);
    if (threadIdx.x < 64) {
      const int s = static_cast<int>(threadIdx.x);
      const uint32_t* f = (s < P && s != r) ? f1(a, r, row * P + s, c) : nullptr;
      bool in_ = (s == r) || (f != nullptr && reached(ld_flag(f), epoch));
      uint32_t m = static_cast<uint32_t>(__ballot(in_)) & all;
      bool timed_out = false;
      while (__popc(m) < a.min_reduce && m != all) {
        __builtin_amdgcn_s_sleep(1);
        if (!in_ && f != nullptr) in_ = reached(ld_flag(f), epoch);
        m = static_cast<uint32_t>(__ballot(in_)) & all;
        if (wall_ticks() > deadline) {
          timed_out = true;
          break;
        }
      }
      if (threadIdx.x == 0) {
        sh_mask = m;
        if (timed_out) __hip_atomic_fetch_or(err, ERR_TIMEOUT_SCATTER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const uint32_t mask = sh_mask;
    const int cnt = __popc(mask);
    const float sc = (a.rescale && cnt > 0) ? a.scale * static_cast<float>(P) / static_cast<float>(cnt) : a.scale;
    if (len > 0)
      reduce_masked<E>(a, P, r, mask, in + (bstart_own + cstart) * es, a.base[r] + rowS + cstart * es, slot,
                       out + (bstart_own + cstart) * es, rowR + r * slot + cstart * es, len, a.fence & 1, sc);
    if (threadIdx.x < static_cast<unsigned>(P) && static_cast<int>(threadIdx.x) != r)
      st_flag(f2c(a, static_cast<int>(threadIdx.x), row * P + r, c), static_cast<uint32_t>(cnt));
    if (threadIdx.x == 0) {
      if (counts) counts[static_cast<int64_t>(r) * a.nch + c] = cnt;
      __hip_atomic_fetch_add(&ctl[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    publish_flags([&](int k) -> uint32_t* { return k == r ? nullptr : f2(a, k, row * P + r, c); }, P, epoch, rel);
  }

  // Phase 3 - gather the other owners' chunks; once min_complete chunks of the round are
  // in, chunks still missing are given up (zeros, count 0). Units of this workgroup are
  // polled round-robin so a late chunk never blocks the count of an early one.
  int mine = 0;
  for (int u = blockIdx.x; u < nu; u += G) ++mine;
  uint64_t pending = mine >= 64 ? ~0ull : ((1ull << mine) - 1ull);
  bool gave_up = false;
  while (pending) {
    bool progressed = false;
    for (int i = 0; i < mine; ++i) {
      if (!((pending >> i) & 1ull)) continue;
      const int u = blockIdx.x + i * G;
      const int c = u / Pm1;
      const int j = (r + 1 + u % Pm1) % P;
      if (threadIdx.x == 0) sh_flag = reached(ld_flag(f2(a, r, row * P + j, c)), epoch) ? 1 : 0;
      __syncthreads();
      const bool arrived = sh_flag != 0;
      __syncthreads();
      if (!arrived) continue;
      if (acq && threadIdx.x < 64) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      __syncthreads();
      const int64_t bstart = static_cast<int64_t>(j) * a.block;
      const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
      const int64_t len = clamp_len(clamp_len(a.n - bstart, a.block) - cstart, a.chunk);
      if (len > 0) copy_from_slab<E>(out + (bstart + cstart) * es, a.base[r] + rowR + j * slot + cstart * es, len);
      if (threadIdx.x == 0) {
        if (counts) counts[static_cast<int64_t>(j) * a.nch + c] = static_cast<int32_t>(ld_flag(f2c(a, r, row * P + j, c)));
        __hip_atomic_fetch_add(&ctl[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      pending &= ~(1ull << i);
      progressed = true;
    }
    if (!pending || progressed) continue;
    if (threadIdx.x == 0) {
      const int64_t done = __hip_atomic_load(&ctl[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int give = done >= a.min_complete ? 1 : 0;
      if (!give && wall_ticks() > deadline) {
        __hip_atomic_fetch_or(err, ERR_TIMEOUT_REDUCE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        give = 1;
      }
      sh_flag = give;
    }
    __syncthreads();
    gave_up = sh_flag != 0;
    __syncthreads();
    if (gave_up) break;
    __builtin_amdgcn_s_sleep(2);
  }
  if (gave_up) {
    for (int i = 0; i < mine; ++i) {
      if (!((pending >> i) & 1ull)) continue;
      const int u = blockIdx.x + i * G;
      const int c = u / Pm1;
      const int j = (r + 1 + u % Pm1) % P;
      const int64_t bstart = static_cast<int64_t>(j) * a.block;
      const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
      const int64_t len = clamp_len(clamp_len(a.n - bstart, a.block) - cstart, a.chunk);
      if (len > 0) zero_fill<E>(out + (bstart + cstart) * es, len);
      if (threadIdx.x == 0 && counts) counts[static_cast<int64_t>(j) * a.nch + c] = 0;
    }
  }

  // Round end: the last workgroup resets the completion counter, advances the round count and
  // tells every peer that this rank is done with row `row` (all its reads happened
  // before the workgroups' tickets).
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(&ctl[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == static_cast<uint32_t>(G) - 1) {
      __hip_atomic_store(&ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctl[3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctl[4], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      for (int k = 0; k < P; ++k)
        if (k != r) st_flag(prog(a, k, r), epoch);
    }
  }
}

void launch_threshold(const CommArgs& a, dim3 grid, hipStream_t s, DType dt) {
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    hipLaunchKernelGGL(threshold_kernel<decltype(tag)>, grid, dim3(kCommThreads), 0, s, a);
  });
}

}  // namespace mxar
