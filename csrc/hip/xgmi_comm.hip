// Fused push-based allreduce over xGMI (gfx950). See xgmi_comm.h for the protocol map to
// the reference (AllreduceWorker.scala scatter/reduce/broadcast/complete).
//
// Slab layout (identical offsets on every rank, fine-grained device memory - the kind HSA
// makes coherent across agents during a kernel; MXAR_SLAB_MEM=uncached|coarse exist for
// study only: uncached slabs showed stale reads on MI355X, tests/test_comm_gpu.py stress):
//   [F1: P x maxch u32][F2: P x maxch u32][FB: P u32]  pad to 64 KiB
//   [S : P slots x slot_bytes]   S_k[s] = contribution of rank s to rank k's block
//   [R : P slots x slot_bytes]   R_k[j] = reduced block j, pushed by its owner j
// Flags hold the epoch of the launch that wrote them; epochs come from a device counter
// so launches replay correctly under hipGraph capture.
#include "../core/env.h"
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <string>

#include "../core/data_buffer.h"
#include "../core/trace.h"
#include "xgmi_device.h"

namespace mxar {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
  }
}

// ---------------------------------------------------------------------------------
// Two-shot: direct reduce-scatter (push) + direct all-gather (push), one launch.
// ---------------------------------------------------------------------------------
template <class E, int PT>
__global__ __launch_bounds__(kCommThreads) void twoshot_kernel(CommArgs a) {
  constexpr int es = 16 / E::ELEMS;
  const int P = PT > 0 ? PT : a.P;
  const int y = blockIdx.y;
  const int r = a.rank0 + y;
  const char* const in = a.in[y];
  char* const out = a.out[y];
  uint32_t* const ctl = a.ctl[y];
  const uint32_t epoch = launch_epoch(ctl);
  const uint64_t deadline = wall_ticks() + a.timeout;
  const int G = gridDim.x;
  const int64_t slot = a.slot_bytes;
  uint32_t* err = &ctl[2];
  const bool rel = a.fence & 1, acq = a.fence & 2;
  const int Pm1 = P > 1 ? P - 1 : 1;
  const int nu = (P - 1) * a.nch;
  __shared__ uint64_t ps_lds[kPhaseSlots];
  PhaseStamps ps(a, ps_lds);

  // Phase 1 - ScatterBlock: push chunk c of block j to its owner j (rotated dest order,
  // AllreduceWorker.scala:194-209), so concurrent workgroups load all links. `sgroup`
  // consecutive chunks of one destination travel as ONE unit (one contiguous copy, one
  // release), each chunk keeping its own flag: small chunks pipeline the reduce, grouped
  // copies keep the scatter at copy speed ("flat" geometry, launch_segment).
  const int gs = a.sgroup > 1 ? a.sgroup : 1;
  const int nsu = Pm1 * ((a.nch + gs - 1) / gs);
  if (static_cast<int>(blockIdx.x) < nsu) entry_guard(a, ctl, r, epoch, kHazS, -1, deadline, err);  // block-uniform
  for (int u = blockIdx.x; u < nsu; u += G) {
    const int c0 = (u / Pm1) * gs;
    const int ncg = a.nch - c0 < gs ? a.nch - c0 : gs;
    const int j = (r + 1 + u % Pm1) % P;
    const int64_t bstart = static_cast<int64_t>(j) * a.block;
    const int64_t cstart = static_cast<int64_t>(c0) * a.chunk;
    const int64_t len = clamp_len(clamp_len(a.n - bstart, a.block) - cstart, static_cast<int64_t>(ncg) * a.chunk);
    if (len > 0 && unit_in_bounds(a, cstart * es, len * es, c0 + ncg - 1, err))
      copy_to_slab<E>(a.base[j] + a.off_S + r * slot + cstart * es, in + (bstart + cstart) * es, len);
    publish_flags([&](int i) { return f1(a, j, r, c0 + i); }, ncg, epoch, rel);
  }

  ps.mark(1);
  // Phase 2 - reduce own block once all P contributions of a chunk have arrived
  // (thReduce = 1), then ReduceBlock-broadcast the sum into every rank's R slot. A chunk
  // is reduced in `sub` pieces by different workgroups so that phase 2 has as many
  // units as phases 1 and 3 (each piece pays one acquire and one release). Units go to
  // workgroups by a static blockIdx stride (a counter-driven walk measured +1 % at 8 logical
  // ranks and slower at 2 - profiles/round4 - and was removed in round 6).
  const int64_t bstart_own = static_cast<int64_t>(r) * a.block;
  const int64_t blen_own = clamp_len(a.n - bstart_own, a.block);
  const int nu2 = a.nch * a.sub;
  for (int u = blockIdx.x; u < nu2; u += G) {
    const int c = u / a.sub;
    const int q = u % a.sub;
    const int64_t cbeg = static_cast<int64_t>(c) * a.chunk;
    const int64_t qbeg = static_cast<int64_t>(q) * a.subchunk;
    const int64_t cstart = cbeg + qbeg;
    const int64_t len = clamp_len(clamp_len(blen_own - cbeg, a.chunk) - qbeg, a.subchunk);
    const uint64_t tw = ps.now();
    wait_flags([&](int s) -> const uint32_t* { return s == r ? nullptr : f1(a, r, s, c); }, P, epoch, deadline, err,
               ERR_TIMEOUT_SCATTER, acq);
    ps.add(2, tw);
    ps.count(6);
    if (len > 0 && unit_in_bounds(a, cstart * es, len * es, u, err)) {
      const char* own_in = in + (bstart_own + cstart) * es;
      const char* S = a.base[r] + a.off_S + cstart * es;
      char* own_out = out + (bstart_own + cstart) * es;
      const int64_t roff = a.off_R + r * slot + cstart * es;
      const RedSrc src{own_in, S, slot, r};
      reduce_to<E, PT>(P, src, P, r, [&](int k) -> char* { return k == r ? own_out : a.base[k] + roff; }, len,
                       a.scale, a.fence & 1);
    }
    publish_flags([&](int k) -> uint32_t* { return k == r ? nullptr : f2(a, k, r, u); }, P, epoch, rel);
  }

  ps.mark(3);
  read_delay(a, r);
  // Phase 3 - complete: gather the other owners' reduced chunks into the output. The
  // workgroup's units are polled together (wave 0, one lane per unit, up to 64 at a time)
  // and copied in ARRIVAL order: owners finish their reduces at different times, and a
  // workgroup waiting on its units one by one idles behind the latest of them while others
  // are ready (the threshold kernel's gather, which does this, was 13 % faster at 8 x 64 MiB
  // - profiles/round3/README.md).
  auto gather_unit = [&](int u) {
    const int c = u / Pm1;
    const int j = (r + 1 + u % Pm1) % P;
    const int64_t bstart = static_cast<int64_t>(j) * a.block;
    const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
    const int64_t len = clamp_len(clamp_len(a.n - bstart, a.block) - cstart, a.chunk);
    ps.count(7);
    if (len > 0 && unit_in_bounds(a, cstart * es, len * es, c, err))
      copy_from_slab<E>(out + (bstart + cstart) * es, a.base[r] + a.off_R + j * slot + cstart * es, len);
  };
  {
    __shared__ uint64_t arrived;
    __shared__ int late_s;
    const int mine = blockIdx.x < static_cast<unsigned>(nu) ? (nu - 1 - static_cast<int>(blockIdx.x)) / G + 1 : 0;
    for (int w0 = 0; w0 < mine; w0 += 64) {
      const int wn = mine - w0 < 64 ? mine - w0 : 64;
      uint64_t pending = wn == 64 ? ~0ull : ((1ull << wn) - 1ull);  // uniform across the workgroup
      const uint64_t tw = ps.now();
      while (pending) {
        if (threadIdx.x < 64) {
          const int lane = static_cast<int>(threadIdx.x);
          bool arr = false;
          if ((pending >> lane) & 1ull) {
            const int u = static_cast<int>(blockIdx.x) + (w0 + lane) * G;
            const int c = u / Pm1;
            const int j = (r + 1 + u % Pm1) % P;
            arr = true;
            for (int q = 0; q < a.sub && arr; ++q) arr = reached(ld_flag(f2(a, r, j, c * a.sub + q)), epoch);
          }
          const uint64_t m = __ballot(arr);
          const bool late = m == 0 && wall_ticks() > deadline;
          if (late && lane == 0) __hip_atomic_fetch_or(err, ERR_TIMEOUT_REDUCE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if (m && acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope, once per batch
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0) {
            arrived = m;
            late_s = late ? 1 : 0;
          }
        }
        __syncthreads();
        uint64_t m = arrived & pending;
        const bool late = late_s != 0;
        __syncthreads();
        if (late) break;  // the rest is given up (error word set, no data moved)
        if (!m) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        pending &= ~m;
        while (m) {
          const int i = __ffsll(static_cast<long long>(m)) - 1;
          m &= m - 1;
          gather_unit(static_cast<int>(blockIdx.x) + (w0 + i) * G);
        }
      }
      ps.add(4, tw);
    }
  }
  ps.mark(5);
  ps.flush();
  finish_launch_done(a, ctl, epoch, r, kHazR);  // peers may still gather from R
}

// ---------------------------------------------------------------------------------
// One-shot (latency path): every rank pushes its whole input into every peer's S slot,
// then reduces all P contributions locally - one xGMI hop instead of two.
// A push unit reads input chunk c ONCE and writes it to all P-1 peers, then publishes
// F1_k[r][c] for every k INCLUDING itself: the own flag means "chunk c of my input has
// been read", which the reduce of chunk c waits for before it may overwrite the input
// (in-place). The reduce reads its own contribution straight from the input.
// ---------------------------------------------------------------------------------
template <class E>
__device__ __forceinline__ void push_to_peers(const CommArgs& a, int P, int r, int64_t slot_off, const char* src,
                                              int64_t len) {
  const int64_t npk = len / E::ELEMS;
  const __amdgpu_buffer_rsrc_t rs = slab_rsrc(src);
  int64_t i = threadIdx.x;
  constexpr int U = 2;
  for (; i + (U - 1) * kCommThreads < npk; i += U * kCommThreads) {
    Pack16 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16_nt(rs, static_cast<uint32_t>((i + u * kCommThreads) * 16));
    for (int k = 0; k < P; ++k) {
      if (k == r) continue;
      const __amdgpu_buffer_rsrc_t rd = slab_rsrc(a.base[k] + slot_off);
#pragma unroll
      for (int u = 0; u < U; ++u) st16_wt(rd, static_cast<uint32_t>((i + u * kCommThreads) * 16), v[u]);
    }
  }
  for (; i < npk; i += kCommThreads) {
    const Pack16 v = ld16_nt(rs, static_cast<uint32_t>(i * 16));
    for (int k = 0; k < P; ++k)
      if (k != r) st16_wt(slab_rsrc(a.base[k] + slot_off), static_cast<uint32_t>(i * 16), v);
  }
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len)
    for (int k = 0; k < P; ++k)
      if (k != r) copy_scalar_wt<E>(slab_rsrc(a.base[k] + slot_off), src, t);
}

template <class E, int PT>
__global__ __launch_bounds__(kCommThreads) void oneshot_kernel(CommArgs a) {
  constexpr int es = 16 / E::ELEMS;
  const int P = PT > 0 ? PT : a.P;
  const int y = blockIdx.y;
  const int r = a.rank0 + y;
  const char* const in = a.in[y];
  char* const out = a.out[y];
  uint32_t* const ctl = a.ctl[y];
  const uint32_t epoch = launch_epoch(ctl);
  const uint64_t deadline = wall_ticks() + a.timeout;
  const int G = gridDim.x;
  const int64_t slot = a.slot_bytes;
  uint32_t* err = &ctl[2];
  const bool rel = a.fence & 1, acq = a.fence & 2;
  // slots alternate between the S and R regions by epoch parity: a fast rank's next one-shot
  // pushes into the region its peers are NOT reading (no guard poll between one-shots)
  const bool odd = epoch & 1u;
  const int64_t region_off = odd ? a.off_R : a.off_S;
  const uint32_t region = odd ? kHazR : kHazS;
  if (static_cast<int>(blockIdx.x) < a.nch) entry_guard(a, ctl, r, epoch, region, -1, deadline, err);
  for (int c = blockIdx.x; c < a.nch; c += G) {
    const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
    const int64_t len = clamp_len(a.n - cstart, a.chunk);
    if (len > 0 && unit_in_bounds(a, cstart * es, len * es, c, err))
      push_to_peers<E>(a, P, r, region_off + r * slot + cstart * es, in + cstart * es, len);
    publish_flags([&](int k) { return f1(a, k, r, c); }, P, epoch, rel);
  }
  read_delay(a, r);
  for (int c = blockIdx.x; c < a.nch; c += G) {
    const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
    const int64_t len = clamp_len(a.n - cstart, a.chunk);
    wait_flags([&](int s) -> const uint32_t* { return f1(a, r, s, c); }, P, epoch, deadline, err, ERR_TIMEOUT_SCATTER,
               acq);
    if (len > 0 && unit_in_bounds(a, cstart * es, len * es, c, err)) {
      const RedSrc src{in + cstart * es, a.base[r] + region_off + cstart * es, slot, r};
      char* o = out + cstart * es;
      reduce_to<E, PT>(P, src, 1, 0, [&](int) -> char* { return o; }, len, a.scale, a.fence & 1);
    }
  }
  finish_launch_done(a, ctl, epoch, r, region);  // peers may still reduce from this region
}

// ---------------------------------------------------------------------------------
// Ring (BASELINE config 3's algorithm, kept for comparison and for topologies where only
// neighbour links are fast): reduce-scatter in P-1 hops + all-gather in P-1 hops, every
// hop a push into the next rank's slab. Each workgroup owns chunk c of every block and
// carries it around the whole ring, so all chunks are pipelined around the ring at once.
//   RS step s (0..P-2): send partial of block (r-s) into next's S[s][c], flag F1_next[s][c]
//                       (step 0 sends the raw input; step s>0 first adds S_r[s-1][c]).
//   final RS          : block (r+1) = S_r[P-2][c] + in[(r+1)][c], scaled once, to out and
//                       into next's R[0][c], flag F2_next[0][c].
//   AG step t (0..P-2): R_r[t][c] = block (r-t): copy to out, forward into next's R[t+1].
// Partial sums travel in fp32 whatever the element type (S slots hold fp32; a bf16 input is
// widened on the first hop), so a bf16 ring is rounded ONCE, at the final RS hop - as the
// two-shot is. For 16-bit types that costs 2x bytes on the RS hops and halves
// the elements one launch carries (XgmiComm::run segments by slot_bytes / 4 per block).
// Slot reuse across launches is safe: rank r's predecessor can only start the next launch
// after it received every block of this one, which transitively follows every read r
// makes of its S/R slots. One xGMI link per direction per rank carries the traffic.
// ---------------------------------------------------------------------------------
template <class E>
__device__ __forceinline__ void copy_slab_fwd(char* out, char* next_slab, const char* slab_src, int64_t len) {
  const int64_t npk = len / E::ELEMS;
  const __amdgpu_buffer_rsrc_t rs = slab_rsrc(slab_src);
  const __amdgpu_buffer_rsrc_t ro = slab_rsrc(out);
  const bool fwd = next_slab != nullptr;
  const __amdgpu_buffer_rsrc_t rn = slab_rsrc(fwd ? next_slab : out);
  int64_t i = threadIdx.x;
  constexpr int U = 4;
  for (; i + (U - 1) * kCommThreads < npk; i += U * kCommThreads) {
    Pack16 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16_nt(rs, static_cast<uint32_t>((i + u * kCommThreads) * 16));
#pragma unroll
    for (int u = 0; u < U; ++u) st16_wt(ro, static_cast<uint32_t>((i + u * kCommThreads) * 16), v[u]);
    if (fwd) {
#pragma unroll
      for (int u = 0; u < U; ++u) st16_wt(rn, static_cast<uint32_t>((i + u * kCommThreads) * 16), v[u]);
    }
  }
  for (; i < npk; i += kCommThreads) {
    const Pack16 v = ld16_nt(rs, static_cast<uint32_t>(i * 16));
    st16_wt(ro, static_cast<uint32_t>(i * 16), v);
    if (fwd) st16_wt(rn, static_cast<uint32_t>(i * 16), v);
  }
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len) {
    const float x = ld_scalar_nt<E>(rs, t);
    st_scalar_wt<E>(ro, t, x);
    if (fwd) st_scalar_wt<E>(rn, t, x);
  }
}

// One ring hop. `partial` (a WT-typed slab slot, null on the first hop) + `in` (element type
// E), summed in fp32 -> either the next partial (`fwd_p`, write-through into the next rank's S
// slot, rounded to WT) or, on the final hop, scale x sum rounded once to E into `out` and the
// next rank's R slot (`fwd_e`). WT = F32 for a 16-bit E is the exact wire (partials travel
// in fp32, E::ELEMS / 4 fp32 packs per E pack); WT = E is the element-type wire (half the RS
// bytes, one extra rounding per intermediate hop). Two steps in flight per lane.
template <class E, class WT, int U>
__device__ __forceinline__ void ring_hop(const char* partial, const char* in, char* fwd_p, char* out, char* fwd_e,
                                         int64_t len, float scale) {
  constexpr bool wide = WT::ELEMS != E::ELEMS;
  constexpr int NP = wide ? E::ELEMS / 4 : 1;  // partial packs per E pack
  const int64_t npk = len / E::ELEMS;
  const bool has_p = partial != nullptr;
  const __amdgpu_buffer_rsrc_t rp = slab_rsrc(has_p ? partial : in);
  const __amdgpu_buffer_rsrc_t ri = slab_rsrc(in);
  const __amdgpu_buffer_rsrc_t rf = slab_rsrc(fwd_p != nullptr ? fwd_p : in);
  const __amdgpu_buffer_rsrc_t ro = slab_rsrc(out != nullptr ? out : in);
  const __amdgpu_buffer_rsrc_t re = slab_rsrc(fwd_e != nullptr ? fwd_e : in);
  // fp32 partial packs (wide wire) are laid out in planes of kCommThreads packs: for each run
  // of 256 E packs, NP planes of 256 fp32 packs - so every load / store instruction of a wave
  // covers 1 KiB of consecutive bytes (pack h of lane l at plane h, slot l). The plain layout
  // (lane l's NP packs side by side) gave each instruction every other 16 B of 2 KiB: twice
  // the lines per instruction, each half written. The last, short run is packed the same way
  // with `rows` slots per plane, so a chunk's partial stays inside its len x 4 bytes. Writer
  // and reader of a hop run this same function over the same len: the layout is private to
  // the ring's S slots.
  auto poff = [&](int64_t i, int h) -> uint32_t {
    const int64_t run = i / kCommThreads;
    const int64_t lane = i - run * kCommThreads;
    const int64_t left = npk - run * kCommThreads;
    const int64_t rows = left < kCommThreads ? left : kCommThreads;
    return static_cast<uint32_t>((run * kCommThreads * NP + h * rows + lane) * 16);
  };
  auto step = [&](int64_t i0, int nu) {
    Pack16 xv[U], pv[U][NP];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= nu) break;
      const int64_t i = i0 + u * kCommThreads;
      xv[u] = ld16_nt(ri, static_cast<uint32_t>(i * 16));
      if (has_p) {
#pragma unroll
        for (int h = 0; h < NP; ++h) pv[u][h] = ld16_nt(rp, wide ? poff(i, h) : static_cast<uint32_t>(i * 16));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= nu) break;
      const int64_t i = i0 + u * kCommThreads;
      Acc<E> acc;
      acc.zero();
      if (has_p) {
        if constexpr (wide) {
#pragma unroll
          for (int h = 0; h < NP; ++h)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc.v[4 * h + q] = __uint_as_float(pv[u][h][q]);
        } else {
          acc.add(pv[u][0]);
        }
      }
      acc.add(xv[u]);
      if (fwd_p != nullptr) {
        if constexpr (wide) {
#pragma unroll
          for (int h = 0; h < NP; ++h) {
            Pack16 o;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = __float_as_uint(acc.v[4 * h + q]);
            st16_wt(rf, poff(i, h), o);
          }
        } else {
          st16_wt(rf, static_cast<uint32_t>(i * 16), acc.pack());
        }
      } else {
        if (scale != 1.f) acc.scale(scale);
        const Pack16 o = acc.pack();
        st16_wt(ro, static_cast<uint32_t>(i * 16), o);
        if (fwd_e != nullptr) st16_wt(re, static_cast<uint32_t>(i * 16), o);
      }
    }
  };
  int64_t i = threadIdx.x;
  for (; i + (U - 1) * kCommThreads < npk; i += U * kCommThreads) step(i, U);
  for (; i < npk; i += kCommThreads) step(i, 1);
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len) {  // ragged tail: one element per lane
    float acc = (has_p ? ld_scalar_nt<WT>(rp, t) : 0.f) + ld_scalar_nt<E>(ri, t);
    if (fwd_p != nullptr) {
      st_scalar_wt<WT>(rf, t, acc);
    } else {
      acc *= scale;
      st_scalar_wt<E>(ro, t, acc);
      if (fwd_e != nullptr) st_scalar_wt<E>(re, t, acc);
    }
  }
}

// The workgroup's chunks are walked STEP-MAJOR: hop s of every chunk the workgroup owns
// (c = blockIdx.x + k * G) before hop s + 1 of any. The wait for chunk c at hop s then finds
// the predecessor's hop s - 1 of c long done (it was issued K - 1 chunks earlier), so flag
// latency and the ranks' jitter hide behind data movement instead of adding up over the
// 2 (P - 1) dependent hops of a chunk-major walk (round 3: 0.56 of the copy roofline at
// 8 logical ranks x 256 MiB bf16). Chunks per workgroup: XgmiComm ring_depth_.
template <class E, class WT, int U>
__global__ __launch_bounds__(kCommThreads) void ring_kernel(CommArgs a) {
  constexpr int es = 16 / E::ELEMS;
  constexpr int ws = 16 / WT::ELEMS;  // wire bytes per element of a reduce-scatter partial
  const int P = a.P;
  const int y = blockIdx.y;
  const int r = a.rank0 + y;
  const int nxt = (r + 1) % P;
  const char* const in = a.in[y];
  char* const out = a.out[y];
  uint32_t* const ctl = a.ctl[y];
  const uint32_t epoch = launch_epoch(ctl);
  const uint64_t deadline = wall_ticks() + a.timeout;
  const int64_t slot = a.slot_bytes;
  const int G = gridDim.x;
  uint32_t* err = &ctl[2];
  const bool rel = a.fence & 1, acq = a.fence & 2;
  __shared__ uint64_t ps_lds[kPhaseSlots];
  PhaseStamps ps(a, ps_lds);  // ring: [1] = end of the reduce-scatter hops, [2]/[4] = waits in RS / AG
  if (static_cast<int>(blockIdx.x) < a.nch) entry_guard(a, ctl, r, epoch, kHazS | kHazR, nxt, deadline, err);
  auto cst = [&](int c) { return static_cast<int64_t>(c) * a.chunk; };
  auto blen = [&](int b, int c) {
    return clamp_len(clamp_len(a.n - static_cast<int64_t>(b) * a.block, a.block) - cst(c), a.chunk);
  };
  auto at = [&](int b, int c) { return (static_cast<int64_t>(b) * a.block + cst(c)) * es; };
  // hop flags: rank k's word for hop h of chunk c, in the row of its only writer (k's
  // predecessor), one column block per hop. ring_hop_rows = the two-writer layout of round 3
  // (row = hop), a negative control only.
  const bool hop_rows = a.ring_hop_rows != 0;
  auto rs_flag = [&](int k, int h, int c) {
    return hop_rows ? f1(a, k, h, c) : f1(a, k, (k + P - 1) % P, h * a.nch + c);
  };
  auto ag_flag = [&](int k, int h, int c) {
    return hop_rows ? f2(a, k, h, c) : f2(a, k, (k + P - 1) % P, h * a.nch + c);
  };
  // every S access of chunk c is WT-typed [cstart, cstart + chunk), every R access E-typed;
  // the highest flag column is (P - 2) * nch + c. The geometry is the same on every rank,
  // so a chunk out of bounds is skipped by all of them (no flag is owed).
  auto inb = [&](int c) {
    return unit_in_bounds(a, cst(c) * ws, clamp_len(a.block - cst(c), a.chunk) * ws, (P - 2) * a.nch + c, err);
  };
  // RS hop 0: the raw own block r
  for (int c = blockIdx.x; c < a.nch; c += G) {
    if (!inb(c)) continue;
    const int64_t len = blen(r, c);
    if (len > 0) ring_hop<E, WT, U>(nullptr, in + at(r, c), a.base[nxt] + a.off_S + cst(c) * ws, nullptr, nullptr, len, 1.f);
    publish_flags([&](int) { return rs_flag(nxt, 0, c); }, 1, epoch, rel);
  }
  read_delay(a, r);  // slow-reader test knob: hold this rank before its first slab read
  // RS hops 1..P-1 (the last one completes block r+1 and starts its all-gather)
  for (int s = 1; s < P; ++s) {
    const int b = (r - s + P) % P;
    for (int c = blockIdx.x; c < a.nch; c += G) {
      if (!inb(c)) continue;
      const int64_t len = blen(b, c);
      const uint64_t tw = ps.now();
      wait_flags([&](int) -> const uint32_t* { return rs_flag(r, s - 1, c); }, 1, epoch, deadline, err,
                 ERR_TIMEOUT_SCATTER, acq);
      ps.add(2, tw);
      ps.count(6);
      const char* part = a.base[r] + a.off_S + (s - 1) * slot + cst(c) * ws;
      if (s < P - 1) {
        if (len > 0)
          ring_hop<E, WT, U>(part, in + at(b, c), a.base[nxt] + a.off_S + s * slot + cst(c) * ws, nullptr, nullptr, len,
                          1.f);
        publish_flags([&](int) { return rs_flag(nxt, s, c); }, 1, epoch, rel);
      } else {
        if (len > 0)
          ring_hop<E, WT, U>(part, in + at(b, c), nullptr, out + at(b, c), a.base[nxt] + a.off_R + cst(c) * es, len,
                          a.scale);
        publish_flags([&](int) { return ag_flag(nxt, 0, c); }, 1, epoch, rel);
      }
    }
  }
  ps.mark(1);
  read_delay(a, r);  // and before its first all-gather read
  // AG hops: receive block (r - t), forward unless it is the last hop
  for (int t = 0; t < P - 1; ++t) {
    const int b = (r - t + P) % P;
    const bool fwd = t < P - 2;
    for (int c = blockIdx.x; c < a.nch; c += G) {
      if (!inb(c)) continue;
      const int64_t len = blen(b, c);
      const uint64_t tw = ps.now();
      wait_flags([&](int) -> const uint32_t* { return ag_flag(r, t, c); }, 1, epoch, deadline, err,
                 ERR_TIMEOUT_REDUCE, acq);
      ps.add(4, tw);
      ps.count(7);
      if (fwd && t == P - 3) forward_delay(a, r);  // test knob: the last forward comes late
      char* d = fwd ? a.base[nxt] + a.off_R + (t + 1) * slot + cst(c) * es : nullptr;
      if (len > 0) copy_slab_fwd<E>(out + at(b, c), d, a.base[r] + a.off_R + t * slot + cst(c) * es, len);
      if (fwd) publish_flags([&](int) { return ag_flag(nxt, t + 1, c); }, 1, epoch, rel);
    }
  }
  ps.mark(3);
  ps.mark(5);
  ps.flush();
  finish_launch_done(a, ctl, epoch, r, kHazS | kHazR);  // the next rank may still read both
}

__global__ __launch_bounds__(kCommThreads) void barrier_kernel(CommArgs a) {
  const int r = a.rank0 + blockIdx.y;
  uint32_t* const ctl = a.ctl[blockIdx.y];
  const uint32_t epoch = launch_epoch(ctl);
  const uint64_t deadline = wall_ticks() + a.timeout;
  publish_flags([&](int k) -> uint32_t* { return fb(a, k, r); }, a.P, epoch);
  wait_flags([&](int s) -> const uint32_t* { return fb(a, r, s); }, a.P, epoch, deadline, &ctl[2],
             ERR_TIMEOUT_BARRIER);
  finish_launch(ctl, epoch);
}

// ---------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------
static int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

static int default_grid(int device) {
  if (const char* g = std::getenv("MXAR_GRID")) return std::max(1, std::atoi(g));
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  return 2 * cus;  // every workgroup must stay resident (they spin): 2 x 256-thread WG per CU
}

int64_t XgmiComm::flag_bytes(int world, int64_t slot_bytes, int threshold_rows, int64_t flag_gran) {
  const int rows = 1 + threshold_rows;
  if (flag_gran <= 0) flag_gran = min_chunk_bytes();
  const int64_t maxch = ceil_div(round_up(std::max<int64_t>(slot_bytes, 64 * 1024), 64 * 1024), flag_gran);
  // [F1: rows x P x maxch][F2: rows x P x maxch][FB: P][PROG: P][F2C: rows x P x maxch][FORCE: P]
  return (3 * rows * world * maxch + 3 * world) * 4;
}

XgmiComm::Layout XgmiComm::layout(int world, int64_t slot_bytes, int threshold_rows, int64_t min_flag_bytes,
                                  int64_t flag_gran) {
  Layout L;
  const int rows = 1 + threshold_rows;
  if (flag_gran <= 0) flag_gran = min_chunk_bytes();
  L.slot_bytes = round_up(std::max<int64_t>(slot_bytes, 64 * 1024), 64 * 1024);
  L.maxch = ceil_div(L.slot_bytes, flag_gran);
  L.off_S = round_up(std::max(flag_bytes(world, slot_bytes, threshold_rows, flag_gran), min_flag_bytes), 64 * 1024);
  // Slots sit back to back (slot_stride = capacity). A pad that takes the P slots a reduce
  // reads off a power-of-two spacing showed no gain for the reduce kernel
  // (benchmarks/bench_reduce.py --pad-kib, profiles/reduce_kernel.md); its study knob was
  // removed in round 6.
  L.slot_stride = L.slot_bytes;
  L.off_R = L.off_S + rows * world * L.slot_stride;
  // low-latency one-shot slots: [2 parities][P sources] x ll_slot (two 8-B LL words per
  // 16-B store: ll_slot = 2 x payload)
  L.ll_max = 512 * 1024;
  if (const char* e = std::getenv("MXAR_LL_MAX")) L.ll_max = std::max<int64_t>(0, std::atoll(e));
  L.ll_max = round_up(L.ll_max, 16);
  L.ll_slot = round_up(std::max<int64_t>(2 * L.ll_max, 16), 64 * 1024);
  L.off_LL = L.off_R + rows * world * L.slot_stride;
  L.slab_bytes = L.off_LL + 2 * world * L.ll_slot;
  // Allocation size: on this ROCm stack hipIpcOpenMemHandle of an allocation whose size has
  // bit 31 set (2-4 GiB, 6-8 GiB, ...) never returns in the importing process, while the
  // sizes around it map and reduce correctly (measured with tools/ipc_size_probe.py, in git history: 1.97,
  // 4.05, 4.33 GiB fine; 2.03-3.9 GiB hang). Such slabs are padded up to the next multiple of
  // 4 GiB - at most 2 GiB of the 288 GB of HBM.
  L.alloc_bytes = ipc_safe_bytes(L.slab_bytes);
  return L;
}

int64_t XgmiComm::ipc_safe_bytes(int64_t bytes) {
  if (bytes & (int64_t{1} << 31)) return round_up(bytes, int64_t{1} << 32);
  return bytes;
}

XgmiComm::XgmiComm(int rank, int world, int device, int64_t slot_bytes, int grid, double timeout_s,
                   int threshold_rows, char* external_slab, int64_t external_bytes, int64_t min_flag_bytes,
                   uint32_t* external_ctl, int64_t flag_gran)
    : rank_(rank), world_(world), device_(device), grid_(grid), rows_(1 + threshold_rows), timeout_s_(timeout_s) {
  if (threshold_rows < 0 || threshold_rows > 64)
    throw std::invalid_argument("XgmiComm: threshold_rows (maxLag + 1) must be in [0, 64]");
  if (world < 1 || world > kMaxRanks) throw std::invalid_argument("XgmiComm: world must be in [1, 16]");
  if (rank < 0 || rank >= world) throw std::invalid_argument("XgmiComm: bad rank");
  const Layout L = layout(world, slot_bytes, threshold_rows, min_flag_bytes, flag_gran);
  slot_bytes_ = L.slot_bytes;
  maxch_ = L.maxch;
  off_S_ = L.off_S;
  slot_stride_ = L.slot_stride;
  off_R_ = L.off_R;
  off_B_ = 2 * rows_ * world_ * maxch_ * 4;
  ll_max_ = L.ll_max;
  ll_slot_ = L.ll_slot;
  off_LL_ = L.off_LL;
  slab_bytes_ = L.slab_bytes;
  alloc_bytes_ = L.alloc_bytes;
  // Automatic dispatch limits (resolve()), measured with P logical ranks in one launch on one
  // MI355X (bench.py latency_vs_size; round 4, with launch-size grids, profiles/round4/README.md
  // section 9): the low-latency one-shot wins up to 512 KiB at 2 and 4 ranks and 256 KiB at 8
  // (it moves 2x bytes as flag-carrying LL words, so it loses to the plain kernels once they
  // are bandwidth bound: 2 ranks x 1 MiB ll 15.8 vs one-shot 12.1 us); the one-shot (one hop,
  // every rank reads all P inputs) up to 8 MiB at 2 ranks and 2 MiB at 4 (2 x 16 MiB: two-shot
  // 37.4 vs one-shot 42.1 us; 4 x 4 MiB: 32.3 vs 39.4 us); at 8 ranks the two-shot takes over
  // from the low-latency kernel directly. Across GPUs the one-shot reads every peer's whole
  // buffer over its link, so the two-shot's crossover comes no later there.
  // MXAR_LL_AUTO_MAX / MXAR_ONESHOT_MAX override (bytes).
  const int64_t mib = int64_t{1} << 20;
  ll_auto_max_ = world_ <= 4 ? mib / 2 : mib / 4;
  if (const char* e = std::getenv("MXAR_LL_AUTO_MAX")) ll_auto_max_ = std::max<int64_t>(0, std::atoll(e));
  oneshot_max_ = std::min<int64_t>(slot_bytes_, world_ <= 2 ? 8 * mib : world_ <= 4 ? 2 * mib : mib / 4);
  if (const char* e = std::getenv("MXAR_ONESHOT_MAX")) oneshot_max_ = std::min<int64_t>(slot_bytes_, std::atoll(e));
  default_grid_ = default_grid(device);
  if (grid_ <= 0) grid_ = default_grid_;
  if (const char* e = std::getenv("MXAR_SIZE_GRID")) size_grid_ = std::atoi(e) != 0;
  if (const char* f = study_env("MXAR_FENCE")) fence_ = std::atoi(f) & 3;
  // Slab reads are `nt` loads: the acquire after each wait (bit 1) is what orders them after
  // the peers' flags. Without it a stale line could be read, so clearing it is a study-only
  // setting that must be asked for explicitly.
  if (const char* u = study_env("MXAR_TWOSHOT_UNITS")) units_per_wg_ = std::max(1, std::atoi(u));
  if (const char* u = study_env("MXAR_TWOSHOT_SUB")) sub_max_ = std::max(1, std::atoi(u));
  if (const char* d = study_env("MXAR_RING_DEPTH")) ring_depth_ = std::max(1, std::atoi(d));
  if (const char* g = std::getenv("MXAR_RING_GRID")) ring_grid_ = std::max(1, std::atoi(g));
  if (const char* f = study_env("MXAR_RING_FLAGS")) {
    // the round-3 layout whose flag words had two writers (ring hop rows vs other kernels'
    // writer rows): kept only as the negative control of tests/test_comm_gpu.py
    ring_hop_rows_ = std::string(f) == "hop";
  }
  if (const char* g = study_env("MXAR_SLOT_GUARD")) noguard_ = std::atoi(g) == 0;
  // A/B of the threshold kernel's lag-gate shortcut
  if (const char* g = study_env("MXAR_GATE_SHORTCUT")) no_gate_shortcut_ = std::atoi(g) == 0;
  if (const char* g = study_env("MXAR_TH_ONESHOT_MAX")) th_oneshot_max_ = std::max<int64_t>(0, std::atoll(g));
  if (const char* g = study_env("MXAR_TWOSHOT_GEOM")) {
    const std::string v = g;
    geom_ = v == "coarse" ? 0 : v == "fine" ? 1 : v == "flat" ? 2 : -1;
  }
  if (const char* f = study_env("MXAR_TWOSHOT_FLAT_MIN")) flat_min_ = std::max<int64_t>(0, std::atoll(f));

  hip_check(hipSetDevice(device_), "hipSetDevice");
  const char* mem = study_env("MXAR_SLAB_MEM");
  const std::string kind = mem ? mem : "fine";
  // study knobs that trade away correctness guarantees: say so once per communicator
  if (fence_ != 3 || kind != "fine")
    std::fprintf(stderr,
                 "[mxar] WARNING rank %d: study settings active (MXAR_FENCE=%d, MXAR_SLAB_MEM=%s); "
                 "results may be wrong - use the defaults in production\n",
                 rank_, fence_, kind.c_str());
  if (external_slab != nullptr) {
    // An arena owned by the caller (xgmi_plane.cc): allocated fine-grained and zeroed ONCE,
    // exported before any peer knew it, and laid out again on every re-initialisation. Its
    // flags are never zeroed here - a peer may already be writing this epoch's flags; stale
    // flags of an older layout are older epochs, which no wait accepts.
    if (external_bytes < slab_bytes_) throw std::invalid_argument("XgmiComm: external slab too small for the layout");
    slab_ = external_slab;
    own_slab_ = false;
    alloc_bytes_ = external_bytes;
  } else if (kind == "coarse") {
    hip_check(hipMalloc(reinterpret_cast<void**>(&slab_), alloc_bytes_), "hipMalloc(slab)");
  } else {
    const unsigned flags = kind == "fine" ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
    hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&slab_), alloc_bytes_, flags), "hipExtMallocWithFlags(slab)");
  }
  if (own_slab_) {
    // Flags start at 0 = "epoch 0 done"; the first launch uses epoch 1.
    hip_check(hipMemset(slab_, 0, off_S_), "hipMemset(flags)");
    hip_check(hipMemset(slab_ + off_LL_, 0, 2 * world_ * ll_slot_), "hipMemset(ll)");  // epoch 0 never occurs
  }
  if (external_ctl != nullptr && !own_slab_) {
    ctl_ = external_ctl;  // reset by the caller, stream-ordered
    own_ctl_ = false;
  } else {
    hip_check(hipMalloc(reinterpret_cast<void**>(&ctl_), 256), "hipMalloc(ctl)");
    hip_check(hipMemset(ctl_, 0, 256), "hipMemset(ctl)");
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  }
  peers_[rank_] = slab_;
}

XgmiComm::~XgmiComm() {
  (void)hipSetDevice(device_);
  if (switch_ev_) (void)hipEventDestroy(switch_ev_);
  for (int k = 0; k < world_; ++k)
    if (ipc_opened_[k] && peers_[k]) (void)hipIpcCloseMemHandle(peers_[k]);
  for (int k = 0; k < static_cast<int>(probe_peers_.size()); ++k)
    if (k != rank_ && probe_peers_[k]) (void)hipIpcCloseMemHandle(probe_peers_[k]);
  if (probe_coarse_) (void)hipFree(probe_coarse_);
  if (slab_ && own_slab_) (void)hipFree(slab_);
  if (ctl_ && own_ctl_) (void)hipFree(ctl_);
}

std::string XgmiComm::ipc_handle() const {
  hipIpcMemHandle_t h;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipIpcGetMemHandle(&h, slab_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void XgmiComm::connect(const std::vector<std::string>& handles) {
  if (static_cast<int>(handles.size()) != world_) throw std::invalid_argument("connect: need one handle per rank");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (int k = 0; k < world_; ++k) {
    if (k == rank_) continue;
    if (handles[k].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("connect: bad handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[k].data(), sizeof(h));
    void* p = nullptr;
    static const bool dbg = std::getenv("MXAR_DEBUG_IPC") != nullptr;
    if (dbg) std::fprintf(stderr, "[mxar ipc] rank %d opening rank %d\n", rank_, k);
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    if (dbg) std::fprintf(stderr, "[mxar ipc] rank %d opened rank %d at %p\n", rank_, k, p);
    peers_[k] = static_cast<char*>(p);
    ipc_opened_[k] = true;
  }
  connected_ = true;
}

void XgmiComm::connect_local(const std::vector<XgmiComm*>& comms) {
  if (static_cast<int>(comms.size()) != world_) throw std::invalid_argument("connect_local: need one comm per rank");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (int k = 0; k < world_; ++k) {
    if (comms[k]->slab_bytes_ != slab_bytes_) throw std::invalid_argument("connect_local: slab geometry differs");
    peers_[k] = comms[k]->slab_;
    if (comms[k]->device_ != device_) {
      int can = 0;
      (void)hipDeviceCanAccessPeer(&can, device_, comms[k]->device_);
      if (!can) throw std::runtime_error("connect_local: no peer access between devices");
      hipError_t e = hipDeviceEnablePeerAccess(comms[k]->device_, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) hip_check(e, "hipDeviceEnablePeerAccess");
      (void)hipGetLastError();
    }
  }
  connected_ = true;
}

void XgmiComm::connect_ptrs(const std::vector<char*>& bases) {
  if (static_cast<int>(bases.size()) != world_) throw std::invalid_argument("connect_ptrs: need one base per rank");
  for (int k = 0; k < world_; ++k) {
    if (k == rank_) continue;
    if (bases[k] == nullptr) throw std::invalid_argument("connect_ptrs: null peer slab");
    peers_[k] = bases[k];
  }
  connected_ = true;
}

void XgmiComm::set_grid(int g) { grid_ = g > 0 ? g : default_grid_; }

int XgmiComm::launch_grid(int64_t bytes, bool oneshot, int64_t full_at) const {
  // Workgroups for a two-shot / one-shot launch moving `bytes` of input (all ranks of the
  // launch). Every unit of work pays flag hand-offs and fenced stores without adding bytes
  // (PMC: 4x the workgroups at 8 x 1 MiB cost 8x the wait cycles, with no extra L2
  // write-back / invalidate operations), so below ~512 MiB per launch the full grid loses
  // to ~one workgroup per 64 KiB (8 / 4 / 2 logical ranks x 64 KiB - 256 MiB, same
  // box: two-shot 1 MiB x 8 ranks 36.6 -> 21.9 us, 16 MiB x 4 ranks 95.4 -> 67.8 us, 64 MiB x 2
  // ranks 132 -> 101 us, 256 MiB unchanged; profiles/round4/README.md section 9):
  //   two-shot: one workgroup per 64 KiB, 64..256, the full grid from `full_at` (512 MiB;
  //             the threshold kernel: 256 MiB - 4 x 64 MiB 288 us full vs 307 us sized);
  //   one-shot: every rank reads all P inputs, so one per 64 KiB of P x bytes, 64..full grid.
  // At the default grid only: an explicit grid is used as given.
  if (!size_grid_ || grid_ != default_grid_) return grid_;
  return size_grid_rule(bytes, grid_, world_, oneshot, full_at);
}

int XgmiComm::shared_launch_cap(int ranks_here) const {
  // Several logical ranks in one launch (one GPU): at most a quarter of the default grid - half
  // the CUs - per rank at the default grid. 2 ranks x 256 MiB bf16 two-shot 426-436 -> 389-395
  // us, threshold 432-440 -> 411-414; 4 x 128 MiB 128 per rank beats 64; 8 x 256 MiB equal
  // (profiles/round5/local_launch_grid.jsonl). One rank per GPU keeps launch_grid's rule.
  const int cap = shared_launch_rule(ranks_here, default_grid_);
  if (cap <= 0 || !size_grid_ || grid_ != default_grid_) return std::numeric_limits<int>::max();
  return cap;
}

static bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

void XgmiComm::order_after_last(hipStream_t s) {
  if (launched_ && s != last_stream_) {
    // Graph capture: a captured stream cannot wait on work outside its graph; the caller
    // orders the graph launch (documented in xgmi_comm.h).
    if (!capturing(s) && !capturing(last_stream_)) {
      if (!switch_ev_)
        hip_check(hipEventCreateWithFlags(&switch_ev_, hipEventDisableTiming), "hipEventCreateWithFlags");
      hip_check(hipEventRecord(switch_ev_, last_stream_), "hipEventRecord(stream switch)");
      hip_check(hipStreamWaitEvent(s, switch_ev_, 0), "hipStreamWaitEvent(stream switch)");
      ++stats_.stream_switches;
    }
  }
  launched_ = true;
  last_stream_ = s;
}

void XgmiComm::order_group(const std::vector<XgmiComm*>& group, hipStream_t s) {
  for (XgmiComm* c : group) c->order_after_last(s);
}

std::vector<uint32_t> XgmiComm::ctl_words() const {
  std::vector<uint32_t> w(16, 0);
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipMemcpy(w.data(), ctl_, w.size() * 4, hipMemcpyDeviceToHost), "hipMemcpy(ctl)");
  return w;
}

uint32_t XgmiComm::error() const {
  uint32_t e = 0;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipMemcpy(&e, ctl_ + 2, 4, hipMemcpyDeviceToHost), "hipMemcpy(err)");
  return e;
}

void XgmiComm::clear_error() {
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipMemset(ctl_ + 2, 0, 4), "hipMemset(err)");
}

void XgmiComm::reset_local() {
  // Back to the state right after construction: every flag, progress word and LL slot 0
  // (= "epoch 0 done"), epoch / ticket / error / threshold-round counters 0. Only valid when
  // no launch of this communicator is in flight on any rank (XgmiCommunicator.reset
  // brackets it with device synchronisation and host barriers).
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  hip_check(hipMemset(slab_, 0, off_S_), "hipMemset(flags)");
  hip_check(hipMemset(slab_ + off_LL_, 0, 2 * world_ * ll_slot_), "hipMemset(ll)");
  hip_check(hipMemset(ctl_, 0, 256), "hipMemset(ctl)");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
}

void XgmiComm::arm_solo_rehearsal() {
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  hip_check(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(slab_), 0x40000000u, static_cast<size_t>(off_S_ / 4)),
            "hipMemsetD32(flags)");
  // the synthetic peers' contributions in the S / R slots: zeros (the sums stay the input)
  hip_check(hipMemset(slab_ + off_S_, 0, static_cast<size_t>(slab_bytes_ - off_S_)), "hipMemset(slots)");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
}

template <class E>
static void launch_typed(const CommArgs& a, dim3 grid, hipStream_t s, Algo kind) {
  const dim3 b(kCommThreads);
  // two packs in flight per lane and hop: 4 and 8 measured no faster (profiles/round5/ring_packs_in_flight_ab.jsonl)
  if (kind == Algo::Ring) {  // exact wire: fp32 partials
    hipLaunchKernelGGL((ring_kernel<E, F32, 2>), grid, b, 0, s, a);
    return;
  }
  if (kind == Algo::RingNative) {  // element-type wire
    hipLaunchKernelGGL((ring_kernel<E, E, 2>), grid, b, 0, s, a);
    return;
  }
  const bool oneshot = kind == Algo::OneShot;
#define MXAR_LAUNCH(PT)                                                                         \
  do {                                                                                          \
    if (oneshot)                                                                                \
      hipLaunchKernelGGL((oneshot_kernel<E, PT>), grid, b, 0, s, a);                            \
    else                                                                                        \
      hipLaunchKernelGGL((twoshot_kernel<E, PT>), grid, b, 0, s, a);                            \
  } while (0)
  switch (a.P) {
    case 1: MXAR_LAUNCH(1); break;
    case 2: MXAR_LAUNCH(2); break;
    case 4: MXAR_LAUNCH(4); break;
    case 8: MXAR_LAUNCH(8); break;
    default: MXAR_LAUNCH(0); break;
  }
#undef MXAR_LAUNCH
}

// Common launch geometry + args for the ranks `group` (all on one device, consecutive
// rank ids starting at group[0]->rank()).
void XgmiComm::launch_segment(const std::vector<XgmiComm*>& group, const char* const* ins, char* const* outs,
                              int64_t n, DType dt, hipStream_t stream, Algo kind, float scale,
                              const std::vector<AdamShard>* adam_state, const AdamW* adam) {
  const bool oneshot = kind == Algo::OneShot;
  const XgmiComm& c0 = *group[0];
  const int W = c0.world_;
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  const int64_t elems = 16 / es;
  CommArgs a;
  std::memset(&a, 0, sizeof(a));
  for (size_t y = 0; y < group.size(); ++y) {
    a.in[y] = ins[y];
    a.out[y] = outs[y];
    a.ctl[y] = group[y]->ctl_;
  }
  a.n = n;
  a.P = W;
  a.rows = c0.rows_;
  a.rank0 = c0.rank_;
  a.maxch = c0.maxch_;
  a.off_S = c0.off_S_;
  a.off_R = c0.off_R_;
  a.slot_bytes = c0.slot_stride_;
  a.slot_cap = c0.slot_bytes_;
  a.timeout = static_cast<uint64_t>(c0.timeout_s_ * 1e8);
  for (int k = 0; k < W; ++k) a.base[k] = c0.peers_[k];
  const int64_t min_chunk = min_chunk_bytes() / es;
  const int ranks_here = static_cast<int>(group.size());
  // all workgroups of the launch stay resident; plain two-shot / one-shot launches size the
  // grid by their bytes (launch_grid); the fused AdamW step (8 streams per element) runs best
  // at 256 workgroups per device (134 M params: 0.745 vs 0.762 ms at 512, same box, twice;
  // profiles/round4/README.md section 5), at the default grid
  const bool sized = adam_state == nullptr && (kind == Algo::TwoShot || oneshot);
  const int gdev = sized ? c0.launch_grid(n * es * ranks_here, oneshot)
                   : (adam_state != nullptr && c0.size_grid_ && c0.grid_ == c0.default_grid_) ? std::min(c0.grid_, 256)
                                                                                            : c0.grid_;
  const int gmax = std::min(std::max(1, gdev / ranks_here), kind == Algo::TwoShot ? c0.shared_launch_cap(ranks_here)
                                                                                  : std::numeric_limits<int>::max());
  int gx;
  a.sub = 1;
  a.off_LL = c0.off_LL_;
  a.ll_slot = c0.ll_slot_;
  if (kind == Algo::LL) {
    const int64_t units = ceil_div(n * es, 8);
    a.block = a.chunk = a.subchunk = n;
    a.nch = 1;
    gx = static_cast<int>(std::min<int64_t>(gmax, std::max<int64_t>(1, ceil_div(units, kCommThreads))));
  } else if (oneshot) {
    a.block = n;
    a.chunk = std::max(min_chunk, round_up(ceil_div(n, gmax), elems));
    a.nch = static_cast<int>(std::max<int64_t>(1, ceil_div(n, a.chunk)));
    a.subchunk = a.chunk;
    gx = static_cast<int>(std::min<int64_t>(gmax, a.nch));
  } else if (kind == Algo::Ring || kind == Algo::RingNative) {
    // ring_depth chunks per workgroup, walked step-major (ring_kernel). Hop flags sit in the
    // row of the WRITER (the previous rank), one column block per hop: every flag word has a
    // single writer across all kernels, so epochs never go backwards (a ring's late forward
    // of launch e-1 landing on a word another rank's all-gather set to e lost that flag -
    // profiles/round3/README.md); (W - 1) * nch columns must fit the flag row.
    // Every hop of every workgroup pays a system-scope release and acquire, and those
    // serialise in the XCD's L2 when hundreds of workgroups fence at once: at 8 logical ranks
    // x 256 MiB the ring ran fastest with 256 workgroups in all (one per CU) and one chunk
    // per workgroup - more chunks per workgroup only multiply the fences (ring_grid sweep,
    // profiles/round4/README.md). MXAR_RING_GRID / MXAR_RING_DEPTH override.
    const int depth = std::max(1, c0.ring_depth_);
    // and at the default grid, one workgroup per 32 KiB of the per-rank bytes, 64..ring_grid:
    // every hop of every workgroup is a dependent hand-off (8 / 2 logical ranks, ring_native
    // p50 at ring grid 64 / 128 / 256 / 512: 8 x 1 MiB 51 / 62 / 99 / 162 us, 8 x 4 MiB 108 / 96
    // / 136 / 250 us, 2 x 16 MiB 72 / 48 / 39 / 46 us; profiles/round4/ring_grid_mid.jsonl)
    int ring_dev = c0.ring_grid_;
    if (c0.size_grid_ && c0.grid_ == c0.default_grid_)
      ring_dev = static_cast<int>(std::min<int64_t>(c0.ring_grid_, std::max<int64_t>(64, n * es / (int64_t{32} << 10))));
    const int gring = std::max(1, std::min(gmax, ring_dev / ranks_here));
    a.block = round_up(ceil_div(n, W), elems);
    a.chunk = std::max(min_chunk, round_up(ceil_div(a.block, int64_t{gring} * depth), elems));
    a.nch = static_cast<int>(std::max<int64_t>(1, ceil_div(a.block, a.chunk)));
    const int64_t cols = std::max<int64_t>(1, c0.maxch_ / std::max(1, W - 1));
    if (a.nch > cols) {
      a.chunk = round_up(ceil_div(a.block, cols), elems);
      a.nch = static_cast<int>(std::max<int64_t>(1, ceil_div(a.block, a.chunk)));
    }
    a.subchunk = a.chunk;
    gx = static_cast<int>(std::min<int64_t>(gring, a.nch));
  } else {
    // ~one scatter unit and one gather unit per workgroup: every unit pays one fence, so
    // units are as large as the parallelism allows. The reduce phase splits each chunk
    // W-1 ways to keep the same unit count.
    a.block = round_up(ceil_div(n, W), elems);
    // Geometry by block size (measured, profiles/twoshot_granularity.md): small blocks want
    // ~one scatter unit per workgroup (fewest flag hand-offs); large blocks (>= 32 MiB) want
    // one chunk per workgroup (W-1 scatter units each) reduced in at most 2 pieces - chunks
    // arrive in a finer stream, so reduces start earlier and the tail is shorter (4 / 8 ranks
    // x 256 MiB: -6 % / -4 %; at 8-16 MiB blocks it loses 14-20 %). MXAR_TWOSHOT_UNITS /
    // MXAR_TWOSHOT_SUB override.
    // Geometry by block size (same-box A/B over 2 / 4 / 8 logical ranks x 1-256 MiB,
    // profiles/round3/twoshot_geometry_ab.jsonl; MXAR_TWOSHOT_GEOM=coarse|fine|flat forces one):
    //   coarse (blocks < 2 MiB): ~one scatter unit per workgroup, each chunk reduced in up to
    //          P-1 pieces - fewest flag hand-offs, best while the round is latency bound;
    //   flat   (blocks >= 2 MiB): one chunk per workgroup (one reduce unit each, no split),
    //          the scatter in groups of `sgroup` chunks per destination (one copy and one
    //          release per group, a flag per chunk) - small chunks start the reduces early,
    //          grouped copies keep the scatter at copy speed: -22 % at 8 x 64 MiB, -7 % at
    //          8 x 256 MiB vs the best of the others, equal at 2 ranks;
    //   fine   (the round-2 choice for blocks >= 32 MiB): one chunk per workgroup for each of
    //          the P-1 destinations, reduced in 2 pieces - no longer the default.
    // an explicit units-per-workgroup (MXAR_TWOSHOT_UNITS, tune()'s "~1" labels) selects the
    // coarse / fine family it parameterises
    const int geom = c0.geom_ >= 0 ? c0.geom_ : c0.units_per_wg_ > 0 ? 0 : (a.block * es >= c0.flat_min_ ? 2 : 0);
    if (geom == 2 && W > 1) {
      a.chunk = std::max(min_chunk, round_up(ceil_div(a.block, gmax), elems));
      a.nch = static_cast<int>(std::max<int64_t>(1, ceil_div(a.block, a.chunk)));
      a.sub = 1;
      a.subchunk = a.chunk;
      gx = static_cast<int>(std::min<int64_t>(gmax, std::max<int64_t>(1, static_cast<int64_t>(W - 1) * a.nch)));
      const int per = std::max(1, gx / (W - 1));  // scatter groups per destination block
      a.sgroup = static_cast<int>(std::min<int64_t>(64, std::max<int64_t>(1, ceil_div(a.nch, per))));
    } else {
      const bool fine = geom == 1;
      const int upw = c0.units_per_wg_ > 0 ? c0.units_per_wg_ : fine ? std::max(1, W - 1) : 1;
      const int sub_max = c0.sub_max_ > 0 ? c0.sub_max_ : fine ? 2 : 64;
      const int64_t target = W > 1 ? std::max<int64_t>(1, int64_t{gmax} * upw / (W - 1)) : int64_t{gmax} * upw;
      a.chunk = std::max(min_chunk, round_up(ceil_div(a.block, target), elems));
      a.nch = static_cast<int>(std::max<int64_t>(1, ceil_div(a.block, a.chunk)));
      int64_t sub = std::max<int64_t>(1, std::min<int64_t>({static_cast<int64_t>(W - 1), a.chunk / min_chunk, 64,
                                                            c0.maxch_ / a.nch, int64_t{sub_max}}));
      a.subchunk = round_up(ceil_div(a.chunk, sub), elems);
      a.sub = static_cast<int>(ceil_div(a.chunk, a.subchunk));
      const int64_t units =
          std::max<int64_t>((W - 1) * static_cast<int64_t>(a.nch), static_cast<int64_t>(a.nch) * a.sub);
      gx = static_cast<int>(std::min<int64_t>(gmax, std::max<int64_t>(1, units)));
    }
  }
  a.fence = c0.fence_;
  a.scale = scale;
  a.rdelay_rank = c0.rdelay_rank_;
  a.rdelay = c0.rdelay_us_ > 0 ? static_cast<uint64_t>(c0.rdelay_us_ * 100.0) : 0;  // 100 MHz ticks
  a.fdelay_rank = c0.fdelay_rank_;
  a.fdelay = c0.fdelay_us_ > 0 ? static_cast<uint64_t>(c0.fdelay_us_ * 100.0) : 0;
  a.noguard = c0.noguard_ ? 1 : 0;
  a.ring_hop_rows = c0.ring_hop_rows_ ? 1 : 0;
  a.stamps = c0.stamps_;
  if (a.stamps != nullptr && gx * ranks_here > c0.stamp_slots_) a.stamps = nullptr;  // buffer too small: off
  const bool ring = kind == Algo::Ring || kind == Algo::RingNative;
  const int64_t block_bytes = a.block * (kind == Algo::Ring ? 4 : es);  // ring: fp32 partial slots
  const int64_t flag_cols = ring ? static_cast<int64_t>(std::max(1, W - 1)) * a.nch
                                              : static_cast<int64_t>(a.nch) * a.sub;
  if (kind != Algo::LL && (flag_cols > c0.maxch_ || block_bytes > c0.slot_bytes_ + 16))
    throw std::logic_error("XgmiComm: segment geometry exceeds slab");
  const dim3 grid(gx, ranks_here);
  if (adam != nullptr) {
    for (size_t y = 0; y < group.size(); ++y) {
      a.opt_p[y] = (*adam_state)[y].param;
      a.opt_m[y] = (*adam_state)[y].exp_avg;
      a.opt_v[y] = (*adam_state)[y].exp_avg_sq;
    }
    a.lr = adam->lr;
    a.beta1 = adam->beta1;
    a.beta2 = adam->beta2;
    a.eps = adam->eps;
    a.wd = adam->weight_decay;
    a.c1 = 1.f - std::pow(adam->beta1, static_cast<float>(adam->step));
    a.c2_sqrt = std::sqrt(1.f - std::pow(adam->beta2, static_cast<float>(adam->step)));
    launch_adamw(a, grid, stream, dt);
    hip_check(hipGetLastError(), "adamw launch");
    for (XgmiComm* c : group) {
      ++c->stats_.launches;
      ++c->stats_.adamw;
    }
    return;
  }
  if (kind == Algo::LL) {
    if (2 * ceil_div(n * es, 8) * 8 > c0.ll_slot_) throw std::logic_error("XgmiComm: LL segment exceeds its slot");
    launch_ll(a, grid, stream, dt);
  } else {
    dispatch_dtype(static_cast<int>(dt), [&](auto tag) { launch_typed<decltype(tag)>(a, grid, stream, kind); });
  }
  hip_check(hipGetLastError(), "allreduce launch");
  for (XgmiComm* c : group) {
    ++c->stats_.launches;
    ++(kind == Algo::LL ? c->stats_.ll
                        : oneshot ? c->stats_.oneshot : ring ? c->stats_.ring : c->stats_.twoshot);
  }
}

void XgmiComm::run(const std::vector<XgmiComm*>& group, const std::vector<const void*>& ins,
                   const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream, Algo algo, float scale) {
  if (group.empty() || ins.size() != group.size() || outs.size() != group.size())
    throw std::invalid_argument("XgmiComm: one input and one output per rank");
  const XgmiComm& c0 = *group[0];
  for (size_t y = 0; y < group.size(); ++y) {
    const XgmiComm& c = *group[y];
    if (!c.connected_) throw std::runtime_error("XgmiComm: connect() first");
    if (c.device_ != c0.device_ || c.rank_ != c0.rank_ + static_cast<int>(y) || c.world_ != c0.world_)
      throw std::invalid_argument("XgmiComm: a grouped launch needs consecutive ranks on one device");
    if ((reinterpret_cast<uintptr_t>(ins[y]) | reinterpret_cast<uintptr_t>(outs[y])) & 15)
      throw std::invalid_argument("XgmiComm: buffers must be 16-byte aligned");
  }
  if (n <= 0) return;
  hip_check(hipSetDevice(c0.device_), "hipSetDevice");
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  for (XgmiComm* c : group) {
    ++c->stats_.calls;
    c->stats_.bytes += n * es;
  }
  order_group(group, stream);
  if (c0.world_ == 1 && scale == 1.f) {  // a 1-rank sum is the identity: copy out-of-place, nothing in place
    for (size_t y = 0; y < group.size(); ++y)
      if (ins[y] != outs[y])
        launch_copy(ins[y], outs[y], n * es, stream);
    return;
  }
  const Algo kind = c0.resolve(n, dt, algo, static_cast<int>(group.size()));
  const bool ll = kind == Algo::LL;
  const bool oneshot = kind == Algo::OneShot;
  TraceScope span("xgmi", [&] {
    return std::make_pair(std::string(ll        ? "ll "
                                      : oneshot ? "oneshot "
                                      : kind == Algo::Ring ? "ring "
                                      : kind == Algo::RingNative ? "ring_native "
                                                           : "twoshot ") +
                              std::to_string(n * es) + "B",
                          "{\"rank\":" + std::to_string(c0.rank_) + ",\"ranks_in_launch\":" +
                              std::to_string(group.size()) + "}");
  });
  // ring: S slots carry fp32 partials, so a block holds slot_bytes / 4 elements
  const int64_t seg = ll ? c0.ll_max_ / es
                      : oneshot ? c0.slot_bytes_ / es
                      : kind == Algo::Ring ? c0.world_ * (c0.slot_bytes_ / 4) : c0.world_ * (c0.slot_bytes_ / es);
  // (RingNative: element-type partials, a block fills a slot like the two-shot's)
  std::vector<const char*> ip(group.size());
  std::vector<char*> op(group.size());
  for (int64_t off = 0; off < n; off += seg) {
    const int64_t len = std::min(seg, n - off);
    for (size_t y = 0; y < group.size(); ++y) {
      ip[y] = static_cast<const char*>(ins[y]) + off * es;
      op[y] = static_cast<char*>(outs[y]) + off * es;
    }
    launch_segment(group, ip.data(), op.data(), len, dt, stream, kind, scale);
  }
}

Algo XgmiComm::resolve(int64_t n, DType dt, Algo algo, int ranks_in_launch) const {
  (void)ranks_in_launch;
  const int64_t bytes = n * static_cast<int64_t>(dtype_size(dt));
  if (algo == Algo::LL) return ll_max_ >= 16 ? Algo::LL : Algo::TwoShot;
  if (algo == Algo::OneShot) return bytes <= slot_bytes_ ? Algo::OneShot : Algo::TwoShot;
  if (algo == Algo::Ring || algo == Algo::RingNative) return algo;
  if (algo == Algo::TwoShot) return Algo::TwoShot;
  // Auto: low-latency one-shot, then one-shot, then two-shot, with size limits per rank count
  // set in the constructor from the bench's latency table (profiles/round3/README.md)
  if (ll_max_ >= 16 && bytes <= ll_auto_max_) return Algo::LL;
  return bytes <= oneshot_max_ ? Algo::OneShot : Algo::TwoShot;
}

int64_t XgmiComm::block_elems(int64_t n, DType dt) const {
  const int64_t elems = 16 / static_cast<int64_t>(dtype_size(dt));
  return round_up(ceil_div(n, world_), elems);
}

void XgmiComm::step_adamw_local(const std::vector<XgmiComm*>& group, const std::vector<const void*>& grads,
                                const std::vector<void*>& params, int64_t n, DType dt, hipStream_t stream,
                                const std::vector<AdamShard>& st, const AdamW& h, float scale) {
  if (group.empty() || grads.size() != group.size() || params.size() != group.size() || st.size() != group.size())
    throw std::invalid_argument("step_adamw: one grads / params / shard state per rank");
  const XgmiComm& c0 = *group[0];
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  for (size_t y = 0; y < group.size(); ++y) {
    const XgmiComm& c = *group[y];
    if (!c.connected_) throw std::runtime_error("XgmiComm: connect() first");
    if (c.device_ != c0.device_ || c.rank_ != c0.rank_ + static_cast<int>(y) || c.world_ != c0.world_)
      throw std::invalid_argument("XgmiComm: a grouped launch needs consecutive ranks on one device");
    const uintptr_t g = reinterpret_cast<uintptr_t>(grads[y]), p = reinterpret_cast<uintptr_t>(params[y]);
    if ((g | p | reinterpret_cast<uintptr_t>(st[y].param) | reinterpret_cast<uintptr_t>(st[y].exp_avg) |
         reinterpret_cast<uintptr_t>(st[y].exp_avg_sq)) & 15)
      throw std::invalid_argument("step_adamw: buffers must be 16-byte aligned");
    if (g < p + static_cast<uintptr_t>(n * es) && p < g + static_cast<uintptr_t>(n * es))
      throw std::invalid_argument("step_adamw: grads and params must not overlap");
  }
  if (n <= 0) return;
  if (n * es > c0.world_ * c0.slot_bytes_)
    throw std::invalid_argument("step_adamw: tensor exceeds one launch (n * dtype <= world * slot_bytes)");
  if (h.step < 1) throw std::invalid_argument("step_adamw: step counts from 1");
  hip_check(hipSetDevice(c0.device_), "hipSetDevice");
  for (XgmiComm* c : group) {
    ++c->stats_.calls;
    c->stats_.bytes += n * es;
  }
  order_group(group, stream);
  TraceScope span("xgmi", [&] {
    return std::make_pair("adamw " + std::to_string(n * es) + "B", "{\"rank\":" + std::to_string(c0.rank_) + "}");
  });
  std::vector<const char*> ip(group.size());
  std::vector<char*> op(group.size());
  for (size_t y = 0; y < group.size(); ++y) {
    ip[y] = static_cast<const char*>(grads[y]);
    op[y] = static_cast<char*>(params[y]);
  }
  launch_segment(group, ip.data(), op.data(), n, dt, stream, Algo::TwoShot, scale, &st, &h);
}

void XgmiComm::step_adamw(const void* grads, void* params, int64_t n, DType dt, hipStream_t stream,
                          const AdamShard& st, const AdamW& h, float scale) {
  step_adamw_local({this}, {grads}, {params}, n, dt, stream, {st}, h, scale);
}

void XgmiComm::allreduce(const void* in, void* out, int64_t n, DType dt, hipStream_t stream, Algo algo, float scale) {
  run({this}, {in}, {out}, n, dt, stream, algo, scale);
}

void XgmiComm::allreduce_local(const std::vector<XgmiComm*>& comms, const std::vector<const void*>& ins,
                               const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream, Algo algo,
                               float scale) {
  run(comms, ins, outs, n, dt, stream, algo, scale);
}

void XgmiComm::geometry_threshold(int64_t n, DType dt, int ranks_here, int64_t* block, int64_t* chunk, int* nch,
                                  int* gx) const {
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  const int64_t elems = 16 / es;
  const int64_t min_chunk = min_chunk_bytes() / es;
  // launch-size grid as for the two-shot (launch_grid; at the default grid only). The full
  // grid from 256 MiB per launch for one rank per device (round 4: 4 x 64 MiB 288 us full vs
  // 307 us sized); several logical ranks in one launch take it from 512 MiB like the two-shot
  // since round 6 (one reduce chunk per workgroup, 2 x 8 reduce batches): 4 x 64 MiB 271 ->
  // 248 us, 4 x 256 MiB 1066 -> 1040 us sized (profiles/round6 section 11)
  const int64_t full_at = ranks_here > 1 ? int64_t{512} << 20 : int64_t{256} << 20;
  const int gmax =
      std::min(std::max(1, launch_grid(n * es * std::max(1, ranks_here), false, full_at) / std::max(1, ranks_here)),
               shared_launch_cap(ranks_here));
  *block = round_up(ceil_div(n, world_), elems);
  // one reduce unit (a chunk: one threshold decision) per workgroup; phase 1/3 get P-1 each,
  // spread over up to (P - 1) x nch workgroups when the chunks are few (small tensors)
  *chunk = std::max(min_chunk, round_up(ceil_div(*block, gmax), elems));
  *nch = static_cast<int>(std::max<int64_t>(1, ceil_div(*block, *chunk)));
  *gx = static_cast<int>(std::min<int64_t>(gmax, std::max<int64_t>(1, static_cast<int64_t>(std::max(world_ - 1, 1)) * *nch)));
}

int XgmiComm::round_grid(int nch) const {
  // one reduce unit per workgroup where possible, and the scatter / gather units (P - 1 per
  // chunk) spread over as many workgroups as there are, up to the grid: a round of few
  // chunks otherwise serialises its hand-offs in one workgroup
  const int64_t units = static_cast<int64_t>(std::max(world_ - 1, 1)) * std::max(nch, 1);
  return static_cast<int>(std::min<int64_t>(grid_, std::max<int64_t>({1, nch, units})));
}

int XgmiComm::threshold_chunks(int64_t n, DType dt, int ranks_in_launch) const {
  int64_t b, c;
  int nch, gx;
  geometry_threshold(n, dt, ranks_in_launch, &b, &c, &nch, &gx);
  return nch;
}

bool XgmiComm::threshold_args(const std::vector<XgmiComm*>& group, const std::vector<const void*>& ins,
                              const std::vector<void*>& outs, int64_t n, DType dt, float thr, float thc,
                              int32_t* counts, float scale, bool rescale, const RoundSpec* spec, void* args,
                              int* gx_out) {
  if (group.empty() || ins.size() != group.size() || outs.size() != group.size())
    throw std::invalid_argument("XgmiComm: one input and one output per rank");
  const XgmiComm& c0 = *group[0];
  for (size_t y = 0; y < group.size(); ++y) {
    const XgmiComm& c = *group[y];
    if (!c.connected_) throw std::runtime_error("XgmiComm: connect() first");
    if (c.device_ != c0.device_ || c.rank_ != c0.rank_ + static_cast<int>(y) || c.world_ != c0.world_ ||
        c.rows_ != c0.rows_)
      throw std::invalid_argument("XgmiComm: a grouped launch needs consecutive ranks on one device");
    if ((reinterpret_cast<uintptr_t>(ins[y]) | reinterpret_cast<uintptr_t>(outs[y])) & 15)
      throw std::invalid_argument("XgmiComm: buffers must be 16-byte aligned");
  }
  if (c0.rows_ < 2)
    throw std::invalid_argument("allreduce_threshold: construct the comm with threshold_rows = maxLag + 1 >= 1");
  if (!(thr >= 0.f && thr <= 1.f && thc >= 0.f && thc <= 1.f))
    throw std::invalid_argument("allreduce_threshold: thresholds must be in [0, 1]");
  if (n <= 0) return false;
  const int W = c0.world_;
  if (W > 32) throw std::invalid_argument("allreduce_threshold: at most 32 ranks");
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  const int ranks_here = static_cast<int>(group.size());
  CommArgs& a = *static_cast<CommArgs*>(args);
  std::memset(&a, 0, sizeof(a));
  for (size_t y = 0; y < group.size(); ++y) {
    a.in[y] = static_cast<const char*>(ins[y]);
    a.out[y] = static_cast<char*>(outs[y]);
    a.ctl[y] = group[y]->ctl_;
  }
  int gx = 1;
  if (spec != nullptr && spec->block > 0) {  // the protocol's geometry (reference block ranges, maxChunkSize)
    if (spec->chunk <= 0) throw std::invalid_argument("round: chunk must be > 0");
    a.block = spec->block;
    a.chunk = spec->chunk;
    a.nch = static_cast<int>(std::max<int64_t>(1, ceil_div(a.block, a.chunk)));
    if (ranks_here != 1) throw std::invalid_argument("round: one rank per launch");
    gx = c0.round_grid(a.nch);
    // Fewer chunks than workgroups (big maxChunkSize): split each chunk into slices of at
    // least 64 KiB, one workgroup each, until the reduce phase covers the grid. A chunk stays
    // ONE threshold decision (xgmi_threshold.hip, split chunks).
    const int64_t min_slice = std::max<int64_t>(64, (int64_t{64} << 10) / es);
    if (spec->split_scratch != nullptr && W <= 30 && a.nch < c0.grid_ && a.chunk >= 2 * min_slice &&
        spec->split_bytes >= split_scratch_bytes(W, c0.maxch_)) {
      const int64_t S = std::min<int64_t>(ceil_div(c0.grid_, a.nch), a.chunk / min_slice);
      if (S > 1) {
        a.subchunk = round_up(ceil_div(a.chunk, S), 64);
        a.sub = static_cast<int>(ceil_div(a.chunk, a.subchunk));
        const int64_t units = static_cast<int64_t>(a.nch) * a.sub;
        gx = static_cast<int>(std::min<int64_t>(
            c0.grid_, std::max<int64_t>(units, ceil_div(static_cast<int64_t>(W - 1) * units, 1024))));
        char* sp = static_cast<char*>(spec->split_scratch);
        a.split_dec = reinterpret_cast<uint64_t*>(sp);
        a.split_ctr = reinterpret_cast<uint32_t*>(sp + static_cast<size_t>(W + 1) * c0.maxch_ * 8);
        a.split_early = reinterpret_cast<uint32_t*>(sp + static_cast<size_t>(W + 1) * c0.maxch_ * 12);
      }
    }
  } else {
    c0.geometry_threshold(n, dt, ranks_here, &a.block, &a.chunk, &a.nch, &gx);
  }
  if (a.block * es > c0.slot_bytes_ || a.nch > c0.maxch_)
    throw std::invalid_argument("allreduce_threshold: tensor exceeds one launch (n * dtype <= world * slot_bytes)");
  if (a.sub < 1) {  // unsplit: one workgroup per chunk
    a.sub = 1;
    a.subchunk = a.chunk;
  }
  // The reference's arrival order needs every reduce chunk of a workgroup in its launch
  // snapshot (xgmi_threshold.hip, S0); at thresholds 1 the order cannot change the result.
  if (spec != nullptr && spec->order_ref && !(thr >= 1.f && thc >= 1.f) &&
      ceil_div(static_cast<int64_t>(a.nch) * a.sub, gx) > kThresholdSnapChunks)
    throw std::invalid_argument("round: more than " + std::to_string(kThresholdSnapChunks) +
                                " chunks per workgroup at thresholds < 1 (the arrival-order snapshot)");
  // unsplit: scatter `sgroup` consecutive chunks per unit so that the (P - 1) x groups units
  // fit the grid once (at most 64: one flag lane each)
  a.sgroup = 1;
  if (a.sub <= 1 && W > 1) {
    const int per = std::max(1, gx / (W - 1));  // groups per destination block
    a.sgroup = static_cast<int>(std::min<int64_t>(64, std::max<int64_t>(1, ceil_div(a.nch, per))));
  }
  if (ceil_div(static_cast<int64_t>(W - 1) * a.nch * a.sub, gx) > kThresholdGatherUnits)
    throw std::invalid_argument("allreduce_threshold: more than " + std::to_string(kThresholdGatherUnits) +
                                " gather units per workgroup (too many chunks for the grid)");
  a.n = n;
  a.P = W;
  a.rows = c0.rows_;
  a.trows = c0.rows_ - 1;
  a.rank0 = c0.rank_;
  a.maxch = c0.maxch_;
  a.off_S = c0.off_S_;
  a.off_R = c0.off_R_;
  a.slot_bytes = c0.slot_stride_;
  a.slot_cap = c0.slot_bytes_;
  a.timeout = static_cast<uint64_t>(c0.timeout_s_ * 1e8);
  a.fence = c0.fence_;
  a.scale = scale;
  a.rescale = rescale ? 1 : 0;
  a.min_reduce = std::max(1, f32_threshold_count(thr, W));
  // thComplete: the reference's (th * P * nch) when every block has nch chunks; with a short
  // last block (uneven blocks) the chunks that exist, as the host WorkerCore
  // counts them (worker_core.cc) - the kernel never counts a chunk past a block's end
  int64_t total = 0;  // chunks that exist in the round
  {
    bool uniform = true;
    for (int j = 0; j < W; ++j) {
      const int64_t bl = std::max<int64_t>(0, std::min<int64_t>(a.block, n - static_cast<int64_t>(j) * a.block));
      const int64_t nc = ceil_div(bl, a.chunk);
      total += nc;
      uniform = uniform && nc == a.nch;
    }
    a.min_complete = uniform ? f32_threshold_chunks(thc, W, a.nch)
                             : std::max(1, f32_threshold_count(thc, static_cast<int>(total)));
  }
  a.full = (a.min_reduce >= W && thc >= 1.f) ? 1 : 0;
  // the lag-gate shortcut (xgmi_threshold.hip): rows for two rounds in flight, and a clean
  // round proves something about EVERY peer - each block holds a chunk, or nothing but a
  // complete round counts as clean (full thresholds)
  a.gate_shortcut = (c0.rows_ - 1 >= 2 && (a.full || n > static_cast<int64_t>(W - 1) * a.block) &&
                     !c0.no_gate_shortcut_) ? 1 : 0;
  // the one-shot body (xgmi_threshold.hip): full thresholds, unsplit, a small round whose chunk
  // boundaries fall on 4-B words (a low-latency word is 4 payload bytes) and whose
  // LL-encoded input (two bytes of slot per byte) fits one S slot
  {
    const int64_t nbytes = n * es;
    a.oneshot = (a.full && a.sub <= 1 && W <= kOneshotRanks && nbytes <= c0.th_oneshot_max_ && nbytes % 4 == 0 &&
                 (a.block * es) % 4 == 0 && (a.chunk * es) % 4 == 0 && 2 * round_up(nbytes, 8) <= c0.slot_bytes_)
                    ? 1
                    : 0;
    // the body reduces every chunk of the round (P x nch): as many chunks per workgroup as fit
    // its fast pass (one 8-B unit per thread, xgmi_threshold.hip), so the fewest workgroups
    // start (their start skew is on the round's critical path) and none walks chunks serially
    if (a.oneshot) {
      const int cap = ranks_here > 1 ? std::max(1, c0.shared_launch_cap(ranks_here)) : c0.grid_;
      const int64_t upc = ceil_div(std::min(a.chunk, a.block) * es, 8) + 1;  // units of one chunk at most
      const int64_t cpw = std::max<int64_t>(1, kCommThreads / upc);
      const int64_t need = ceil_div(static_cast<int64_t>(W) * a.nch, cpw);
      // only where the grid holds a workgroup for each of those groups: a grid too small for
      // that (a small default grid, a shared launch's cap) left workgroups walking several
      // chunks chunk by chunk, which timed out (MXAR_GRID=64, 8 x 128 KiB; profiles/round6
      // section 12). One chunk of more than kCommThreads units per workgroup stays one-shot
      // (every workgroup walks its one chunk: the plane's coarsened forced rounds, T13).
      if (need > cap)
        a.oneshot = 0;
      else
        gx = static_cast<int>(need);
    }
  }
  a.counts = counts;
  if (spec != nullptr) {
    a.epoch_set = spec->epoch;
    a.cold = spec->cold ? 1 : 0;
    a.order_ref = spec->order_ref ? 1 : 0;
    a.hforce = spec->host_force;
    a.habort = spec->host_abort;
    a.err_out = spec->err_out;
    a.done_out = spec->done_out;
    a.counts_host = counts != nullptr ? spec->counts_host : nullptr;
    // lag skip: unsplit chunks (a split chunk's slices publish one flag between them, so they
    // would have to agree on the skip) and thresholds under which a round can complete
    // without one peer - its contribution (min_reduce < P) and its block's chunks
    // (min_complete within the other blocks' chunks)
    if (spec->lag_wait_us >= 0.0 && a.sub <= 1 && W >= 2 && a.min_reduce < W && a.min_complete <= total - a.nch) {
      a.lag_skip = 1;
      a.lag_wait = static_cast<uint64_t>(spec->lag_wait_us * 100.0);  // s_memrealtime: 100 MHz
    }
  }
  a.delay_rank = -1;
  for (XgmiComm* c : group)
    if (c->delay_rank_ >= 0 && c->delay_us_ > 0) {
      a.delay_rank = c->delay_rank_;
      a.delay = static_cast<uint64_t>(c->delay_us_ * 100.0);  // s_memrealtime: 100 MHz
    }
  for (int k = 0; k < W; ++k) a.base[k] = c0.peers_[k];
  a.stamps = c0.stamps_;
  if (a.stamps != nullptr && gx * ranks_here > c0.stamp_slots_) a.stamps = nullptr;  // buffer too small: off
  *gx_out = gx;
  return true;
}

void XgmiComm::run_threshold(const std::vector<XgmiComm*>& group, const std::vector<const void*>& ins,
                             const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream, float thr,
                             float thc, int32_t* counts, float scale, bool rescale, const RoundSpec* spec) {
  CommArgs a;
  int gx = 1;
  if (!threshold_args(group, ins, outs, n, dt, thr, thc, counts, scale, rescale, spec, &a, &gx)) return;
  const XgmiComm& c0 = *group[0];
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  const int ranks_here = static_cast<int>(group.size());
  hip_check(hipSetDevice(c0.device_), "hipSetDevice");
  TraceScope span("xgmi", [&] {
    return std::make_pair("threshold " + std::to_string(n * es) + "B",
                          "{\"rank\":" + std::to_string(c0.rank_) + ",\"ranks_in_launch\":" +
                              std::to_string(ranks_here) + "}");
  });
  order_group(group, stream);
  launch_threshold(a, dim3(gx, ranks_here), stream, dt);
  hip_check(hipGetLastError(), "threshold launch");
  for (XgmiComm* c : group) {
    ++c->stats_.calls;
    ++c->stats_.launches;
    ++c->stats_.threshold;
    c->stats_.bytes += n * es;
  }
}

XgmiComm::ResidentPlan XgmiComm::plan_resident(int64_t n, DType dt, float th_reduce, float th_complete,
                                               const RoundSpec& spec, int max_grid, bool allow_split) const {
  ResidentPlan p;
  auto a = std::make_shared<CommArgs>();
  int gx = 0;
  XgmiComm* self = const_cast<XgmiComm*>(this);
  if (!threshold_args({self}, {nullptr}, {nullptr}, n, dt, th_reduce, th_complete, nullptr, 1.f, false, &spec,
                      a.get(), &gx))
    return p;
  // split chunks (the spec carried split scratch and the geometry used it) run on the launch
  // path of a lone worker; a plane group's kernel runs them
  if ((a->sub > 1 && !allow_split) || gx > max_grid || a->delay_rank >= 0) return p;  // big rounds / test knobs
  p.args = a;
  p.grid = gx;
  p.dt = dt;
  p.n = n;
  return p;
}

void XgmiComm::launch_resident(const ResidentPlan& p, const ResidentDoor* door, uint32_t* hstate, uint32_t* dm,
                               uint32_t seq, uint32_t gen, uint64_t idle_ticks, hipStream_t stream) {
  if (!p.args || p.grid <= 0) throw std::invalid_argument("launch_resident: no resident plan");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  order_after_last(stream);
  launch_threshold_resident(*static_cast<const CommArgs*>(p.args.get()), p.grid, stream, p.dt, door, hstate, dm, seq, gen,
                            idle_ticks);
  hip_check(hipGetLastError(), "resident threshold launch");
  ++stats_.launches;
}

void XgmiComm::publish_progress(uint32_t value, hipStream_t stream) {
  if (!connected_) throw std::runtime_error("XgmiComm: connect() first");
  if (rows_ < 2) throw std::invalid_argument("publish_progress: no threshold rows");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  CommArgs a;
  std::memset(&a, 0, sizeof(a));
  a.P = world_;
  a.rows = rows_;
  a.rank0 = rank_;
  a.maxch = maxch_;
  for (int k = 0; k < world_; ++k) a.base[k] = peers_[k];
  order_after_last(stream);
  launch_publish_progress(a, value, stream);
  hip_check(hipGetLastError(), "publish_progress launch");
}

void XgmiComm::round(const void* in, void* out, int64_t n, DType dt, hipStream_t stream, float th_reduce,
                     float th_complete, int32_t* counts, const RoundSpec& spec, float scale) {
  run_threshold({this}, {in}, {out}, n, dt, stream, th_reduce, th_complete, counts, scale, false, &spec);
}

// Two rounds of co-located workers may share a launch: the same geometry, thresholds and slabs.
static bool same_round_shape(const CommArgs& b, const CommArgs& a0) {
  bool same = b.n == a0.n && b.block == a0.block && b.chunk == a0.chunk && b.subchunk == a0.subchunk &&
              b.nch == a0.nch && b.sub == a0.sub && b.sgroup == a0.sgroup && b.P == a0.P && b.rows == a0.rows &&
              b.full == a0.full && b.min_reduce == a0.min_reduce &&
              b.min_complete == a0.min_complete && b.maxch == a0.maxch && b.off_S == a0.off_S && b.off_R == a0.off_R &&
              b.slot_bytes == a0.slot_bytes && b.order_ref == a0.order_ref && b.fence == a0.fence &&
              b.gate_shortcut == a0.gate_shortcut && b.scale == a0.scale && b.rescale == a0.rescale &&
              b.timeout == a0.timeout;
  for (int k = 0; same && k < a0.P; ++k) same = b.base[k] == a0.base[k];
  return same;
}

void XgmiComm::launch_group_resident(const std::vector<XgmiComm*>& comms, const std::vector<const ResidentPlan*>& plans,
                                     const std::vector<GroupResidentMember>& members, uint32_t* gstate, uint64_t* gdm,
                                     uint32_t gen, uint64_t idle_ticks, hipStream_t stream) {
  const int Y = static_cast<int>(plans.size());
  if (Y < 1 || Y > kMaxRanks || comms.size() != plans.size() || members.size() != plans.size())
    throw std::invalid_argument("launch_group_resident: one communicator, plan and member per worker, at most " +
                                std::to_string(kMaxRanks));
  for (const ResidentPlan* p : plans)
    if (p == nullptr || !p->args || p->grid <= 0) throw std::invalid_argument("launch_group_resident: no resident plan");
  const ResidentPlan& p0 = *plans[0];
  const CommArgs& a0 = *static_cast<const CommArgs*>(p0.args.get());
  CommArgs a = a0;
  GroupResArgs g;
  std::memset(&g, 0, sizeof(g));
  for (int y = 0; y < Y; ++y) {
    const ResidentPlan& p = *plans[y];
    const CommArgs& b = *static_cast<const CommArgs*>(p.args.get());
    if (p.grid != p0.grid || p.dt != p0.dt || p.n != p0.n || comms[y]->device_ != comms[0]->device_ ||
        !same_round_shape(b, a0))
      throw std::invalid_argument("launch_group_resident: the workers' rounds must share geometry and slabs");
    a.ctl[y] = comms[y]->ctl_;
    g.m[y] = members[y];
    g.m[y].rank = comms[y]->rank_;
    g.m[y].stamps = comms[y]->stamp_slots_ >= p0.grid ? comms[y]->stamps_ : nullptr;  // study knob
    g.m[y].split_dec = b.split_dec;  // each worker's own scratch (its plan's spec)
    g.m[y].split_ctr = b.split_ctr;
    g.m[y].split_early = b.split_early;
  }
  a.stamps = nullptr;
  a.delay_rank = -1;
  g.gstate = gstate;
  g.gdm = gdm;
  g.idle = idle_ticks;
  g.gen = gen;
  g.Y = Y;
  hip_check(hipSetDevice(comms[0]->device_), "hipSetDevice");
  order_group(comms, stream);
  launch_threshold_group_resident(a, g, p0.grid, stream, p0.dt);
  hip_check(hipGetLastError(), "group resident threshold launch");
  for (XgmiComm* c : comms) ++c->stats_.launches;
}

void XgmiComm::allreduce_threshold(const void* in, void* out, int64_t n, DType dt, hipStream_t stream,
                                   float th_reduce, float th_complete, int32_t* counts, float scale, bool rescale) {
  run_threshold({this}, {in}, {out}, n, dt, stream, th_reduce, th_complete, counts, scale, rescale);
}

void XgmiComm::allreduce_threshold_local(const std::vector<XgmiComm*>& comms, const std::vector<const void*>& ins,
                                         const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream,
                                         float th_reduce, float th_complete, int32_t* counts, float scale,
                                         bool rescale) {
  run_threshold(comms, ins, outs, n, dt, stream, th_reduce, th_complete, counts, scale, rescale);
}

void XgmiComm::barrier_group(const std::vector<XgmiComm*>& group, hipStream_t stream) {
  const XgmiComm& c0 = *group[0];
  for (XgmiComm* c : group)
    if (!c->connected_) throw std::runtime_error("XgmiComm: connect() first");
  hip_check(hipSetDevice(c0.device_), "hipSetDevice");
  CommArgs a;
  std::memset(&a, 0, sizeof(a));
  for (size_t y = 0; y < group.size(); ++y) a.ctl[y] = group[y]->ctl_;
  a.P = c0.world_;
  a.rows = c0.rows_;
  a.rank0 = c0.rank_;
  a.maxch = c0.maxch_;
  a.timeout = static_cast<uint64_t>(c0.timeout_s_ * 1e8);
  a.fence = 3;
  for (int k = 0; k < c0.world_; ++k) a.base[k] = c0.peers_[k];
  order_group(group, stream);
  hipLaunchKernelGGL(barrier_kernel, dim3(1, static_cast<unsigned>(group.size())), dim3(kCommThreads), 0, stream, a);
  hip_check(hipGetLastError(), "barrier launch");
}

void XgmiComm::barrier(hipStream_t stream) { barrier_group({this}, stream); }

void XgmiComm::run_coll(const std::vector<XgmiComm*>& group, Coll op, const std::vector<const void*>& ins,
                        const std::vector<void*>& outs, int64_t m, DType dt, hipStream_t stream, float scale) {
  if (group.empty() || ins.size() != group.size() || outs.size() != group.size())
    throw std::invalid_argument("XgmiComm: one input and one output per rank");
  const XgmiComm& c0 = *group[0];
  const int W = c0.world_;
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  const int64_t in_blocks = op == Coll::AllGather ? 1 : W, out_blocks = op == Coll::ReduceScatter ? 1 : W;
  for (size_t y = 0; y < group.size(); ++y) {
    const XgmiComm& c = *group[y];
    if (!c.connected_) throw std::runtime_error("XgmiComm: connect() first");
    if (c.device_ != c0.device_ || c.rank_ != c0.rank_ + static_cast<int>(y) || c.world_ != W)
      throw std::invalid_argument("XgmiComm: a grouped launch needs consecutive ranks on one device");
    const uintptr_t i0 = reinterpret_cast<uintptr_t>(ins[y]), o0 = reinterpret_cast<uintptr_t>(outs[y]);
    if ((i0 | o0) & 15) throw std::invalid_argument("XgmiComm: buffers must be 16-byte aligned");
    if (i0 < o0 + static_cast<uintptr_t>(out_blocks * m * es) && o0 < i0 + static_cast<uintptr_t>(in_blocks * m * es))
      throw std::invalid_argument("XgmiComm: collective input and output must not overlap");
  }
  if ((m * es) & 15) throw std::invalid_argument("XgmiComm: block size (m x dtype) must be a multiple of 16 bytes");
  if (m <= 0) return;
  hip_check(hipSetDevice(c0.device_), "hipSetDevice");
  for (XgmiComm* c : group) {
    ++c->stats_.calls;
    c->stats_.bytes += in_blocks * m * es;
  }
  order_group(group, stream);
  if (W == 1) {  // one rank: a copy (scaled for reduce-scatter)
    for (size_t y = 0; y < group.size(); ++y) {
      if (op == Coll::ReduceScatter && scale != 1.f)
        launch_reduce_slots(ins[y], m, 1, outs[y], m, dt, scale, stream);
      else
        launch_copy(ins[y], outs[y], m * es, stream);
    }
    return;
  }
  static const char* names[] = {"all_to_all ", "all_gather ", "reduce_scatter "};
  TraceScope span("xgmi", [&] {
    return std::make_pair(std::string(names[static_cast<int>(op)]) + std::to_string(in_blocks * m * es) + "B",
                          "{\"rank\":" + std::to_string(c0.rank_) + ",\"ranks_in_launch\":" +
                              std::to_string(group.size()) + "}");
  });
  const int ranks_here = static_cast<int>(group.size());
  const int gmax = std::max(1, c0.grid_ / ranks_here);
  const int64_t elems = 16 / es, min_chunk = min_chunk_bytes() / es;
  const int64_t seg = c0.slot_bytes_ / es;  // per block per launch
  for (int64_t off = 0; off < m; off += seg) {
    const int64_t len = std::min(seg, m - off);
    CommArgs a;
    std::memset(&a, 0, sizeof(a));
    for (size_t y = 0; y < group.size(); ++y) {
      a.in[y] = static_cast<const char*>(ins[y]) + off * es;
      a.out[y] = static_cast<char*>(outs[y]) + off * es;
      a.ctl[y] = group[y]->ctl_;
    }
    a.n = len;
    a.block = m;
    a.P = W;
    a.rows = c0.rows_;
    a.rank0 = c0.rank_;
    a.maxch = c0.maxch_;
    a.off_S = c0.off_S_;
    a.off_R = c0.off_R_;
    a.slot_bytes = c0.slot_stride_;
    a.slot_cap = c0.slot_bytes_;
    a.timeout = static_cast<uint64_t>(c0.timeout_s_ * 1e8);
    a.fence = c0.fence_;
    a.scale = scale;
    a.rdelay_rank = c0.rdelay_rank_;
    a.rdelay = c0.rdelay_us_ > 0 ? static_cast<uint64_t>(c0.rdelay_us_ * 100.0) : 0;
    a.noguard = c0.noguard_ ? 1 : 0;
    for (int k = 0; k < W; ++k) a.base[k] = c0.peers_[k];
    // launch-size grid as for the two-shot (launch_grid), over P x block bytes per rank: a
    // block goes to every peer (all-gather) or P blocks come in (all-to-all, reduce-scatter).
    // 8 / 2 logical ranks x 128 KiB - 8 MiB blocks, grid 64 - 512 (coll_grid_sweep.jsonl):
    // 8 x 512 KiB all-gather 58.4 -> 50.1 us, all-to-all 50.7 -> 41.2, reduce-scatter 44.9 ->
    // 35.4; the full grid pays off from 512 MiB (all-gather, all-to-all) / not yet at 512 MiB
    // for the reduce-scatter (8 x 8 MiB: 331 us full vs 284 us at 256).
    int gcap = gmax;
    if (c0.size_grid_ && c0.grid_ == c0.default_grid_) {
      const int64_t bytes = static_cast<int64_t>(ranks_here) * W * len * es;
      const int64_t full_at = op == Coll::ReduceScatter ? (int64_t{1} << 30) : (int64_t{512} << 20);
      if (bytes < full_at) gcap = std::max(1, size_grid_rule(bytes, c0.grid_, W, false, full_at) / ranks_here);
    }
    const int64_t target = std::max<int64_t>(1, gcap / (W - 1));
    a.chunk = std::max(min_chunk, round_up(ceil_div(len, target), elems));
    a.nch = static_cast<int>(std::max<int64_t>(1, ceil_div(len, a.chunk)));
    a.subchunk = a.chunk;
    a.sub = 1;
    if (op == Coll::ReduceScatter) {  // reduce units = push units: split every chunk W-1 ways
      const int64_t sub = std::max<int64_t>(1, std::min<int64_t>(W - 1, a.chunk / min_chunk));
      a.subchunk = round_up(ceil_div(a.chunk, sub), elems);
      a.sub = static_cast<int>(ceil_div(a.chunk, a.subchunk));
    }
    if (a.nch > c0.maxch_) throw std::logic_error("XgmiComm: collective geometry exceeds the flag table");
    const int gx = static_cast<int>(std::min<int64_t>(gcap, std::max<int64_t>(1, (W - 1) * int64_t{a.nch})));
    launch_coll(a, dim3(gx, ranks_here), stream, dt, static_cast<int>(op));
    hip_check(hipGetLastError(), "collective launch");
    for (XgmiComm* c : group) {
      ++c->stats_.launches;
      ++c->stats_.coll;
    }
  }
}

void XgmiComm::collective(Coll op, const void* in, void* out, int64_t m, DType dt, hipStream_t stream, float scale) {
  run_coll({this}, op, {in}, {out}, m, dt, stream, scale);
}

void XgmiComm::collective_local(const std::vector<XgmiComm*>& comms, Coll op, const std::vector<const void*>& ins,
                                const std::vector<void*>& outs, int64_t m, DType dt, hipStream_t stream,
                                float scale) {
  run_coll(comms, op, ins, outs, m, dt, stream, scale);
}

}  // namespace mxar
