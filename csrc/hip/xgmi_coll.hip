// Direct all-to-all, all-gather and reduce-scatter over xGMI (gfx950).
//
// The reference only ever allreduces, but its two phases are these collectives: the
// ScatterBlock fan-out (AllreduceWorker.scala:194-209) is an all-to-all of blocks, the
// owner's reduce of what it received is a reduce-scatter (:240-251), and the ReduceBlock
// broadcast (:230-238) is an all-gather. Split out, they are the collectives DP-with-sharding
// (reduce-scatter / all-gather), TP/SP and expert parallelism (all-to-all) need, and each
// runs as ONE launch that drives all P-1 links at once:
//   all_to_all     : in[P][m] -> out[P][m], out_r[s] = in_s[r]
//   all_gather     : in[m]    -> out[P][m], out_r[s] = in_s
//   reduce_scatter : in[P][m] -> out[m],    out_r   = scale * sum_s in_s[r] (fp32, rank order)
// Phase 1 pushes block j (chunked) into rank j's S (or R) slot with write-through stores and
// a flag per chunk; phase 2 waits per chunk and copies (or reduces) out of the own slab.
// Slot reuse: phase 1 waits (entry_guard, xgmi_device.h) until the target peers have
// finished reading the region in an earlier launch, and the last workgroup tells every peer
// when this launch's slab reads are done (FB words) - no end-of-launch barrier, so a fast
// rank leaves as soon as its own data is out.
#include <hip/hip_runtime.h>

#include "xgmi_device.h"

namespace mxar {

namespace {

template <class E>
__device__ __forceinline__ void copy_plain(char* dst, const char* src, int64_t len) {
  const int64_t npk = len / E::ELEMS;
  for (int64_t i = threadIdx.x; i < npk; i += kCommThreads) st16(dst + i * 16, ld16(src + i * 16));
  const int64_t t = npk * E::ELEMS + threadIdx.x;
  if (t < len) Scalar<E>::copy(dst, src, t);
}

}  // namespace

// MODE: 0 all-to-all, 1 all-gather, 2 reduce-scatter. a.block = block stride (elements) in
// the [P][m] buffers, a.n = elements of this segment per block.
template <class E, int MODE, int PT>
__global__ __launch_bounds__(kCommThreads) void coll_kernel(CommArgs a) {
  constexpr int es = 16 / E::ELEMS;
  const int P = a.P;
  const int y = blockIdx.y;
  const int r = a.rank0 + y;
  const char* const in = a.in[y];
  char* const out = a.out[y];
  uint32_t* const ctl = a.ctl[y];
  uint32_t* const err = &ctl[2];
  const uint32_t epoch = launch_epoch(ctl);
  const uint64_t deadline = wall_ticks() + a.timeout;
  const int G = gridDim.x;
  const int64_t slot = a.slot_bytes;
  const int64_t bs = a.block;
  const bool rel = a.fence & 1, acq = a.fence & 2;
  const int Pm1 = P > 1 ? P - 1 : 1;
  const int nu = (P - 1) * a.nch;

  constexpr uint32_t region = MODE == 1 ? kHazR : kHazS;
  // Phase 1: push this rank's part for peer j into j's slab (rotated peer order)
  if (static_cast<int>(blockIdx.x) < nu) entry_guard(a, ctl, r, epoch, region, -1, deadline, err);
  for (int u = blockIdx.x; u < nu; u += G) {
    const int c = u / Pm1;
    const int j = (r + 1 + u % Pm1) % P;
    const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
    const int64_t len = clamp_len(a.n - cstart, a.chunk);
    const char* src = MODE == 1 ? in + cstart * es : in + (static_cast<int64_t>(j) * bs + cstart) * es;
    char* dst = a.base[j] + (MODE == 1 ? a.off_R : a.off_S) + r * slot + cstart * es;
    if (len > 0 && unit_in_bounds(a, cstart * es, len * es, c, err)) copy_to_slab<E>(dst, src, len);
    publish_flags([&](int) { return MODE == 1 ? f2(a, j, r, c) : f1(a, j, r, c); }, 1, epoch, rel);
  }

  read_delay(a, r);
  if constexpr (MODE == 2) {
    // Phase 2 (reduce-scatter): own block r = own input + the P-1 received contributions.
    // Each chunk is reduced in `sub` pieces by different workgroups (as many reduce units as
    // push units), all P loads of a pack in flight (static P).
    const int nu2 = a.nch * a.sub;
    for (int u = blockIdx.x; u < nu2; u += G) {
      const int c = u / a.sub;
      const int q = u % a.sub;
      const int64_t cstart = static_cast<int64_t>(c) * a.chunk + static_cast<int64_t>(q) * a.subchunk;
      const int64_t len = clamp_len(clamp_len(a.n - static_cast<int64_t>(c) * a.chunk, a.chunk) -
                                        static_cast<int64_t>(q) * a.subchunk,
                                    a.subchunk);
      wait_flags([&](int s) -> const uint32_t* { return s == r ? nullptr : f1(a, r, s, c); }, P, epoch, deadline,
                 err, ERR_TIMEOUT_SCATTER, acq);
      if (len > 0 && unit_in_bounds(a, cstart * es, len * es, c, err)) {
        const RedSrc src{in + (static_cast<int64_t>(r) * bs + cstart) * es, a.base[r] + a.off_S + cstart * es, slot,
                         r};
        char* o = out + cstart * es;
        reduce_to<E, PT>(P, src, 1, 0, [&](int) -> char* { return o; }, len, a.scale, a.fence & 1);
      }
    }
  } else {
    // own block: no transfer
    for (int c = blockIdx.x; c < a.nch; c += G) {
      const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
      const int64_t len = clamp_len(a.n - cstart, a.chunk);
      const char* src = MODE == 1 ? in + cstart * es : in + (static_cast<int64_t>(r) * bs + cstart) * es;
      if (len > 0) copy_plain<E>(out + (static_cast<int64_t>(r) * bs + cstart) * es, src, len);
    }
    // Phase 2: block of source s out of the own slab
    for (int u = blockIdx.x; u < nu; u += G) {
      const int c = u / Pm1;
      const int s = (r + 1 + u % Pm1) % P;
      const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
      const int64_t len = clamp_len(a.n - cstart, a.chunk);
      wait_flags([&](int) -> const uint32_t* { return MODE == 1 ? f2(a, r, s, c) : f1(a, r, s, c); }, 1, epoch,
                 deadline, err, ERR_TIMEOUT_SCATTER, acq);
      if (len > 0 && unit_in_bounds(a, cstart * es, len * es, c, err))
        copy_from_slab<E>(out + (static_cast<int64_t>(s) * bs + cstart) * es,
                          a.base[r] + (MODE == 1 ? a.off_R : a.off_S) + s * slot + cstart * es, len);
    }
  }
  finish_launch_done(a, ctl, epoch, r, region);
}

void launch_coll(const CommArgs& a, dim3 grid, hipStream_t s, DType dt, int mode) {
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    using E = decltype(tag);
    if (mode == 0) {
      hipLaunchKernelGGL((coll_kernel<E, 0, 0>), grid, dim3(kCommThreads), 0, s, a);
    } else if (mode == 1) {
      hipLaunchKernelGGL((coll_kernel<E, 1, 0>), grid, dim3(kCommThreads), 0, s, a);
    } else {
      switch (a.P) {
        case 2: hipLaunchKernelGGL((coll_kernel<E, 2, 2>), grid, dim3(kCommThreads), 0, s, a); break;
        case 4: hipLaunchKernelGGL((coll_kernel<E, 2, 4>), grid, dim3(kCommThreads), 0, s, a); break;
        case 8: hipLaunchKernelGGL((coll_kernel<E, 2, 8>), grid, dim3(kCommThreads), 0, s, a); break;
        default: hipLaunchKernelGGL((coll_kernel<E, 2, 0>), grid, dim3(kCommThreads), 0, s, a); break;
      }
    }
  });
}

}  // namespace mxar
