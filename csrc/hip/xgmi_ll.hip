// Low-latency one-shot allreduce over xGMI (gfx950): flags travel inside the data.
//
// The lock-step kernels hand each chunk over with payload stores -> drain -> system-scope
// release -> flag store, and the consumer polls the flag, then acquires, then loads: two
// xGMI round trips per hand-off plus the fences. For small tensors that hand-off is most
// of the latency. Here every 16-B store carries two 8-byte words {payload u32, epoch u32}:
// an aligned 8-byte store is delivered whole, so a reader that sees the epoch in a word
// also sees that word's payload - no fence, no separate flag, one hop. Half of every
// store is flag, so this is for small tensors only (ll_max_bytes, default 512 KiB).
//
//   rank r, payload unit i (8 bytes of its input):
//     push   : LL_k[par][r][i] = {in[i].lo, e, in[i].hi, e}   for every peer k != r
//     reduce : out[i] = sum over s of (s == r ? in[i] : LL_r[par][s][i] once both epochs == e)
// The same thread pushes and reduces unit i, so in-place calls are safe. LL slots are
// double-buffered by the launch epoch's parity: a rank can run at most one launch ahead
// of a peer that is still reading (finishing launch e needs every peer's data of e), so
// the slot it writes next is never the one being read. Epochs come from the same device
// counter as the other kernels (ctl[0]) and are never 0, the value the slab starts with.
#include <hip/hip_runtime.h>

#include "xgmi_device.h"

namespace mxar {

namespace {

constexpr int kAuxSys = 17;  // sc0 | sc1: system-coherent (loads see peers' xGMI stores in HBM)

// 8 payload bytes at unit i of a byte range of length nbytes (zero-padded past the end).
__device__ __forceinline__ uint2 load_unit(const char* p, int64_t i, int64_t nbytes) {
  const int64_t off = i * 8;
  if (off + 8 <= nbytes) return *reinterpret_cast<const uint2*>(p + off);
  uint32_t w[2] = {0u, 0u};
  const uint16_t* h = reinterpret_cast<const uint16_t*>(p + off);
  for (int k = 0; k < 4 && off + 2 * k < nbytes; ++k)
    w[k >> 1] |= static_cast<uint32_t>(h[k]) << (16 * (k & 1));
  return make_uint2(w[0], w[1]);
}

__device__ __forceinline__ void store_unit(char* p, int64_t i, int64_t nbytes, uint2 v) {
  const int64_t off = i * 8;
  if (off + 8 <= nbytes) {
    *reinterpret_cast<uint2*>(p + off) = v;
    return;
  }
  uint16_t* h = reinterpret_cast<uint16_t*>(p + off);
  const uint32_t w[2] = {v.x, v.y};
  for (int k = 0; k < 4 && off + 2 * k < nbytes; ++k) h[k] = static_cast<uint16_t>(w[k >> 1] >> (16 * (k & 1)));
}

}  // namespace

template <class E>
__global__ __launch_bounds__(kCommThreads) void oneshot_ll_kernel(CommArgs a) {
  constexpr int es = 16 / E::ELEMS;
  const int P = a.P;
  const int y = blockIdx.y;
  const int r = a.rank0 + y;
  const char* const in = a.in[y];
  char* const out = a.out[y];
  uint32_t* const ctl = a.ctl[y];
  uint32_t* const err = &ctl[2];
  const uint32_t epoch = launch_epoch(ctl);
  const int par = static_cast<int>(epoch & 1u);
  const uint64_t deadline = wall_ticks() + a.timeout;
  const int64_t nbytes = a.n * es;
  const int64_t units = (nbytes + 7) / 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kCommThreads;
  const int64_t first = static_cast<int64_t>(blockIdx.x) * kCommThreads + threadIdx.x;
  auto slot = [&](int k, int s) {  // LL slot of source s in rank k's slab
    return a.base[k] + a.off_LL + (static_cast<int64_t>(par) * P + s) * a.ll_slot;
  };
  if (units * 16 > a.ll_slot) {  // host guarantees this; never store out of bounds
    if (threadIdx.x == 0) __hip_atomic_fetch_or(err, ERR_BAD_ARGS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    finish_launch(ctl, epoch);
    return;
  }

  // push: one 16-B store = two {payload, epoch} words, to every peer
  for (int64_t i = first; i < units; i += stride) {
    const uint2 d = load_unit(in, i, nbytes);
    Pack16 v;
    v[0] = d.x;
    v[1] = epoch;
    v[2] = d.y;
    v[3] = epoch;
    for (int k = 0; k < P; ++k)
      if (k != r) st16_wt(slab_rsrc(slot(k, r)), static_cast<uint32_t>(i * 16), v);
  }

  // reduce: own unit from the input, peers' units from the own slab once their epochs show
  bool late = false;
  // The peers' units of a batch of B sources are loaded together (one load latency per
  // batch instead of one per source), then each is re-polled only if its epoch is not in yet;
  // the sum keeps the fixed order s = 0..P-1.
  constexpr int B = 8;
  for (int64_t i = first; i < units; i += stride) {
    Acc8<E> acc;
    for (int s0 = 0; s0 < P; s0 += B) {
      Pack16 v[B];
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const int s = s0 + b;
        if (s < P && s != r)
          v[b] = __builtin_amdgcn_raw_buffer_load_b128(slab_rsrc(slot(r, s)), static_cast<int>(i * 16), 0, kAuxSys);
      }
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const int s = s0 + b;
        if (s >= P) continue;
        if (s == r) {
          acc.add(load_unit(in, i, nbytes));
          continue;
        }
        const __amdgpu_buffer_rsrc_t rs = slab_rsrc(slot(r, s));
        Pack16 w = v[b];
        while ((w[1] != epoch || w[3] != epoch) && !late) {
          __builtin_amdgcn_s_sleep(1);
          w = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(i * 16), 0, kAuxSys);
          if (wall_ticks() > deadline) late = true;
        }
        if (w[1] == epoch && w[3] == epoch) acc.add(make_uint2(w[0], w[2]));
      }
    }
    store_unit(out, i, nbytes, acc.pack(a.scale));
  }
  if (late) __hip_atomic_fetch_or(err, ERR_TIMEOUT_SCATTER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  finish_launch(ctl, epoch);
}

void launch_ll(const CommArgs& a, dim3 grid, hipStream_t s, DType dt) {
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    hipLaunchKernelGGL(oneshot_ll_kernel<decltype(tag)>, grid, dim3(kCommThreads), 0, s, a);
  });
}

}  // namespace mxar
