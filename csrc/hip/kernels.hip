// Standalone data-plane kernels (gfx950), all HBM-bound, 16 B per lane:
//   reduce_slots  - K1 of SURVEY §2.4: out[i] = sum_p slot[p][i] (AllreduceWorker.scala:240-251),
//                   fp32 accumulation in fixed peer order, optional scale (mean).
//   fill_iota     - K9: reference data source data[i] = i + iteration (AllreduceWorker.scala:285-291)
//   fill_uniform  - synthetic random gradients for the benchmarks (counter-based hash, no state)
//   cast          - fp32 <-> bf16
//   bucket_copy   - gather many gradient tensors into one flat bucket and scatter back
//                   (bucket fusion for the data-parallel reducer)
// Grids are grid-stride, capped at 8 workgroups per CU (cdna_hip_programming.md Guideline 11).
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include <algorithm>

#include "device_common.h"
#include "xgmi_comm.h"

namespace mxar {
using namespace dev;

static constexpr int kThreads = 256;

static int grid_for(int64_t packs) {
  static int cap = 0;
  if (cap == 0) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    cap = 8 * cus;
  }
  const int64_t g = (packs + kThreads - 1) / kThreads;
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(g, cap)));
}

// Tiled like the fastest copy variant: each workgroup sweeps contiguous tiles of
// U x 4 KiB per slot (one 1 KiB wave access per pack), tiles dealt grid-stride.
// P is a template parameter for 2..8 slots so every slot's loads of a tile are issued
// before the first add (P*U*16 bytes in flight per lane); the sum still runs in peer
// order 0..P-1. NT bit 0 = nontemporal loads, bit 1 = nontemporal stores (streaming data,
// no reuse), bit 2 = write-through (sc0 sc1) stores - the store probe's fastest copy pairs nt
// loads with them (round-3 store probe, profiles/round3/store_probe.json).
// out may alias one slot row (in-place reduce): every element is read and written by the
// same lane, loads before the store.
template <class E, int U, int P, int NT>
__global__ __launch_bounds__(kThreads) void reduce_slots_static(const char* __restrict__ slots, int64_t stride_bytes,
                                                                char* out, int64_t n, float scale) {
  constexpr int64_t kTile = static_cast<int64_t>(U) * kThreads;
  const int64_t npk = n / E::ELEMS;
  const int64_t ntiles = npk / kTile;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t base = t * kTile + threadIdx.x;
    Pack16 v[P][U];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const Pack16* s = reinterpret_cast<const Pack16*>(slots + p * stride_bytes);
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[p][u] = (NT & 1) ? __builtin_nontemporal_load(s + base + u * kThreads) : s[base + u * kThreads];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      Acc<E> a;
      a.zero();
#pragma unroll
      for (int p = 0; p < P; ++p) a.add(v[p][u]);
      if (scale != 1.f) a.scale(scale);
      Pack16* d = reinterpret_cast<Pack16*>(out) + base + u * kThreads;
      if (NT & 4)  // sc0 sc1 write-through buffer store (aux 17), offset from the tile's base
        __builtin_amdgcn_raw_buffer_store_b128(a.pack(), slab_rsrc(out + t * kTile * 16),
                                               static_cast<int>((threadIdx.x + u * kThreads) * 16), 0, 17);
      else if (NT & 2)
        __builtin_nontemporal_store(a.pack(), d);
      else
        *d = a.pack();
    }
  }
  for (int64_t i = ntiles * kTile + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < npk;
       i += static_cast<int64_t>(gridDim.x) * kThreads) {
    Acc<E> a0;
    a0.zero();
#pragma unroll
    for (int p = 0; p < P; ++p) a0.add(ld16(slots + p * stride_bytes + i * 16));
    if (scale != 1.f) a0.scale(scale);
    st16(out + i * 16, a0.pack());
  }
  const int64_t t = npk * E::ELEMS + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (t < n) {
    float acc = 0.f;
#pragma unroll
    for (int p = 0; p < P; ++p) acc += Scalar<E>::load(slots + p * stride_bytes, t);
    Scalar<E>::store(out, t, acc * scale);
  }
}

// Any slot count: the runtime-P loop (loads of one slot in flight at a time).
template <class E>
__global__ __launch_bounds__(kThreads) void reduce_slots_kernel(const char* __restrict__ slots, int64_t stride_bytes,
                                                                int nslots, char* out, int64_t n, float scale) {
  constexpr int U = 2;
  constexpr int64_t kTile = static_cast<int64_t>(U) * kThreads;
  const int64_t npk = n / E::ELEMS;
  const int64_t ntiles = npk / kTile;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t base = t * kTile + threadIdx.x;
    Acc<E> a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u].zero();
    for (int p = 0; p < nslots; ++p) {
      const char* s = slots + p * stride_bytes;
      Pack16 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld16(s + (base + u * kThreads) * 16);
#pragma unroll
      for (int u = 0; u < U; ++u) a[u].add(v[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (scale != 1.f) a[u].scale(scale);
      st16(out + (base + u * kThreads) * 16, a[u].pack());
    }
  }
  for (int64_t i = ntiles * kTile + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < npk;
       i += static_cast<int64_t>(gridDim.x) * kThreads) {
    Acc<E> a0;
    a0.zero();
    for (int p = 0; p < nslots; ++p) a0.add(ld16(slots + p * stride_bytes + i * 16));
    if (scale != 1.f) a0.scale(scale);
    st16(out + i * 16, a0.pack());
  }
  const int64_t t = npk * E::ELEMS + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (t < n) {
    float acc = 0.f;
    for (int p = 0; p < nslots; ++p) acc += Scalar<E>::load(slots + p * stride_bytes, t);
    Scalar<E>::store(out, t, acc * scale);
  }
}

static int g_reduce_variant = -1;  // -1: default (see launch_reduce_slots)

void set_reduce_variant(int v) { g_reduce_variant = v; }

template <class E, int U, int NT>
static void launch_static(int P, const char* s, int64_t stride, char* o, int64_t n, float scale, int g,
                          hipStream_t st) {
#define MXAR_RS(PP)                                                                                            \
  case PP:                                                                                                     \
    hipLaunchKernelGGL((reduce_slots_static<E, U, PP, NT>), dim3(g), dim3(kThreads), 0, st, s, stride, o, n, \
                       scale);                                                                                 \
    break;
  switch (P) {
    MXAR_RS(1) MXAR_RS(2) MXAR_RS(3) MXAR_RS(4) MXAR_RS(5) MXAR_RS(6) MXAR_RS(7) MXAR_RS(8)
    default: hipLaunchKernelGGL(reduce_slots_kernel<E>, dim3(g), dim3(kThreads), 0, st, s, stride, P, o, n, scale);
  }
#undef MXAR_RS
}

template <class E>
static void launch_reduce_typed(int v, int P, const char* s, int64_t stride, char* o, int64_t n, float scale,
                                hipStream_t st) {
  const int64_t npk = n / E::ELEMS;
  auto grid = [&](int U) {
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(npk / (int64_t(U) * kThreads), 2048)));
  };
  switch (v) {
    case 0: hipLaunchKernelGGL(reduce_slots_kernel<E>, dim3(grid(2)), dim3(kThreads), 0, st, s, stride, P, o, n, scale);
      break;
    case 1: launch_static<E, 2, 0>(P, s, stride, o, n, scale, grid(2), st); break;
    case 2: launch_static<E, 2, 3>(P, s, stride, o, n, scale, grid(2), st); break;
    case 3: launch_static<E, 4, 3>(P, s, stride, o, n, scale, grid(4), st); break;
    case 5: launch_static<E, 2, 3>(P, s, stride, o, n, scale, grid(2), st); break;
    case 6: launch_static<E, 8, 3>(P, s, stride, o, n, scale, grid(8), st); break;
    case 7:  // U by slot count: ~ the same bytes in flight per lane for every P
      if (P > 4) launch_static<E, 2, 3>(P, s, stride, o, n, scale, grid(2), st);
      else launch_static<E, 4, 3>(P, s, stride, o, n, scale, grid(4), st);
      break;
    case 8: launch_static<E, 4, 1>(P, s, stride, o, n, scale, grid(4), st); break;  // NT loads only
    case 9: launch_static<E, 4, 2>(P, s, stride, o, n, scale, grid(4), st); break;  // NT stores only
    case 10: launch_static<E, 4, 5>(P, s, stride, o, n, scale, grid(4), st); break;  // NT loads, write-through stores
    case 11: launch_static<E, 8, 5>(P, s, stride, o, n, scale, grid(8), st); break;
    default: launch_static<E, 4, 0>(P, s, stride, o, n, scale, grid(4), st); break;
  }
}

void launch_reduce_slots(const void* slots, int64_t slot_stride_elems, int nslots, void* out, int64_t n, DType dt,
                         float scale, hipStream_t stream) {
  if (n <= 0) return;
  const int64_t es = static_cast<int64_t>(dtype_size(dt));
  if (((reinterpret_cast<uintptr_t>(slots) | reinterpret_cast<uintptr_t>(out)) & 15) || ((slot_stride_elems * es) & 15))
    throw std::invalid_argument("reduce_slots: slots, out and slot stride must be 16-byte aligned");
  const int v = g_reduce_variant < 0 ? 3 : g_reduce_variant;  // 3: measured fastest (profiles/reduce_kernel.md)
  const char* s = static_cast<const char*>(slots);
  char* o = static_cast<char*>(out);
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    launch_reduce_typed<decltype(tag)>(v, nslots, s, slot_stride_elems * es, o, n, scale, stream);
  });
  hip_check(hipGetLastError(), "reduce_slots launch");
}

template <class E>
__global__ __launch_bounds__(kThreads) void fill_affine_kernel(char* out, int64_t n, double slope, double offset) {
  const int64_t step = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n; i += step)
    Scalar<E>::store(out, i, static_cast<float>(slope * static_cast<double>(i) + offset));
}

void launch_fill_affine(void* dst, int64_t n, double slope, double offset, DType dt, hipStream_t stream) {
  if (n <= 0) return;
  const int g = grid_for(n);
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    hipLaunchKernelGGL(fill_affine_kernel<decltype(tag)>, dim3(g), dim3(kThreads), 0, stream, static_cast<char*>(dst),
                       n, slope, offset);
  });
  hip_check(hipGetLastError(), "fill_affine launch");
}

void launch_fill_iota(void* dst, int64_t n, double offset, DType dt, hipStream_t stream) {
  launch_fill_affine(dst, n, 1.0, offset, dt, stream);
}

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

template <class E>
__global__ __launch_bounds__(kThreads) void fill_uniform_kernel(char* out, int64_t n, uint64_t seed) {
  const int64_t step = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n; i += step) {
    const uint32_t h = hash32(seed * 0x9E3779B97F4A7C15ULL + static_cast<uint64_t>(i));
    const float u = static_cast<float>(h >> 8) * (1.0f / 16777216.0f);  // [0, 1)
    Scalar<E>::store(out, i, 2.f * u - 1.f);
  }
}

void launch_fill_uniform(void* dst, int64_t n, uint64_t seed, DType dt, hipStream_t stream) {
  if (n <= 0) return;
  const int g = grid_for(n);
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    hipLaunchKernelGGL(fill_uniform_kernel<decltype(tag)>, dim3(g), dim3(kThreads), 0, stream, static_cast<char*>(dst),
                       n, seed);
  });
  hip_check(hipGetLastError(), "fill_uniform launch");
}

// Clock probe (study tool, tools/overlap_trace.py): ONE wave samples the shader-clock counter
// (s_memtime, counts core clock cycles - power management moves it) against the constant
// 100 MHz counter (s_memrealtime) every `interval` ticks, `samples` times, into
// out[2 * i] / out[2 * i + 1]. Sharing the GPU with other work it reports the core clock
// that work ran at; it exits after `samples` samples (bounded: samples x interval ticks).
__global__ __launch_bounds__(64) void clock_probe_kernel(uint64_t* out, int samples, uint64_t interval) {
  if (threadIdx.x != 0) return;
  uint64_t next = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < samples; ++i) {
    uint64_t rt;
    do {
      __builtin_amdgcn_s_sleep(2);
      rt = __builtin_amdgcn_s_memrealtime();
    } while (rt < next);
    const uint64_t ct = __builtin_amdgcn_s_memtime();
    out[2 * i] = ct;
    out[2 * i + 1] = rt;
    next = rt + interval;
  }
}

void launch_clock_probe(uint64_t* out, int samples, uint64_t interval_ticks, hipStream_t stream) {
  if (samples <= 0) return;
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, stream, out, samples, interval_ticks);
  hip_check(hipGetLastError(), "clock_probe launch");
}

// Plain device copy, 16 B per lane (used for the 1-rank allreduce: a kernel keeps the copy
// in stream order with the kernels around it, with no DMA-engine hand-off).
// Variants (A/B study, tools/bench_copy.py): UNROLL packs in flight per lane, NT = nontemporal
// loads/stores (streaming data that is not re-read soon should not displace cached lines).
template <int UNROLL, bool NT>
__global__ __launch_bounds__(kThreads) void copy16_kernel(const char* __restrict__ in, char* __restrict__ out,
                                                           int64_t bytes) {
  const int64_t npk = bytes / 16;
  const int64_t step = static_cast<int64_t>(gridDim.x) * kThreads;
  const Pack16* src = reinterpret_cast<const Pack16*>(in);
  Pack16* dst = reinterpret_cast<Pack16*>(out);
  int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  for (; i + (UNROLL - 1) * step < npk; i += UNROLL * step) {
    Pack16 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * step) : src[i + u * step];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (NT)
        __builtin_nontemporal_store(v[u], dst + i + u * step);
      else
        dst[i + u * step] = v[u];
    }
  }
  for (; i < npk; i += step) dst[i] = src[i];
  const int64_t t = npk * 16 + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (t < bytes) out[t] = in[t];
}

// Blocked variant: workgroup-contiguous tiles of UNROLL x 4 KiB (one 1 KiB wave access per
// pack, all packs of a tile in one contiguous region), tiles dealt grid-stride.
template <int UNROLL, bool NT>
__global__ __launch_bounds__(kThreads) void copy_tiles_kernel(const char* __restrict__ in, char* __restrict__ out,
                                                               int64_t bytes) {
  constexpr int64_t kTile = static_cast<int64_t>(UNROLL) * kThreads;  // packs per tile
  const int64_t npk = bytes / 16;
  const int64_t ntiles = npk / kTile;
  const Pack16* src = reinterpret_cast<const Pack16*>(in);
  Pack16* dst = reinterpret_cast<Pack16*>(out);
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t base = t * kTile + threadIdx.x;
    Pack16 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = NT ? __builtin_nontemporal_load(src + base + u * kThreads) : src[base + u * kThreads];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (NT)
        __builtin_nontemporal_store(v[u], dst + base + u * kThreads);
      else
        dst[base + u * kThreads] = v[u];
    }
  }
  for (int64_t i = ntiles * kTile + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < npk;
       i += static_cast<int64_t>(gridDim.x) * kThreads)
    dst[i] = src[i];
  const int64_t t = npk * 16 + static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (t < bytes) out[t] = in[t];
}

// Unit variant (round 3 store probe, profiles/round3/store_probe.json): every workgroup copies contiguous units of
// 512 KiB with nt buffer loads (aux 2: the input stream is read once) and sc0 sc1
// write-through buffer stores (aux 17) - 6.77 TB/s in the store probe against 5.2-5.6 for the
// plain / nt-store flavours. U packs of 16 B per lane in flight.
template <int U>
__global__ __launch_bounds__(kThreads) void copy_units_kernel(const char* __restrict__ in, char* __restrict__ out,
                                                               int64_t bytes, int64_t unit) {
  const int64_t nunits = (bytes + unit - 1) / unit;
  for (int64_t u = blockIdx.x; u < nunits; u += gridDim.x) {
    const char* s = in + u * unit;
    char* d = out + u * unit;
    const int64_t len = std::min<int64_t>(unit, bytes - u * unit);
    const int64_t npk = len / 16;
    const __amdgpu_buffer_rsrc_t rs = slab_rsrc(s), rd = slab_rsrc(d);
    int64_t i = threadIdx.x;
    for (; i + (U - 1) * kThreads < npk; i += U * kThreads) {
      Pack16 v[U];
#pragma unroll
      for (int q = 0; q < U; ++q)
        v[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>((i + q * kThreads) * 16), 0, 2);
#pragma unroll
      for (int q = 0; q < U; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(v[q], rd, static_cast<int>((i + q * kThreads) * 16), 0, 17);
    }
    for (; i < npk; i += kThreads) reinterpret_cast<Pack16*>(d)[i] = reinterpret_cast<const Pack16*>(s)[i];
    for (int64_t t = npk * 16 + threadIdx.x; t < len; t += kThreads) d[t] = s[t];
  }
}

static int g_copy_variant = -1;  // -1: default (see launch_copy)

void set_copy_variant(int v) { g_copy_variant = v; }

void launch_copy(const void* src, void* dst, int64_t bytes, hipStream_t stream) {
  if (bytes <= 0) return;
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15)
    throw std::invalid_argument("copy: buffers must be 16-byte aligned");
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  const int v = g_copy_variant < 0 ? 5 : g_copy_variant;  // 5: measured fastest (profiles/copy_variants.md)
  // grid: ~4 packs per thread for the unrolled variants, capped at 8 WG/CU
  const int unroll = (v == 0) ? 2 : 4;
  const int g = grid_for(std::max<int64_t>(bytes / 16 / unroll, 1));
  const int64_t tiles4 = std::max<int64_t>(1, bytes / (16LL * 4 * kThreads));
  const int64_t tiles8 = std::max<int64_t>(1, bytes / (16LL * 8 * kThreads));
  switch (v) {
    case 0: hipLaunchKernelGGL((copy16_kernel<2, false>), dim3(g), dim3(kThreads), 0, stream, s, d, bytes); break;
    case 1: hipLaunchKernelGGL((copy16_kernel<4, false>), dim3(g), dim3(kThreads), 0, stream, s, d, bytes); break;
    case 2: hipLaunchKernelGGL((copy16_kernel<4, true>), dim3(g), dim3(kThreads), 0, stream, s, d, bytes); break;
    case 3: hipLaunchKernelGGL((copy16_kernel<8, true>), dim3(g), dim3(kThreads), 0, stream, s, d, bytes); break;
    case 4: hipLaunchKernelGGL((copy_tiles_kernel<4, false>), dim3(std::min<int64_t>(tiles4, 2048)), dim3(kThreads), 0,
                               stream, s, d, bytes); break;
    case 5: hipLaunchKernelGGL((copy_tiles_kernel<4, true>), dim3(std::min<int64_t>(tiles4, 2048)), dim3(kThreads), 0,
                               stream, s, d, bytes); break;
    case 6: hipLaunchKernelGGL((copy_tiles_kernel<8, false>), dim3(std::min<int64_t>(tiles8, 1024)), dim3(kThreads), 0,
                               stream, s, d, bytes); break;
    case 7: {
      const int64_t unit = int64_t{512} << 10;
      const int64_t units = (bytes + unit - 1) / unit;
      hipLaunchKernelGGL((copy_units_kernel<8>), dim3(std::min<int64_t>(units, 512)), dim3(kThreads), 0, stream, s, d,
                         bytes, unit);
      break;
    }
    default: hipLaunchKernelGGL((copy_tiles_kernel<4, false>), dim3(tiles4), dim3(kThreads), 0, stream, s, d, bytes);
      break;
  }
  hip_check(hipGetLastError(), "copy launch");
}

template <class Ei, class Eo>
__global__ __launch_bounds__(kThreads) void cast_kernel(const char* in, char* out, int64_t n) {
  const int64_t step = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n; i += step)
    Scalar<Eo>::store(out, i, Scalar<Ei>::load(in, i));
}

void launch_cast(const void* src, DType dt_in, void* dst, DType dt_out, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  const int g = grid_for(n);
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  dispatch_dtype(static_cast<int>(dt_in), [&](auto ti) {
    dispatch_dtype(static_cast<int>(dt_out), [&](auto to) {
      hipLaunchKernelGGL((cast_kernel<decltype(ti), decltype(to)>), dim3(g), dim3(kThreads), 0, stream, s, d, n);
    });
  });
  hip_check(hipGetLastError(), "cast launch");
}

// table: count x {tensor ptr, numel, bucket offset (elements)} as 3 u64 each.
// One workgroup row per tensor slice: blockIdx.y = tensor, blockIdx.x strides its elements.
template <class E>
__global__ __launch_bounds__(kThreads) void bucket_copy_kernel(const uint64_t* table, char* bucket, int pack) {
  constexpr int es = 16 / E::ELEMS;
  const uint64_t* t = table + 3 * blockIdx.y;
  char* tp = reinterpret_cast<char*>(t[0]);
  const int64_t numel = static_cast<int64_t>(t[1]);
  char* bp = bucket + static_cast<int64_t>(t[2]) * es;
  const bool aligned = ((reinterpret_cast<uintptr_t>(tp) | reinterpret_cast<uintptr_t>(bp)) & 15) == 0;
  const int64_t step = static_cast<int64_t>(gridDim.x) * kThreads;
  const int64_t first = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  char* dst = pack ? bp : tp;
  const char* src = pack ? tp : bp;
  int64_t done = 0;
  if (aligned) {
    const int64_t npk = numel / E::ELEMS;
    for (int64_t i = first; i < npk; i += step) st16(dst + i * 16, ld16(src + i * 16));
    done = npk * E::ELEMS;
  }
  for (int64_t i = done + first; i < numel; i += step) Scalar<E>::copy(dst, src, i);
}

void launch_bucket_copy(const uint64_t* dev_table, int count, void* bucket, DType dt, bool pack, int64_t total,
                        hipStream_t stream) {
  if (count <= 0) return;
  const int64_t avg_packs = std::max<int64_t>(1, total * static_cast<int64_t>(dtype_size(dt)) / 16 / count);
  const int gx = static_cast<int>(std::min<int64_t>(64, (avg_packs + kThreads - 1) / kThreads));
  dim3 g(std::max(gx, 1), count);
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    hipLaunchKernelGGL(bucket_copy_kernel<decltype(tag)>, g, dim3(kThreads), 0, stream, dev_table,
                       static_cast<char*>(bucket), pack ? 1 : 0);
  });
  hip_check(hipGetLastError(), "bucket_copy launch");
}

// ---------------------------------------------------------------------------------
// Hardware-queue independence probe. HIP deals a process's streams onto a few hardware
// queues (GPU_MAX_HW_QUEUES, 4 on the boxes); two streams on one queue run their kernels in
// order. A persistent round kernel that spins waiting for a co-located peer's kernel must
// not share a queue with it. The probe: a spinning kernel on `a` waits (bounded) for a flag
// a kernel on `b` sets - it only returns "seen" when b's kernel could run while a's spun.
// ---------------------------------------------------------------------------------
__global__ void queue_probe_spin(int* flag, int* seen, uint64_t ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + ticks;
  int v = 0;
  while ((v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) == 0 &&
         __builtin_amdgcn_s_memrealtime() < deadline)
    __builtin_amdgcn_s_sleep(4);
  __hip_atomic_store(seen, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void queue_probe_set(int* flag) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

bool streams_independent(hipStream_t a, hipStream_t b, double timeout_ms) {
  // one probe word pair per device, allocated once: hipFree would synchronise the device,
  // i.e. wait for every kernel on it (another plane's round, a resident kernel)
  static std::mutex mu;
  static std::map<int, int*> words;
  int dev = 0;
  hip_check(hipGetDevice(&dev), "hipGetDevice(queue probe)");
  std::lock_guard<std::mutex> g(mu);
  int*& mem = words[dev];
  if (mem == nullptr) hip_check(hipMalloc(reinterpret_cast<void**>(&mem), 128), "hipMalloc(queue probe)");
  hip_check(hipMemsetAsync(mem, 0, 128, a), "hipMemsetAsync(queue probe)");
  hip_check(hipStreamSynchronize(a), "hipStreamSynchronize(queue probe)");
  hipLaunchKernelGGL(queue_probe_spin, dim3(1), dim3(64), 0, a, mem, mem + 16,
                     static_cast<uint64_t>(timeout_ms * 1e5));  // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(queue_probe_set, dim3(1), dim3(64), 0, b, mem);
  hip_check(hipStreamSynchronize(a), "hipStreamSynchronize(queue probe)");
  hip_check(hipStreamSynchronize(b), "hipStreamSynchronize(queue probe)");
  int seen = 0;
  hip_check(hipMemcpyAsync(&seen, mem + 16, 4, hipMemcpyDeviceToHost, a), "hipMemcpyAsync(queue probe)");
  hip_check(hipStreamSynchronize(a), "hipStreamSynchronize(queue probe)");
  return seen != 0;
}

}  // namespace mxar
