// Device-side helpers shared by the gfx950 kernels of the data plane.
//
//   * 16-byte vector packs (one `global_load/store_dwordx4` per lane): every kernel in
//     csrc/hip moves data 16 B per lane (cdna_hip_programming.md Guideline 13); bf16 is
//     never loaded as scalars.
//   * fp32 accumulation of bf16/fp32 packs (bf16 -> fp32 is a 16-bit shift; fp32 -> bf16
//     goes through the hardware `v_cvt_pk_bf16_f32` round-to-nearest-even, NaN-safe).
//   * Cross-GPU signalling over xGMI, as shipped: flags AND payload slots live in
//     fine-grained device memory (hipDeviceMallocFinegrained, the default of XgmiComm;
//     `MXAR_SLAB_MEM=uncached|coarse` exist for study only - uncached slabs showed stale
//     reads, profiles/memory_ordering_study.md) that peers map through IPC, and the
//     communicator runs with release AND acquire on (`fence = 3`).
//     Producer: write-through payload stores (`sc0 sc1`) -> every storing wave drains its
//     `vmcnt` -> workgroup barrier -> ONE lane: system-scope release fence -> asm drain ->
//     relaxed system-scope flag store. The release is required: a drained write-through
//     store is only known to have reached the producer's L2 channel, and without the
//     fence the flag was seen to arrive first (stale slab reads). Because every kernel
//     store is write-through, the release's L2 writeback finds (almost) nothing dirty.
//     Consumer: ONE wave polls relaxed (with `s_sleep`), then ONE system-scope acquire
//     (invalidates this CU's L1 and the non-coherent L2 lines), then a workgroup barrier
//     before any payload load; payload loads additionally use `sc1` (L1 bypass)
//     (MI355X_MICROARCH.md "Valid forms"; the asm drain after the fence is the ROCm 7.2
//     compiler-hazard fix from the same section).
//   * Every spin is bounded by a wall-clock deadline (`s_memrealtime`, 100 MHz): a wedged
//     peer turns into an error word the host reads, never into a hung GPU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mxar {
namespace dev {

// 16-byte pack as a native 4 x u32 vector (a struct-of-array pack gets promoted to LDS
// by the alloca promotion pass when several packs are in flight per lane).
typedef unsigned int Pack16 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------
// dtype traits: E = element type tag, ELEMS = elements per 16-B pack
// ---------------------------------------------------------------------------------
struct F32 {
  static constexpr int ELEMS = 4;
  typedef float scalar;
};
struct BF16 {
  static constexpr int ELEMS = 8;
  typedef uint16_t scalar;
};
struct F16 {
  static constexpr int ELEMS = 8;
  typedef uint16_t scalar;
};

// Host-side dtype dispatch: f(F32{}) / f(BF16{}) / f(F16{}) for DType codes 0 / 1 / 2.
template <class Fn>
inline void dispatch_dtype(int code, Fn&& f) {
  if (code == 0)
    f(F32{});
  else if (code == 1)
    f(BF16{});
  else
    f(F16{});
}

__device__ __forceinline__ float bf16_to_f32(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  // v_cvt_pk_bf16_f32: RNE, NaN stays NaN (MI355X_MICROARCH.md numerics table)
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 v = {lo, hi};
  bf2 r = __builtin_convertvector(v, bf2);
  return __builtin_bit_cast(uint32_t, r);
}

__device__ __forceinline__ float f16_to_f32(uint32_t bits16) {
  return static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(bits16)));
}

__device__ __forceinline__ uint32_t pack_f16x2(float lo, float hi) {
  // v_cvt_pk_f16_f32 family: RNE, overflow -> inf (IEEE half)
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 v = {lo, hi};
  h2 r = __builtin_convertvector(v, h2);
  return __builtin_bit_cast(uint32_t, r);
}

template <typename E>
struct Acc;

template <>
struct Acc<F32> {
  float v[4];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = 0.f;
  }
  __device__ __forceinline__ void add(const Pack16& p) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] += __uint_as_float(p[i]);
  }
  __device__ __forceinline__ void scale(float s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= s;
  }
  __device__ __forceinline__ Pack16 pack() const {
    Pack16 p;
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = __float_as_uint(v[i]);
    return p;
  }
};

template <>
struct Acc<BF16> {
  float v[8];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
  }
  __device__ __forceinline__ void add(const Pack16& p) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] += bf16_to_f32(p[i] & 0xFFFFu);
      v[2 * i + 1] += bf16_to_f32(p[i] >> 16);
    }
  }
  __device__ __forceinline__ void scale(float s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] *= s;
  }
  __device__ __forceinline__ Pack16 pack() const {
    Pack16 p;
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = pack_bf16x2(v[2 * i], v[2 * i + 1]);
    return p;
  }
};

template <>
struct Acc<F16> {
  float v[8];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
  }
  __device__ __forceinline__ void add(const Pack16& p) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] += f16_to_f32(p[i] & 0xFFFFu);
      v[2 * i + 1] += f16_to_f32(p[i] >> 16);
    }
  }
  __device__ __forceinline__ void scale(float s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] *= s;
  }
  __device__ __forceinline__ Pack16 pack() const {
    Pack16 p;
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = pack_f16x2(v[2 * i], v[2 * i + 1]);
    return p;
  }
};

// fp32 accumulation of one 8-byte unit (low-latency kernels: xgmi_ll.hip, threshold LL rounds) (2 fp32 or 4 bf16/fp16 elements)
template <class E>
struct Acc8;
template <>
struct Acc8<F32> {
  float v[2] = {0.f, 0.f};
  __device__ __forceinline__ void add(uint2 d) {
    v[0] += __uint_as_float(d.x);
    v[1] += __uint_as_float(d.y);
  }
  __device__ __forceinline__ uint2 pack(float s) const { return make_uint2(__float_as_uint(v[0] * s), __float_as_uint(v[1] * s)); }
};
template <>
struct Acc8<BF16> {
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  __device__ __forceinline__ void add(uint2 d) {
    v[0] += bf16_to_f32(d.x & 0xFFFFu);
    v[1] += bf16_to_f32(d.x >> 16);
    v[2] += bf16_to_f32(d.y & 0xFFFFu);
    v[3] += bf16_to_f32(d.y >> 16);
  }
  __device__ __forceinline__ uint2 pack(float s) const {
    return make_uint2(pack_bf16x2(v[0] * s, v[1] * s), pack_bf16x2(v[2] * s, v[3] * s));
  }
};
template <>
struct Acc8<F16> {
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  __device__ __forceinline__ void add(uint2 d) {
    v[0] += f16_to_f32(d.x & 0xFFFFu);
    v[1] += f16_to_f32(d.x >> 16);
    v[2] += f16_to_f32(d.y & 0xFFFFu);
    v[3] += f16_to_f32(d.y >> 16);
  }
  __device__ __forceinline__ uint2 pack(float s) const {
    return make_uint2(pack_f16x2(v[0] * s, v[1] * s), pack_f16x2(v[2] * s, v[3] * s));
  }
};


// Scalar element access for ragged tails (< one pack).
template <typename E>
struct Scalar;
template <>
struct Scalar<F32> {
  __device__ __forceinline__ static float load(const void* p, int64_t i) { return static_cast<const float*>(p)[i]; }
  __device__ __forceinline__ static void store(void* p, int64_t i, float x) { static_cast<float*>(p)[i] = x; }
  __device__ __forceinline__ static void copy(void* d, const void* s, int64_t i) {
    static_cast<float*>(d)[i] = static_cast<const float*>(s)[i];
  }
};
template <>
struct Scalar<BF16> {
  __device__ __forceinline__ static float load(const void* p, int64_t i) {
    return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
  }
  __device__ __forceinline__ static void store(void* p, int64_t i, float x) {
    static_cast<uint16_t*>(p)[i] = static_cast<uint16_t>(pack_bf16x2(x, 0.f) & 0xFFFFu);
  }
  __device__ __forceinline__ static void copy(void* d, const void* s, int64_t i) {
    static_cast<uint16_t*>(d)[i] = static_cast<const uint16_t*>(s)[i];
  }
};

template <>
struct Scalar<F16> {
  __device__ __forceinline__ static float load(const void* p, int64_t i) {
    return f16_to_f32(static_cast<const uint16_t*>(p)[i]);
  }
  __device__ __forceinline__ static void store(void* p, int64_t i, float x) {
    static_cast<uint16_t*>(p)[i] = static_cast<uint16_t>(pack_f16x2(x, 0.f) & 0xFFFFu);
  }
  __device__ __forceinline__ static void copy(void* d, const void* s, int64_t i) {
    static_cast<uint16_t*>(d)[i] = static_cast<const uint16_t*>(s)[i];
  }
};

__device__ __forceinline__ Pack16 ld16(const void* p) { return *static_cast<const Pack16*>(p); }
__device__ __forceinline__ void st16(void* p, const Pack16& v) { *static_cast<Pack16*>(p) = v; }

// ---------------------------------------------------------------------------------
// Data-plane reads: `buffer_load ... nt` (non-temporal). Like `sc1` it bypasses the reading
// CU's L1 (MI355X_MICROARCH.md, load flavours), so after the consumer's acquire it reads
// what the peers' write-through stores left in memory - the acquire (wait_flags, fence bit
// 1, on by default) is what makes the peers' xGMI stores visible, not the load flavour. As a
// streaming hint it also keeps one-pass streams from displacing each other in L2: a copy of
// 256 MiB with nt loads + write-through stores runs 6.77 TB/s vs 5.18 with sc1 or plain loads
// (a one-off store probe, removed in round 4 - git history - profiles/round3/store_probe.json), into fine-grained and coarse
// memory alike. Every slab read AND every read of a kernel's own input stream uses it.
// Descriptor built from wave-uniform values only (cdna_hip_programming.md T8/T20).
// ---------------------------------------------------------------------------------
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
constexpr int kAuxNt = 2;  // CPol NT (slc)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), static_cast<short>(0), 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ Pack16 ld16_nt(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(off), 0, kAuxNt);
}
// Slab writes: `buffer_store ... sc0 sc1` = system-coherent write-through. A drained
// (`s_waitcnt vmcnt(0)`) write-through store has reached memory, so the flag that follows
// needs no `buffer_wbl2` release (which would also write back every unrelated dirty L2
// line, e.g. the output) - the guide's R1 hand-off, at system scope for xGMI peers.
constexpr int kAuxWt = 17;  // sc0 | sc1
__device__ __forceinline__ void st16_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, const Pack16& v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, static_cast<int>(off), 0, kAuxWt);
}
template <class E>
__device__ __forceinline__ void st_scalar_wt(__amdgpu_buffer_rsrc_t r, int64_t i, float x);
template <>
__device__ __forceinline__ void st_scalar_wt<F32>(__amdgpu_buffer_rsrc_t r, int64_t i, float x) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, static_cast<int>(i * 4), 0, kAuxWt);
}
template <>
__device__ __forceinline__ void st_scalar_wt<BF16>(__amdgpu_buffer_rsrc_t r, int64_t i, float x) {
  __builtin_amdgcn_raw_buffer_store_b16(static_cast<unsigned short>(pack_bf16x2(x, 0.f) & 0xFFFFu), r,
                                        static_cast<int>(i * 2), 0, kAuxWt);
}
template <>
__device__ __forceinline__ void st_scalar_wt<F16>(__amdgpu_buffer_rsrc_t r, int64_t i, float x) {
  __builtin_amdgcn_raw_buffer_store_b16(static_cast<unsigned short>(pack_f16x2(x, 0.f) & 0xFFFFu), r,
                                        static_cast<int>(i * 2), 0, kAuxWt);
}
template <class E>
__device__ __forceinline__ void copy_scalar_wt(__amdgpu_buffer_rsrc_t r, const void* src, int64_t i);
template <>
__device__ __forceinline__ void copy_scalar_wt<F32>(__amdgpu_buffer_rsrc_t r, const void* src, int64_t i) {
  __builtin_amdgcn_raw_buffer_store_b32(static_cast<const uint32_t*>(src)[i], r, static_cast<int>(i * 4), 0, kAuxWt);
}
template <>
__device__ __forceinline__ void copy_scalar_wt<BF16>(__amdgpu_buffer_rsrc_t r, const void* src, int64_t i) {
  __builtin_amdgcn_raw_buffer_store_b16(static_cast<const uint16_t*>(src)[i], r, static_cast<int>(i * 2), 0, kAuxWt);
}

template <>
__device__ __forceinline__ void copy_scalar_wt<F16>(__amdgpu_buffer_rsrc_t r, const void* src, int64_t i) {
  __builtin_amdgcn_raw_buffer_store_b16(static_cast<const uint16_t*>(src)[i], r, static_cast<int>(i * 2), 0, kAuxWt);
}

template <class E>
__device__ __forceinline__ float ld_scalar_nt(__amdgpu_buffer_rsrc_t r, int64_t i);
template <>
__device__ __forceinline__ float ld_scalar_nt<F32>(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(i * 4), 0, kAuxNt));
}
template <>
__device__ __forceinline__ float ld_scalar_nt<BF16>(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return bf16_to_f32(__builtin_amdgcn_raw_buffer_load_b16(r, static_cast<int>(i * 2), 0, kAuxNt));
}
template <>
__device__ __forceinline__ float ld_scalar_nt<F16>(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return f16_to_f32(__builtin_amdgcn_raw_buffer_load_b16(r, static_cast<int>(i * 2), 0, kAuxNt));
}

// ---------------------------------------------------------------------------------
// Clock + bounded spin
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wall_ticks() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// Error codes written to the host-visible error word (bitwise OR).
enum : uint32_t {
  ERR_TIMEOUT_SCATTER = 1u,
  ERR_TIMEOUT_REDUCE = 2u,
  ERR_TIMEOUT_BARRIER = 4u,
  ERR_BAD_ARGS = 8u,
  ERR_TIMEOUT_LAG = 16u,  // threshold kernel: a peer stayed more than maxLag rounds behind
};

__device__ __forceinline__ uint32_t ld_flag(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_flag(uint32_t* f, uint32_t v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool reached(uint32_t flag, uint32_t epoch) {
  return static_cast<int32_t>(flag - epoch) >= 0;  // wrap-safe epoch compare
}

// Producer side: called by ALL threads of the workgroup after their payload stores.
// Lane i < nflags of wave 0 stores flag `addr(i)` (skipped when it returns nullptr).
// `release` = false drops the system-scope release fence (measurement knob only, fence
// bit 0 cleared: the payload then relies on the vmcnt drain alone, which is NOT enough on
// fine-grained memory - see the header comment).
// Lanes with no flag (nullptr: the own rank, or a 1-rank launch) skip the fence: its
// `buffer_wbl2` would write back every dirty L2 line of the kernel (e.g. half-updated
// AdamW state lines of other workgroups, which are then written again) and order nothing.
template <typename FlagAddr>
__device__ __forceinline__ void publish_flags(FlagAddr addr, int nflags, uint32_t epoch, bool release = true) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x < static_cast<unsigned>(nflags)) {
    uint32_t* f = addr(static_cast<int>(threadIdx.x));
    if (f) {
      if (release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope (xGMI peers)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_flag(f, epoch);
    }
  }
}

// Consumer side: called by ALL threads. Lane i < nflags of wave 0 polls flag `addr(i)`
// (nullptr = nothing to wait for) until every flag has reached `epoch` or the deadline
// passes. Returns false on timeout (uniform across the workgroup) after OR-ing `code`
// into the error word. On success the payload may be read with plain loads.
template <typename FlagAddr>
__device__ __forceinline__ bool wait_flags(FlagAddr addr, int nflags, uint32_t epoch, uint64_t deadline,
                                           uint32_t* err, uint32_t code, bool acquire = true) {
  __shared__ int ok_s;
  if (threadIdx.x < 64) {
    const uint32_t* f = threadIdx.x < static_cast<unsigned>(nflags) ? addr(static_cast<int>(threadIdx.x)) : nullptr;
    // nothing to wait for (a 1-rank launch, the own contribution only): no acquire either -
    // its L2 invalidate would order nothing (and can write back other workgroups' dirty lines)
    if (!__any(f != nullptr)) acquire = false;
    bool ok = (f == nullptr) || reached(ld_flag(f), epoch);
    while (!__all(ok)) {
      __builtin_amdgcn_s_sleep(1);
      if (!ok) ok = reached(ld_flag(f), epoch);
      if (wall_ticks() > deadline) break;
    }
    const bool all_ok = __all(ok);
    if (threadIdx.x == 0) {
      ok_s = all_ok ? 1 : 0;
      if (!all_ok) __hip_atomic_fetch_or(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return ok_s != 0;
}

}  // namespace dev
}  // namespace mxar
