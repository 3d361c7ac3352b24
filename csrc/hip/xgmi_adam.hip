// Fused sharded-data-parallel step over xGMI (gfx950): reduce-scatter of the gradients,
// AdamW on the owned shard and all-gather of the updated parameters in ONE launch.
//
// The reference hands every reduced vector to a user `dataSink` (AllreduceWorker.scala:
// 180-192); in training that sink is an optimizer. Here the sink runs inside the owner's
// reduce (the allreduce's phase 2): the moment chunk c of the own block has all P gradient
// contributions, the owner sums them (fp32, rank order, x scale), applies AdamW to its fp32
// master copy and moments of that chunk, rounds the new parameters once to the parameter
// dtype and pushes THEM - not the gradient sum - to every peer. Phase 3 gathers the peers'
// updated parameter chunks. Compared with reduce-scatter + optimizer + all-gather this saves
// two launches, the round trip of the reduced gradient through HBM and the serialisation
// between the three steps; the wire bytes are those of one allreduce.
//
// Slot reuse across launches is the two-shot's: a rank finishes a launch only after it has
// received every owner's updated chunk, which each owner sends after reading its S slot for
// that chunk; peers' pending reads of R are covered by entry_guard / finish_launch_done.
#include "../core/env.h"
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "xgmi_device.h"

namespace mxar {

namespace {

// AdamW (decoupled weight decay, PyTorch semantics) of one element; returns the new param.
__device__ __forceinline__ float adamw(float g, float* p, float* m, float* v, const CommArgs& a) {
  float pv = *p;
  pv *= 1.f - a.lr * a.wd;
  const float mv = a.beta1 * *m + (1.f - a.beta1) * g;
  const float vv = a.beta2 * *v + (1.f - a.beta2) * g * g;
  const float denom = sqrtf(vv) / a.c2_sqrt + a.eps;
  pv -= (a.lr / a.c1) * mv / denom;
  *p = pv;
  *m = mv;
  *v = vv;
  return pv;
}

}  // namespace

// fp32 state access: plain loads / stores (STREAM = false, the default) or nt loads +
// write-through stores (STREAM = true, MXAR_ADAM_STREAM=1: the store probe's fastest copy
// form, profiles/round3/store_probe.json). The state is read and written back at the same
// addresses, and the streaming form is 1.56x slower (1.00 vs 0.64 ms for the 134 M-parameter
// step, same box: profiles/round3/adamw_stream_ab.jsonl); the gradients (read once, summed)
// come in with nt loads either way.
// MODE 0 (default): plain state loads and stores. MODE 1 (MXAR_ADAM_STREAM=1): nt loads +
// write-through stores (the store probe's fastest copy form, profiles/round3/store_probe.json)
// - the state is read and written back at the same addresses, and that form was 1.56x slower
// (1.00 vs 0.64 ms for the 134 M-parameter step, same box: profiles/round3/README.md).
// MODE 2 (MXAR_ADAM_STREAM=2): nt loads, plain stores. The gradients (read once, summed) come
// in with nt loads in every mode.
template <int MODE>
__device__ __forceinline__ float4 ld_state(const float* p, __amdgpu_buffer_rsrc_t r, int64_t i) {
  if constexpr (MODE != 0) {
    const Pack16 v = ld16_nt(r, static_cast<uint32_t>(i * 4));
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
  } else {
    return *reinterpret_cast<const float4*>(p + i);
  }
}
template <int MODE>
__device__ __forceinline__ void st_state(float* p, __amdgpu_buffer_rsrc_t r, int64_t i, const float4& x) {
  if constexpr (MODE == 1) {
    Pack16 v;
    v[0] = __float_as_uint(x.x);
    v[1] = __float_as_uint(x.y);
    v[2] = __float_as_uint(x.z);
    v[3] = __float_as_uint(x.w);
    st16_wt(r, static_cast<uint32_t>(i * 4), v);
  } else {
    *reinterpret_cast<float4*>(p + i) = x;
  }
}

template <class E, int PT, int STREAM, int U>
__global__ __launch_bounds__(kCommThreads) void twoshot_adamw_kernel(CommArgs a) {
  constexpr int es = 16 / E::ELEMS;
  constexpr int EL = E::ELEMS;
  const int P = PT > 0 ? PT : a.P;
  const int y = blockIdx.y;
  const int r = a.rank0 + y;
  const char* const grad = a.in[y];
  char* const param = a.out[y];
  float* const mp = a.opt_p[y];
  float* const m1 = a.opt_m[y];
  float* const m2 = a.opt_v[y];
  uint32_t* const ctl = a.ctl[y];
  const uint32_t epoch = launch_epoch(ctl);
  const uint64_t deadline = wall_ticks() + a.timeout;
  const int G = gridDim.x;
  const int64_t slot = a.slot_bytes;
  uint32_t* err = &ctl[2];
  const bool rel = a.fence & 1, acq = a.fence & 2;
  const int Pm1 = P > 1 ? P - 1 : 1;
  const int nu = (P - 1) * a.nch;

  // Phase 1 - gradient ScatterBlock: chunk c of block j to its owner j
  if (static_cast<int>(blockIdx.x) < nu) entry_guard(a, ctl, r, epoch, kHazS, -1, deadline, err);
  for (int u = blockIdx.x; u < nu; u += G) {
    const int c = u / Pm1;
    const int j = (r + 1 + u % Pm1) % P;
    const int64_t bstart = static_cast<int64_t>(j) * a.block;
    const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
    const int64_t len = clamp_len(clamp_len(a.n - bstart, a.block) - cstart, a.chunk);
    if (len > 0 && unit_in_bounds(a, cstart * es, len * es, c, err))
      copy_to_slab<E>(a.base[j] + a.off_S + r * slot + cstart * es, grad + (bstart + cstart) * es, len);
    publish_flags([&](int) { return f1(a, j, r, c); }, 1, epoch, rel);
  }

  // Phase 2 - reduce own chunk, AdamW on the owned shard, push the new parameters
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
    wait_flags([&](int s) -> const uint32_t* { return s == r ? nullptr : f1(a, r, s, c); }, P, epoch, deadline, err,
               ERR_TIMEOUT_SCATTER, acq);
    if (len > 0 && unit_in_bounds(a, cstart * es, len * es, u, err)) {
      const RedSrc src{grad + (bstart_own + cstart) * es, a.base[r] + a.off_S + cstart * es, slot, r};
      char* own_out = param + (bstart_own + cstart) * es;
      const int64_t roff = a.off_R + r * slot + cstart * es;
      float* const sp = mp + cstart;
      float* const sm = m1 + cstart;
      float* const sv = m2 + cstart;
      const __amdgpu_buffer_rsrc_t rp = slab_rsrc(sp), rm = slab_rsrc(sm), rv = slab_rsrc(sv);
      const int64_t npk = len / EL;
      if constexpr (STREAM == 3 && EL == 8) {
        // Run-contiguous halves (16-bit parameters, the default): lane l of a run of 256 packs
        // takes elements [4l, 4l + 4) of each half of the run's 2048 elements, so every fp32
        // state load / store instruction of a wave covers 1 KiB of consecutive bytes and every
        // 16-bit one 512 B. (One 16-B parameter pack per lane made each fp32 state access hit
        // every other 16 B of 2 KiB: half-written lines, 15.3 B written per parameter instead
        // of 14 - profiles/round4/README.md section 5.) The last, short run is split the same
        // way with `rows` lanes per half. Scatter and gather stay plain contiguous copies.
        auto eoff = [&](int64_t i, int h) -> int64_t {
          const int64_t run = i / kCommThreads;
          const int64_t l = i - run * kCommThreads;
          const int64_t left = npk - run * kCommThreads;
          const int64_t rows = left < kCommThreads ? left : kCommThreads;
          return run * kCommThreads * EL + h * rows * 4 + l * 4;
        };
        for (int64_t i0 = threadIdx.x; i0 < npk; i0 += U * kCommThreads) {
          Acc8<E> acc[U][2];
          float4 p4[U][2], m4[U][2], v4[U][2];
          bool live[U];
#pragma unroll
          for (int w = 0; w < U; ++w) {
            const int64_t i = i0 + w * kCommThreads;
            live[w] = i < npk;
            if (!live[w]) continue;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int64_t e0 = eoff(i, h);
              if constexpr (PT > 0) {
                uint2 g[PT];
#pragma unroll
                for (int s = 0; s < PT; ++s) {
                  const auto v = __builtin_amdgcn_raw_buffer_load_b64(src.rsrc(s), static_cast<int>(e0 * 2), 0, kAuxNt);
                  g[s] = make_uint2(v[0], v[1]);
                }
#pragma unroll
                for (int s = 0; s < PT; ++s) acc[w][h].add(g[s]);
              } else {
                for (int s = 0; s < P; ++s) {
                  const auto v = __builtin_amdgcn_raw_buffer_load_b64(src.rsrc(s), static_cast<int>(e0 * 2), 0, kAuxNt);
                  acc[w][h].add(make_uint2(v[0], v[1]));
                }
              }
              p4[w][h] = *reinterpret_cast<const float4*>(sp + e0);
              m4[w][h] = *reinterpret_cast<const float4*>(sm + e0);
              v4[w][h] = *reinterpret_cast<const float4*>(sv + e0);
            }
          }
#pragma unroll
          for (int w = 0; w < U; ++w) {
            if (!live[w]) continue;
            const int64_t i = i0 + w * kCommThreads;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int64_t e0 = eoff(i, h);
              Acc8<E>& ac = acc[w][h];
              ac.v[0] = adamw(ac.v[0] * a.scale, &p4[w][h].x, &m4[w][h].x, &v4[w][h].x, a);
              ac.v[1] = adamw(ac.v[1] * a.scale, &p4[w][h].y, &m4[w][h].y, &v4[w][h].y, a);
              ac.v[2] = adamw(ac.v[2] * a.scale, &p4[w][h].z, &m4[w][h].z, &v4[w][h].z, a);
              ac.v[3] = adamw(ac.v[3] * a.scale, &p4[w][h].w, &m4[w][h].w, &v4[w][h].w, a);
              *reinterpret_cast<float4*>(sp + e0) = p4[w][h];
              *reinterpret_cast<float4*>(sm + e0) = m4[w][h];
              *reinterpret_cast<float4*>(sv + e0) = v4[w][h];
              const uint2 o = ac.pack(1.f);
              *reinterpret_cast<uint2*>(own_out + e0 * 2) = o;
              typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
              const u32x2 ov = {o.x, o.y};
              for (int k = 0; k < P; ++k)
                if (k != r)
                  __builtin_amdgcn_raw_buffer_store_b64(ov, slab_rsrc(a.base[k] + roff), static_cast<int>(e0 * 2), 0,
                                                        kAuxWt);
            }
          }
        }
      } else
      // U packs per lane per iteration, every load issued before the first use: the
      // persistent grid has only 2 workgroups per CU, so bytes in flight come from ILP
      for (int64_t i0 = threadIdx.x; i0 < npk; i0 += U * kCommThreads) {
        Acc<E> acc[U];
        float4 p4[U][EL / 4], m4[U][EL / 4], v4[U][EL / 4];
        bool live[U];
#pragma unroll
        for (int w = 0; w < U; ++w) {
          const int64_t i = i0 + w * kCommThreads;
          live[w] = i < npk;
          acc[w].zero();
          if (!live[w]) continue;
          if constexpr (PT > 0) {
            Pack16 g[PT];
#pragma unroll
            for (int s = 0; s < PT; ++s) g[s] = ld16_nt(src.rsrc(s), static_cast<uint32_t>(i * 16));
#pragma unroll
            for (int s = 0; s < PT; ++s) acc[w].add(g[s]);
          } else {
            for (int s = 0; s < P; ++s) acc[w].add(ld16_nt(src.rsrc(s), static_cast<uint32_t>(i * 16)));
          }
#pragma unroll
          for (int e = 0; e < EL / 4; ++e) {
            p4[w][e] = ld_state<STREAM>(sp, rp, i * EL + 4 * e);
            m4[w][e] = ld_state<STREAM>(sm, rm, i * EL + 4 * e);
            v4[w][e] = ld_state<STREAM>(sv, rv, i * EL + 4 * e);
          }
        }
#pragma unroll
        for (int w = 0; w < U; ++w) {
          if (!live[w]) continue;
          const int64_t i = i0 + w * kCommThreads;
#pragma unroll
          for (int e = 0; e < EL / 4; ++e) {
            acc[w].v[4 * e + 0] = adamw(acc[w].v[4 * e + 0] * a.scale, &p4[w][e].x, &m4[w][e].x, &v4[w][e].x, a);
            acc[w].v[4 * e + 1] = adamw(acc[w].v[4 * e + 1] * a.scale, &p4[w][e].y, &m4[w][e].y, &v4[w][e].y, a);
            acc[w].v[4 * e + 2] = adamw(acc[w].v[4 * e + 2] * a.scale, &p4[w][e].z, &m4[w][e].z, &v4[w][e].z, a);
            acc[w].v[4 * e + 3] = adamw(acc[w].v[4 * e + 3] * a.scale, &p4[w][e].w, &m4[w][e].w, &v4[w][e].w, a);
            st_state<STREAM>(sp, rp, i * EL + 4 * e, p4[w][e]);
            st_state<STREAM>(sm, rm, i * EL + 4 * e, m4[w][e]);
            st_state<STREAM>(sv, rv, i * EL + 4 * e, v4[w][e]);
          }
          const Pack16 o = acc[w].pack();
          if constexpr (STREAM == 1)
            st16_wt(slab_rsrc(own_out), static_cast<uint32_t>(i * 16), o);
          else
            st16(own_out + i * 16, o);
          for (int k = 0; k < P; ++k)
            if (k != r) st16_wt(slab_rsrc(a.base[k] + roff), static_cast<uint32_t>(i * 16), o);
        }
      }
      const int64_t t = npk * EL + threadIdx.x;
      if (t < len) {
        float g = 0.f;
        for (int s = 0; s < P; ++s) g += ld_scalar_nt<E>(src.rsrc(s), t);
        const float pv = adamw(g * a.scale, sp + t, sm + t, sv + t, a);
        Scalar<E>::store(own_out, t, pv);
        for (int k = 0; k < P; ++k)
          if (k != r) st_scalar_wt<E>(slab_rsrc(a.base[k] + roff), t, pv);
      }
    }
    publish_flags([&](int k) -> uint32_t* { return k == r ? nullptr : f2(a, k, r, u); }, P, epoch, rel);
  }

  // Phase 3 - gather the other owners' updated parameter chunks
  for (int u = blockIdx.x; u < nu; u += G) {
    const int c = u / Pm1;
    const int j = (r + 1 + u % Pm1) % P;
    const int64_t bstart = static_cast<int64_t>(j) * a.block;
    const int64_t cstart = static_cast<int64_t>(c) * a.chunk;
    const int64_t len = clamp_len(clamp_len(a.n - bstart, a.block) - cstart, a.chunk);
    wait_flags([&](int q) -> const uint32_t* { return f2(a, r, j, c * a.sub + q); }, a.sub, epoch, deadline, err,
               ERR_TIMEOUT_REDUCE, acq);
    if (len > 0 && unit_in_bounds(a, cstart * es, len * es, c, err))
      copy_from_slab<E>(param + (bstart + cstart) * es, a.base[r] + a.off_R + j * slot + cstart * es, len);
  }
  finish_launch_done(a, ctl, epoch, r, kHazR);  // peers may still gather from R
}

template <int STREAM, int U>
static void launch_adamw_t(const CommArgs& a, dim3 grid, hipStream_t s, DType dt) {
  dispatch_dtype(static_cast<int>(dt), [&](auto tag) {
    using E = decltype(tag);
    // P is a template constant wherever it can be: the reduce then issues every source's
    // load before the first add (the PT = 0 loop waits on each load in turn) - P = 1 is the
    // single-GPU optimizer step
    switch (a.P) {
      case 1: hipLaunchKernelGGL((twoshot_adamw_kernel<E, 1, STREAM, U>), grid, dim3(kCommThreads), 0, s, a); break;
      case 2: hipLaunchKernelGGL((twoshot_adamw_kernel<E, 2, STREAM, U>), grid, dim3(kCommThreads), 0, s, a); break;
      case 4: hipLaunchKernelGGL((twoshot_adamw_kernel<E, 4, STREAM, U>), grid, dim3(kCommThreads), 0, s, a); break;
      case 8: hipLaunchKernelGGL((twoshot_adamw_kernel<E, 8, STREAM, U>), grid, dim3(kCommThreads), 0, s, a); break;
      default: hipLaunchKernelGGL((twoshot_adamw_kernel<E, 0, STREAM, U>), grid, dim3(kCommThreads), 0, s, a); break;
    }
  });
}

void launch_adamw(const CommArgs& a, dim3 grid, hipStream_t s, DType dt) {
  // study knob MXAR_ADAM_STREAM (state access form, above); two packs per lane in flight (1
  // and 4 measured no better - their knob was removed in round 6)
  static const int mode = [] {
    const char* e = study_env("MXAR_ADAM_STREAM");
    return e != nullptr ? std::atoi(e) : -1;
  }();
  if (mode == 3 || (mode < 0 && dt != DType::F32))
    launch_adamw_t<3, 2>(a, grid, s, dt);  // 16-bit parameters: run-contiguous halves (default)
  else if (mode == 1)
    launch_adamw_t<1, 2>(a, grid, s, dt);
  else if (mode == 2)
    launch_adamw_t<2, 2>(a, grid, s, dt);
  else
    launch_adamw_t<0, 2>(a, grid, s, dt);
}

}  // namespace mxar
