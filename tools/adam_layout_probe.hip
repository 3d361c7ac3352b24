// AdamW state layout probe (study, not part of the engine): the world-size-1 fused step's
// memory pattern - bf16 grad in, fp32 master / exp_avg / exp_avg_sq read and written back,
// bf16 param out - with the state as three arrays (SoA, what xgmi_adam.hip uses) or
// interleaved per 4 parameters as {p[4], m[4], v[4]} (AoS: one state stream instead of three).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/adam_probe tools/adam_layout_probe.hip
//   ./adam_probe [millions of params]
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr int kThreads = 256;
constexpr float lr = 1e-4f, b1 = 0.9f, b2 = 0.95f, eps = 1e-8f, wd = 0.1f, c1 = 0.1f, c2s = 0.3f;

__device__ __forceinline__ float adamw(float g, float& p, float& m, float& v) {
  p *= 1.f - lr * wd;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  p -= (lr / c1) * m / (sqrtf(v) / c2s + eps);
  return p;
}

__device__ __forceinline__ float bf(uint16_t x) { return __uint_as_float(static_cast<uint32_t>(x) << 16); }
__device__ __forceinline__ uint16_t tobf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fff + ((u >> 16) & 1);
  return static_cast<uint16_t>(u >> 16);
}

// 8 params per lane per iteration (one 16-byte bf16 grad pack), workgroup-contiguous tiles
template <bool NT>
__global__ __launch_bounds__(kThreads) void soa(const uint4* g, float4* p, float4* m, float4* v, uint4* out,
                                                int64_t npk) {
  const int64_t per = (npk + gridDim.x - 1) / gridDim.x;
  const int64_t beg = blockIdx.x * per, end = beg + per < npk ? beg + per : npk;
  for (int64_t i = beg + threadIdx.x; i < end; i += kThreads) {
    uint4 gg;
    if (NT) {
      const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(g) + i);
      gg = make_uint4(t.x, t.y, t.z, t.w);
    } else {
      gg = g[i];
    }
    float4 P[2] = {p[2 * i], p[2 * i + 1]}, M[2] = {m[2 * i], m[2 * i + 1]}, V[2] = {v[2 * i], v[2 * i + 1]};
    const uint32_t w[4] = {gg.x, gg.y, gg.z, gg.w};
    float* pp = reinterpret_cast<float*>(P);
    float* mm = reinterpret_cast<float*>(M);
    float* vv = reinterpret_cast<float*>(V);
    uint16_t o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      o[e] = tobf(adamw(bf(static_cast<uint16_t>(w[e / 2] >> (16 * (e & 1)))), pp[e], mm[e], vv[e]));
    p[2 * i] = P[0], p[2 * i + 1] = P[1], m[2 * i] = M[0], m[2 * i + 1] = M[1], v[2 * i] = V[0], v[2 * i + 1] = V[1];
    const uint4 ov = make_uint4(o[0] | (uint32_t(o[1]) << 16), o[2] | (uint32_t(o[3]) << 16),
                                o[4] | (uint32_t(o[5]) << 16), o[6] | (uint32_t(o[7]) << 16));
    if (NT)
      __builtin_nontemporal_store(u32x4{ov.x, ov.y, ov.z, ov.w}, reinterpret_cast<u32x4*>(out) + i);
    else
      out[i] = ov;
  }
}

// lane-contiguous: 4 params per lane per access (8-byte bf16 grad, one float4 per state
// array), adjacent lanes adjacent, so every store instruction writes a full 1 KiB span;
// two accesses in flight per lane (loads of both issued before the first update)
__global__ __launch_bounds__(kThreads) void soa_lc(const uint2* g, float4* p, float4* m, float4* v, uint2* out,
                                                   int64_t nq) {
  const int64_t per = (nq + gridDim.x - 1) / gridDim.x;
  const int64_t beg = blockIdx.x * per, end = beg + per < nq ? beg + per : nq;
  for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += 2 * kThreads) {
    uint2 gg[2];
    float4 P[2], M[2], V[2];
    bool live[2];
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const int64_t i = i0 + w * kThreads;
      live[w] = i < end;
      if (!live[w]) continue;
      gg[w] = g[i];
      P[w] = p[i], M[w] = m[i], V[w] = v[i];
    }
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      if (!live[w]) continue;
      const int64_t i = i0 + w * kThreads;
      const uint32_t wd2[2] = {gg[w].x, gg[w].y};
      float* pp = reinterpret_cast<float*>(&P[w]);
      float* mm = reinterpret_cast<float*>(&M[w]);
      float* vv = reinterpret_cast<float*>(&V[w]);
      uint16_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = tobf(adamw(bf(static_cast<uint16_t>(wd2[e / 2] >> (16 * (e & 1)))), pp[e], mm[e], vv[e]));
      p[i] = P[w], m[i] = M[w], v[i] = V[w];
      out[i] = make_uint2(o[0] | (uint32_t(o[1]) << 16), o[2] | (uint32_t(o[3]) << 16));
    }
  }
}

// state interleaved: per 4 params {p4, m4, v4} = 48 bytes; 8 params = 6 float4
__global__ __launch_bounds__(kThreads) void aos(const uint4* g, float4* st, uint4* out, int64_t npk) {
  const int64_t per = (npk + gridDim.x - 1) / gridDim.x;
  const int64_t beg = blockIdx.x * per, end = beg + per < npk ? beg + per : npk;
  for (int64_t i = beg + threadIdx.x; i < end; i += kThreads) {
    const uint4 gg = g[i];
    float4 S[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) S[k] = st[6 * i + k];
    const uint32_t w[4] = {gg.x, gg.y, gg.z, gg.w};
    uint16_t o[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float* pp = reinterpret_cast<float*>(&S[3 * h]);
      float* mm = reinterpret_cast<float*>(&S[3 * h + 1]);
      float* vv = reinterpret_cast<float*>(&S[3 * h + 2]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = 4 * h + e;
        o[q] = tobf(adamw(bf(static_cast<uint16_t>(w[q / 2] >> (16 * (q & 1)))), pp[e], mm[e], vv[e]));
      }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) st[6 * i + k] = S[k];
    out[i] = make_uint4(o[0] | (uint32_t(o[1]) << 16), o[2] | (uint32_t(o[3]) << 16), o[4] | (uint32_t(o[5]) << 16),
                        o[6] | (uint32_t(o[7]) << 16));
  }
}

int main(int argc, char** argv) {
  const int64_t n = (argc > 1 ? std::atoll(argv[1]) : 512) * 1000000LL / 8 * 8;
  const int64_t npk = n / 8;
  uint4 *g, *out;
  float4 *p, *m, *v, *st;
  CK(hipMalloc(&g, n * 2));
  CK(hipMalloc(&out, n * 2));
  CK(hipMalloc(&p, n * 4));
  CK(hipMalloc(&m, n * 4));
  CK(hipMalloc(&v, n * 4));
  CK(hipMalloc(&st, n * 12));
  CK(hipMemset(g, 0x3c, n * 2));
  CK(hipMemset(p, 0, n * 4));
  CK(hipMemset(m, 0, n * 4));
  CK(hipMemset(v, 0, n * 4));
  CK(hipMemset(st, 0, n * 12));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes = 28.0 * n;
  for (int grid : {256, 512, 1024}) {
    for (int rep = 0; rep < 2; ++rep) {
      for (int layout = 0; layout < 4; ++layout) {
        auto run = [&] {
          if (layout == 0)
            hipLaunchKernelGGL(soa<false>, dim3(grid), dim3(kThreads), 0, 0, g, p, m, v, out, npk);
          else if (layout == 2)
            hipLaunchKernelGGL(soa<true>, dim3(grid), dim3(kThreads), 0, 0, g, p, m, v, out, npk);
          else if (layout == 3)
            hipLaunchKernelGGL(soa_lc, dim3(grid), dim3(kThreads), 0, 0, reinterpret_cast<const uint2*>(g), p, m, v,
                               reinterpret_cast<uint2*>(out), 2 * npk);
          else
            hipLaunchKernelGGL(aos, dim3(grid), dim3(kThreads), 0, 0, g, st, out, npk);
        };
        run();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int it = 0; it < 10; ++it) {
          CK(hipEventRecord(a));
          run();
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const float med = ts[ts.size() / 2];
        std::printf("{\"layout\": \"%s\", \"grid\": %d, \"rep\": %d, \"params\": %lld, \"ms\": %.3f, \"TBps\": %.2f}\n",
                    layout == 3 ? "soa_lc" : layout == 2 ? "soa_nt_grad_out" : layout ? "aos" : "soa", grid, rep, static_cast<long long>(n), med, bytes / med / 1e9);
        std::fflush(stdout);
      }
    }
  }
  return 0;
}
