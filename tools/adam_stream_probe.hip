// Roofline of the fused AdamW step's memory pattern (xgmi_adam.hip at world 1): per parameter
// read bf16 grad + fp32 master / m / v, write fp32 master / m / v + bf16 param = 28 B, eight
// streams, no communication. A plain streaming kernel with the same streams and a trivial
// update, so the fused kernel's TB/s can be set against what the pattern itself reaches.
//   mode 0: plain loads / stores
//   mode 1: nontemporal loads / stores (__builtin_nontemporal_*)
//   mode 2: plain loads, nontemporal stores
// Output: one JSON line per (mode, grid): ms per step, HBM TB/s at 28 B/param; plus a 2-stream
// copy of the same byte count for the copy roofline.
//   hipcc --offload-arch=gfx950 -O3 -o tools/adam_stream_probe.bin tools/adam_stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int MODE>
__device__ __forceinline__ f4 ldf(const f4* p) {
  if constexpr (MODE == 1) return __builtin_nontemporal_load(p);
  return *p;
}
template <int MODE>
__device__ __forceinline__ u4 ldu(const u4* p) {
  if constexpr (MODE == 1) return __builtin_nontemporal_load(p);
  return *p;
}
template <int MODE>
__device__ __forceinline__ void stf(f4* p, f4 v) {
  if constexpr (MODE == 1 || MODE == 2) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <int MODE>
__device__ __forceinline__ void stu(u4* p, u4 v) {
  if constexpr (MODE == 1 || MODE == 2) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__device__ __forceinline__ float bf(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ uint32_t tobf(float f) { return __float_as_uint(f) >> 16; }

// one unit = 8 parameters: 16 B of bf16 grad, 2 x 16 B of each fp32 array, 16 B of bf16 param
// MODE 3: plain access, but each workgroup walks ONE contiguous range of the arrays (blocked)
// instead of the grid-stride interleave: fewer concurrently open DRAM pages per stream
template <int MODE>
__global__ __launch_bounds__(256) void adam_like(const u4* g, f4* p, f4* m, f4* v, u4* w, int64_t units, float lr) {
  int64_t u0 = blockIdx.x * 256 + threadIdx.x, stride = static_cast<int64_t>(gridDim.x) * 256, u1 = units;
  if constexpr (MODE == 3) {
    const int64_t per = (units + gridDim.x - 1) / gridDim.x;
    u0 = blockIdx.x * per + threadIdx.x;
    u1 = units < (blockIdx.x + 1) * per ? units : (blockIdx.x + 1) * per;
    stride = 256;
  }
  for (int64_t u = u0; u < u1; u += stride) {
    const u4 gg = ldu<MODE>(g + u);
    f4 p0 = ldf<MODE>(p + 2 * u), p1 = ldf<MODE>(p + 2 * u + 1);
    f4 m0 = ldf<MODE>(m + 2 * u), m1 = ldf<MODE>(m + 2 * u + 1);
    f4 v0 = ldf<MODE>(v + 2 * u), v1 = ldf<MODE>(v + 2 * u + 1);
    float gf[8];
    for (int i = 0; i < 4; ++i) {
      gf[2 * i] = bf(gg[i] & 0xffffu);
      gf[2 * i + 1] = bf(gg[i] >> 16);
    }
    u4 out;
    for (int i = 0; i < 4; ++i) {
      const float ga = gf[i], gb = gf[4 + i];
      m0[i] = 0.9f * m0[i] + 0.1f * ga;
      m1[i] = 0.9f * m1[i] + 0.1f * gb;
      v0[i] = 0.999f * v0[i] + 0.001f * ga * ga;
      v1[i] = 0.999f * v1[i] + 0.001f * gb * gb;
      p0[i] -= lr * m0[i] * __frsqrt_rn(v0[i] + 1e-8f);
      p1[i] -= lr * m1[i] * __frsqrt_rn(v1[i] + 1e-8f);
    }
    for (int i = 0; i < 2; ++i) out[i] = tobf(p0[2 * i]) | (tobf(p0[2 * i + 1]) << 16);
    for (int i = 0; i < 2; ++i) out[2 + i] = tobf(p1[2 * i]) | (tobf(p1[2 * i + 1]) << 16);
    stf<MODE>(p + 2 * u, p0);
    stf<MODE>(p + 2 * u + 1, p1);
    stf<MODE>(m + 2 * u, m0);
    stf<MODE>(m + 2 * u + 1, m1);
    stf<MODE>(v + 2 * u, v0);
    stf<MODE>(v + 2 * u + 1, v1);
    stu<MODE>(w + u, out);
  }
}

// MODE 4: the same 28 B/param, lane-contiguous: unit u = 8 parameters as two halves of 4, at
// element offsets [4l, 4l + 4) of each 1024-parameter half of a 256-lane run (the fused
// kernel's default layout since round 5), so every fp32 access of a wave is 1 KiB of
// consecutive bytes and every bf16 one 512 B. Modes 0-3 give each lane 32 consecutive fp32
// bytes, so each 16-B instruction touches every other 16 B of 2 KiB.
__global__ __launch_bounds__(256) void adam_like_halves(const uint2* g, f4* p, f4* m, f4* v, uint2* w, int64_t units,
                                                         float lr) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  for (int64_t u = blockIdx.x * 256 + threadIdx.x; u < units; u += stride) {
    const int64_t run = u / 256, l = u - run * 256;
    for (int h = 0; h < 2; ++h) {
      const int64_t q = run * 512 + h * 256 + l;  // index in units of 4 parameters
      const uint2 gg = g[q];
      f4 p0 = p[q], m0 = m[q], v0 = v[q];
      const float gf[4] = {bf(gg.x & 0xffffu), bf(gg.x >> 16), bf(gg.y & 0xffffu), bf(gg.y >> 16)};
      for (int i = 0; i < 4; ++i) {
        m0[i] = 0.9f * m0[i] + 0.1f * gf[i];
        v0[i] = 0.999f * v0[i] + 0.001f * gf[i] * gf[i];
        p0[i] -= lr * m0[i] * __frsqrt_rn(v0[i] + 1e-8f);
      }
      p[q] = p0;
      m[q] = m0;
      v[q] = v0;
      w[q] = make_uint2(tobf(p0[0]) | (tobf(p0[1]) << 16), tobf(p0[2]) | (tobf(p0[3]) << 16));
    }
  }
}

__global__ __launch_bounds__(256) void copy4(const f4* a, f4* b, int64_t n4) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) b[i] = a[i];
}

template <int MODE>
int run(int grid, const u4* g, f4* p, f4* m, f4* v, u4* w, int64_t units, hipEvent_t e0, hipEvent_t e1) {
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(adam_like<MODE>, dim3(grid), dim3(256), 0, 0, g, p, m, v, w, units, 1e-6f);
  CHECK(hipDeviceSynchronize());
  const int it = 20;
  CHECK(hipEventRecord(e0, 0));
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(adam_like<MODE>, dim3(grid), dim3(256), 0, 0, g, p, m, v, w, units, 1e-6f);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= it;
  const double bytes = 28.0 * 8.0 * static_cast<double>(units);
  std::printf("{\"kernel\": \"adam_like\", \"mode\": %d, \"grid\": %d, \"params\": %lld, \"ms\": %.4f, \"TBps\": %.3f}\n", MODE,
              grid, static_cast<long long>(units * 8), ms, bytes / (ms * 1e-3) / 1e12);
  return 0;
}

int main() {
  const int64_t params = int64_t{134217728};
  const int64_t units = params / 8;
  u4 *g = nullptr, *w = nullptr;
  f4 *p = nullptr, *m = nullptr, *v = nullptr;
  CHECK(hipMalloc(&g, params * 2));
  CHECK(hipMalloc(&w, params * 2));
  CHECK(hipMalloc(&p, params * 4));
  CHECK(hipMalloc(&m, params * 4));
  CHECK(hipMalloc(&v, params * 4));
  CHECK(hipMemset(g, 0x3c, params * 2));
  CHECK(hipMemset(p, 0, params * 4));
  CHECK(hipMemset(m, 0, params * 4));
  CHECK(hipMemset(v, 0, params * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int grid : {1024, 2048, 4096, 8192}) {
    if (run<0>(grid, g, p, m, v, w, units, e0, e1) || run<1>(grid, g, p, m, v, w, units, e0, e1) ||
        run<2>(grid, g, p, m, v, w, units, e0, e1))
      return 1;
  }
  for (int grid : {256, 512, 1024, 2048}) {
    if (run<3>(grid, g, p, m, v, w, units, e0, e1)) return 1;
  }
  for (int grid : {1024, 2048, 4096, 8192}) {  // MODE 4: lane-contiguous halves
    for (int i = 0; i < 3; ++i)
      hipLaunchKernelGGL(adam_like_halves, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const uint2*>(g), p, m, v,
                         reinterpret_cast<uint2*>(w), units, 1e-6f);
    CHECK(hipDeviceSynchronize());
    const int it = 20;
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < it; ++i)
      hipLaunchKernelGGL(adam_like_halves, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const uint2*>(g), p, m, v,
                         reinterpret_cast<uint2*>(w), units, 1e-6f);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    const double bytes = 28.0 * 8.0 * static_cast<double>(units);
    std::printf("{\"kernel\": \"adam_like\", \"mode\": 4, \"grid\": %d, \"params\": %lld, \"ms\": %.4f, \"TBps\": %.3f}\n",
                grid, static_cast<long long>(units * 8), ms, bytes / (ms * 1e-3) / 1e12);
  }
  // copy roofline: the fp32 master array into v (4 B/param read + 4 B/param written)
  {
    const int64_t n4 = params / 4;  // f4 elements of one fp32 array
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(copy4, dim3(4096), dim3(256), 0, 0, p, v, n4);
    CHECK(hipDeviceSynchronize());
    const int it = 20;
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL(copy4, dim3(4096), dim3(256), 0, 0, p, v, n4);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    const double bytes = 2.0 * 16.0 * static_cast<double>(n4);
    std::printf("{\"kernel\": \"copy\", \"bytes_moved\": %.0f, \"ms\": %.4f, \"TBps\": %.3f}\n", bytes, ms,
                bytes / (ms * 1e-3) / 1e12);
  }
  return 0;
}
