// Store-path probe for the two-shot's scatter phase: copy a 256 MiB
// stream into (a) fine-grained device memory (hipDeviceMallocFinegrained, what the xGMI slabs
// are) and (b) ordinary hipMalloc memory, with the load / store flavours the data-plane copy
// loops could use. Geometry = the scatter's: every workgroup copies contiguous units of
// `unit` bytes (256 threads x 16 B x U packs per step). Reports TB/s (read + write).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_probe tools/store_probe.hip
//   tools/store_probe [MiB=256] [unit_KiB=512] [grid=512]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e = (x);                                                                         \
    if (e != hipSuccess) {                                                                      \
      std::fprintf(stderr, "HIP error %s at %s:%d: %s\n", #x, __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(2);                                                                             \
    }                                                                                           \
  } while (0)

typedef unsigned int Pack16 __attribute__((ext_vector_type(4)));
constexpr int kT = 256;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), static_cast<short>(0), 0x7fffffff, 0x00020000);
}

// LOAD: 0 plain global, 1 nt buffer load (aux 2), 2 sc1 buffer load (aux 16)
// STORE: 0 plain global, 1 sc0 sc1 write-through buffer store (aux 17), 2 nt buffer store (aux 2),
//        3 sc1 buffer store (aux 16)
template <int LOAD, int STORE, int U>
__global__ __launch_bounds__(kT) void copy_units(const char* __restrict__ src, char* __restrict__ dst, int64_t bytes,
                                                 int64_t unit) {
  const int64_t nunits = (bytes + unit - 1) / unit;
  for (int64_t u = blockIdx.x; u < nunits; u += gridDim.x) {
    const char* s = src + u * unit;
    char* d = dst + u * unit;
    const int64_t len = std::min<int64_t>(unit, bytes - u * unit);
    const int64_t npk = len / 16;
    const __amdgpu_buffer_rsrc_t rs = rsrc(s), rd = rsrc(d);
    for (int64_t i = threadIdx.x; i + (U - 1) * kT < npk; i += U * kT) {
      Pack16 v[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int64_t k = i + q * kT;
        if constexpr (LOAD == 0)
          v[q] = reinterpret_cast<const Pack16*>(s)[k];
        else
          v[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(k * 16), 0, LOAD == 1 ? 2 : 16);
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int64_t k = i + q * kT;
        if constexpr (STORE == 0)
          reinterpret_cast<Pack16*>(d)[k] = v[q];
        else
          __builtin_amdgcn_raw_buffer_store_b128(v[q], rd, static_cast<int>(k * 16), 0,
                                                 STORE == 1 ? 17 : STORE == 2 ? 2 : 16);
      }
    }
  }
}

struct Variant {
  const char* name;
  void (*k)(const char*, char*, int64_t, int64_t);
};

template <int L, int S, int U>
void launch(const char* a, char* b, int64_t bytes, int64_t unit, int grid) {
  hipLaunchKernelGGL((copy_units<L, S, U>), dim3(grid), dim3(kT), 0, 0, a, b, bytes, unit);
}

int main(int argc, char** argv) {
  const int64_t mib = argc > 1 ? std::atoll(argv[1]) : 256;
  const int64_t unit = (argc > 2 ? std::atoll(argv[2]) : 512) << 10;
  const int grid = argc > 3 ? std::atoi(argv[3]) : 512;
  const int64_t bytes = mib << 20;
  char *src = nullptr, *fine = nullptr, *coarse = nullptr;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&coarse, bytes));
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&fine), bytes, hipDeviceMallocFinegrained));
  CK(hipMemset(src, 1, bytes));
  CK(hipMemset(coarse, 0, bytes));
  CK(hipMemset(fine, 0, bytes));
  CK(hipDeviceSynchronize());
  struct V {
    const char* name;
    void (*fn)(const char*, char*, int64_t, int64_t, int);
  };
  const V vs[] = {
      {"plain ld / wt st (copy_to_slab), U8", launch<0, 1, 8>},
      {"plain ld / wt st, U4", launch<0, 1, 4>},
      {"nt ld / wt st, U8", launch<1, 1, 8>},
      {"sc1 ld / wt st, U8", launch<2, 1, 8>},
      {"plain ld / plain st, U8", launch<0, 0, 8>},
      {"plain ld / nt st, U8", launch<0, 2, 8>},
      {"nt ld / nt st, U8", launch<1, 2, 8>},
      {"plain ld / sc1 st, U8", launch<0, 3, 8>},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("{\"bytes\": %lld, \"unit\": %lld, \"grid\": %d, \"rows\": [\n", (long long)bytes, (long long)unit, grid);
  bool first = true;
  for (int rep = 0; rep < 2; ++rep)
    for (const V& v : vs)
      for (int kind = 0; kind < 2; ++kind) {
        char* dst = kind == 0 ? fine : coarse;
        for (int w = 0; w < 3; ++w) v.fn(src, dst, bytes, unit, grid);
        std::vector<float> ts;
        for (int it = 0; it < 15; ++it) {
          CK(hipEventRecord(e0, 0));
          v.fn(src, dst, bytes, unit, grid);
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const float p50 = ts[ts.size() / 2];
        std::printf("%s {\"rep\": %d, \"variant\": \"%s\", \"dst\": \"%s\", \"p50_us\": %.1f, \"TBps\": %.3f}\n",
                    first ? " " : ",", rep, v.name, kind == 0 ? "fine" : "coarse", p50 * 1e3,
                    2.0 * bytes / (p50 / 1e3) / 1e12);
        first = false;
      }
  std::printf("]}\n");
  CK(hipFree(src));
  CK(hipFree(coarse));
  CK(hipFree(fine));
  return 0;
}
