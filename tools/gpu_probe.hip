// Environment probe for the MI355X box: memory-type bandwidth and cross-process IPC
// (same device) with system-scope flag hand-off. Not part of the product; its output
// decides which allocation kinds the xGMI engine uses for slabs and flags.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <sys/wait.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d: %s\n", #x, __FILE__, __LINE__, hipGetErrorString(e)); exit(2);} } while (0)

__global__ void copy_k(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = a[i];
}
__global__ void fill_k(float* p, size_t n, float base) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) p[i] = base + (float)(i % 1000);
}
// producer: write payload to (remote) buffer, release at system scope, then raise flag
__global__ void produce_k(float* remote, size_t n, unsigned* flag, unsigned epoch) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) remote[i] = (float)epoch + (float)(i % 977);
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);  // default: system scope
    __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// consumer: wait for all producer blocks, acquire, verify
__global__ void consume_k(const float* buf, size_t n, unsigned* flag, unsigned target,
                          unsigned epoch, unsigned* bad, unsigned* timeout) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    long long t0 = wall_clock64();
    ok = 1;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > 100LL * 1000 * 1000 * 5) { atomicAdd(timeout, 1u); ok = 0; break; }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
  if (!ok) return;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  unsigned b = 0;
  for (; i < n; i += s) if (buf[i] != (float)epoch + (float)(i % 977)) b++;
  if (b) atomicAdd(bad, b);
}

static double bw_test(unsigned flags, const char* name) {
  size_t bytes = 1ull << 30; size_t n4 = bytes / 16;
  void *a, *b;
  CK(hipExtMallocWithFlags(&a, bytes, flags)); CK(hipExtMallocWithFlags(&b, bytes, flags));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; w++) copy_k<<<2048, 256>>>((float4*)a, (float4*)b, n4);
  CK(hipEventRecord(e0));
  int it = 10;
  for (int w = 0; w < it; w++) copy_k<<<2048, 256>>>((float4*)a, (float4*)b, n4);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  double gbs = 2.0 * bytes * it / (ms * 1e-3) / 1e9;
  printf("BW %-12s copy 1GiB: %.1f GB/s (%.3f ms/iter)\n", name, gbs, ms / it);
  CK(hipFree(a)); CK(hipFree(b));
  return gbs;
}

int main(int argc, char** argv) {
  int p2c[2], c2p[2];
  if (pipe(p2c) || pipe(c2p)) return 3;
  // fork BEFORE any HIP call
  pid_t pid = fork();
  if (pid == 0) {  // child = producer process
    hipIpcMemHandle_t h[2];
    if (read(p2c[0], h, sizeof(h)) != (ssize_t)sizeof(h)) { fprintf(stderr, "child read failed\n"); _exit(4); }
    CK(hipSetDevice(0));
    void *buf, *flag;
    hipError_t e1 = hipIpcOpenMemHandle(&buf, h[0], hipIpcMemLazyEnablePeerAccess);
    hipError_t e2 = hipIpcOpenMemHandle(&flag, h[1], hipIpcMemLazyEnablePeerAccess);
    printf("child: open data=%s flag=%s\n", hipGetErrorString(e1), hipGetErrorString(e2));
    fflush(stdout);
    if (e1 != hipSuccess || e2 != hipSuccess) { char c = 'x'; write(c2p[1], &c, 1); _exit(5); }
    size_t n = (64u << 20) / 4;
    for (unsigned ep = 1; ep <= 4; ++ep) {
      produce_k<<<512, 256>>>((float*)buf, n, (unsigned*)flag, ep);
      CK(hipDeviceSynchronize());
      char c = 'k'; if (write(c2p[1], &c, 1) != 1) _exit(6);
      if (read(p2c[0], &c, 1) != 1) _exit(7);
    }
    CK(hipIpcCloseMemHandle(buf)); CK(hipIpcCloseMemHandle(flag));
    printf("child: done\n");
    _exit(0);
  }
  // parent = consumer process
  CK(hipSetDevice(0));
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  printf("device %s gcn=%s CUs=%d mem=%.1f GiB l2=%d\n", prop.name, prop.gcnArchName,
         prop.multiProcessorCount, prop.totalGlobalMem / 1073741824.0, prop.l2CacheSize);
  int ndev; CK(hipGetDeviceCount(&ndev)); printf("ndev=%d\n", ndev);
  bw_test(hipDeviceMallocDefault, "default");
  bw_test(hipDeviceMallocFinegrained, "finegrained");
  bw_test(hipDeviceMallocUncached, "uncached");
  const char* kinds[3] = {"default", "finegrained", "uncached"};
  unsigned kflags[3] = {hipDeviceMallocDefault, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
  int kind = argc > 1 ? atoi(argv[1]) : 1;
  size_t n = (64u << 20) / 4;
  void *buf, *flag;
  CK(hipExtMallocWithFlags(&buf, n * 4, kflags[kind]));
  CK(hipExtMallocWithFlags(&flag, 4096, hipDeviceMallocUncached));
  CK(hipMemset(buf, 0, n * 4)); CK(hipMemset(flag, 0, 4096)); CK(hipDeviceSynchronize());
  hipIpcMemHandle_t h[2];
  hipError_t g1 = hipIpcGetMemHandle(&h[0], buf), g2 = hipIpcGetMemHandle(&h[1], flag);
  printf("parent: data kind=%s gethandle data=%s flag=%s\n", kinds[kind], hipGetErrorString(g1), hipGetErrorString(g2));
  if (write(p2c[1], h, sizeof(h)) != (ssize_t)sizeof(h)) return 8;
  unsigned *bad, *tmo; CK(hipMalloc(&bad, 8)); CK(hipMalloc(&tmo, 8));
  for (unsigned ep = 1; ep <= 4; ++ep) {
    char c; if (read(c2p[0], &c, 1) != 1 || c != 'k') { printf("parent: child failed\n"); break; }
    CK(hipMemset(bad, 0, 8)); CK(hipMemset(tmo, 0, 8));
    consume_k<<<512, 256>>>((float*)buf, n, (unsigned*)flag, ep * 512, ep, bad, tmo);
    unsigned hb[2]; CK(hipMemcpy(hb, bad, 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(hb + 1, tmo, 4, hipMemcpyDeviceToHost));
    printf("parent: epoch %u bad=%u timeout=%u\n", ep, hb[0], hb[1]);
    c = 'g'; if (write(p2c[1], &c, 1) != 1) break;
  }
  int st; waitpid(pid, &st, 0);
  printf("child exit=%d\n", WEXITSTATUS(st));
  return 0;
}
