// xGMI bring-up probes (bench.py `xgmi_links`; XgmiComm::probe_push / probe_pingpong).
//
// The reference's whole data plane is the all-peer fan-out: every worker scatters a chunk to
// every other worker (AllreduceWorker.scala:194-209) and broadcasts every reduced chunk to
// all of them (:230-238). On an 8 x MI355X node that is 7 xGMI links per GPU driven at once.
// Before the first multi-GPU allreduce is timed, these probes measure what those links give
// THIS store path - the two-shot's own write-through `st16_wt` pushes into a peer's
// fine-grained slab and its relaxed system-scope flag store + poll - so a slow or failing
// first 8-GPU run says whether the links, the flag hand-off or the kernels are at fault:
//   * probe_push: raw push rate into one peer, or into every peer at once (gridDim.y = peers);
//   * probe_pingpong: flag round trip between two ranks, relaxed (the wire) and with the
//     kernels' release / acquire fences (the production hand-off).
// Neither touches a flag word or a control word of the collectives: the push lands in the
// S slot the two-shot's scatter writes (row 0, column = this rank) and the ping-pong words
// sit at the end of that slot, past any probe payload. Callers run them between collective
// quiet points (every rank idle, barriers around), which bench.py does.
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "xgmi_device.h"

namespace mxar {

namespace {

struct ProbeArgs {
  const char* src;
  char* dst[kMaxRanks];  // per row y: the peer's slot (mode 0, 2) or coarse buffer (mode 1)
  int64_t bytes;         // per destination, a multiple of 16
};

// Workgroup x of row y moves its contiguous piece between src and dst[y], 16 B per lane:
//   MODE 0  src -> peer slab: nt loads, write-through stores (copy_to_slab, the scatter's loop)
//   MODE 1  src -> peer coarse buffer: plain loads and stores (4 in flight per lane), then one
//           system-scope release per workgroup (its dirty lines written back to the peer)
//   MODE 2  peer slab -> src: remote loads (system-coherent: fine-grained memory is not
//           cached), plain local stores
template <int MODE>
__global__ __launch_bounds__(kCommThreads) void probe_push_kernel(ProbeArgs a) {
  const int64_t npk = a.bytes / 16;
  const int64_t per = (npk + gridDim.x - 1) / gridDim.x;
  const int64_t p0 = static_cast<int64_t>(blockIdx.x) * per;
  const int64_t len = clamp_len(npk - p0, per);
  if constexpr (MODE == 0) {
    if (len > 0) copy_to_slab<F32>(a.dst[blockIdx.y] + p0 * 16, a.src + p0 * 16, len * F32::ELEMS);
  } else {
    const uint4* s = reinterpret_cast<const uint4*>(MODE == 1 ? a.src : a.dst[blockIdx.y]) + p0;
    uint4* d = reinterpret_cast<uint4*>(MODE == 1 ? a.dst[blockIdx.y] : const_cast<char*>(a.src)) + p0;
    constexpr int U = 4;
    int64_t i = threadIdx.x;
    for (; i + (U - 1) * kCommThreads < len; i += U * kCommThreads) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = s[i + u * kCommThreads];
#pragma unroll
      for (int u = 0; u < U; ++u) d[i + u * kCommThreads] = v[u];
    }
    for (; i < len; i += kCommThreads) d[i] = s[i];
    if constexpr (MODE == 1) {
      __syncthreads();
      if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    }
  }
}

// One lane per side. Token i of this probe = nonce << 16 | i (the words may hold any older
// value, never one of these tokens unless the nonce repeats). Leader: store, then wait for the
// echo; echo: wait, then store back. `fenced`: the kernels' hand-off (system release before the
// store, system acquire after the wait) instead of the bare relaxed store / poll.
__global__ void probe_pingpong_kernel(uint32_t* mine, uint32_t* theirs, int leader, int iters, uint32_t nonce,
                                      int fenced, uint64_t timeout, uint64_t* out, uint32_t* err) {
  if (threadIdx.x != 0) return;
  const uint64_t deadline = wall_ticks() + timeout;
  bool ok = true;
  const uint64_t t0 = wall_ticks();
  for (int i = 1; i <= iters && ok; ++i) {
    const uint32_t tok = (nonce << 16) | static_cast<uint32_t>(i);
    if (leader) {
      if (fenced) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      st_flag(theirs, tok);
    }
    while (ld_flag(mine) != tok) {
      if (wall_ticks() > deadline) {
        ok = false;
        break;
      }
    }
    if (fenced) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (!leader && ok) {
      if (fenced) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      st_flag(theirs, tok);
    }
  }
  const uint64_t t1 = wall_ticks();
  if (!ok) __hip_atomic_fetch_or(err, ERR_TIMEOUT_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  out[0] = ok ? t1 - t0 : 0;
}

}  // namespace

int64_t XgmiComm::probe_max_bytes() const { return slot_bytes_ - 4096; }

void XgmiComm::probe_push(const void* src, int64_t bytes, uint32_t peer_mask, int grid, hipStream_t stream, int mode) {
  if (!connected_) throw std::runtime_error("XgmiComm.probe_push: connect() first");
  if (bytes <= 0 || bytes % 16 || bytes > probe_max_bytes() || (reinterpret_cast<uintptr_t>(src) & 15))
    throw std::invalid_argument("XgmiComm.probe_push: bytes must be a positive multiple of 16 <= probe_max_bytes() "
                                "and src 16-byte aligned");
  if (mode < 0 || mode > 2) throw std::invalid_argument("XgmiComm.probe_push: mode 0 (push), 1 (coarse push), 2 (pull)");
  if (mode == 1 && static_cast<int>(probe_peers_.size()) != world_)
    throw std::runtime_error("XgmiComm.probe_push(mode=1): probe_coarse_connect() first");
  ProbeArgs a{};
  a.src = static_cast<const char*>(src);
  a.bytes = bytes;
  int np = 0;
  for (int k = 0; k < world_; ++k)
    if (k != rank_ && (peer_mask >> k) & 1u)
      a.dst[np++] = mode == 1 ? probe_peers_[k] : peers_[k] + off_S_ + static_cast<int64_t>(rank_) * slot_stride_;
  if (np == 0) return;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  order_after_last(stream);
  const dim3 g(std::max(1, grid), np), b(kCommThreads);
  if (mode == 0) hipLaunchKernelGGL(probe_push_kernel<0>, g, b, 0, stream, a);
  if (mode == 1) hipLaunchKernelGGL(probe_push_kernel<1>, g, b, 0, stream, a);
  if (mode == 2) hipLaunchKernelGGL(probe_push_kernel<2>, g, b, 0, stream, a);
  hip_check(hipGetLastError(), "probe_push launch");
}

std::string XgmiComm::probe_coarse_handle() {
  hip_check(hipSetDevice(device_), "hipSetDevice");
  if (probe_coarse_ == nullptr)
    hip_check(hipMalloc(reinterpret_cast<void**>(&probe_coarse_), ipc_safe_bytes(probe_max_bytes())),
              "hipMalloc(coarse probe buffer)");
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, probe_coarse_), "hipIpcGetMemHandle(coarse probe buffer)");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void XgmiComm::probe_coarse_connect(const std::vector<std::string>& handles) {
  if (static_cast<int>(handles.size()) != world_) throw std::invalid_argument("probe_coarse_connect: one handle per rank");
  if (probe_coarse_ == nullptr) throw std::runtime_error("probe_coarse_connect: probe_coarse_handle() first");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  if (!probe_peers_.empty()) return;  // mapped by an earlier probe
  probe_peers_.assign(world_, nullptr);
  for (int k = 0; k < world_; ++k) {
    if (k == rank_) {
      probe_peers_[k] = probe_coarse_;
      continue;
    }
    if (handles[k].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("probe_coarse_connect: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[k].data(), sizeof(h));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(coarse probe buffer)");
    probe_peers_[k] = static_cast<char*>(p);
  }
}

void XgmiComm::probe_pingpong(int peer, int iters, uint32_t nonce, bool fenced, uint64_t* out, hipStream_t stream) {
  if (!connected_) throw std::runtime_error("XgmiComm.probe_pingpong: connect() first");
  if (peer < 0 || peer >= world_ || peer == rank_ || iters < 1 || iters > 65535)
    throw std::invalid_argument("XgmiComm.probe_pingpong: bad peer or iters (1..65535)");
  const int64_t word = slot_bytes_ - 64;  // past any probe_push payload (probe_max_bytes)
  uint32_t* mine = reinterpret_cast<uint32_t*>(slab_ + off_S_ + static_cast<int64_t>(peer) * slot_stride_ + word);
  uint32_t* theirs = reinterpret_cast<uint32_t*>(peers_[peer] + off_S_ + static_cast<int64_t>(rank_) * slot_stride_ + word);
  hip_check(hipSetDevice(device_), "hipSetDevice");
  order_after_last(stream);
  hipLaunchKernelGGL(probe_pingpong_kernel, dim3(1), dim3(64), 0, stream, mine, theirs, rank_ < peer ? 1 : 0, iters,
                     nonce & 0xFFFFu, fenced ? 1 : 0, static_cast<uint64_t>(timeout_s_ * 1e8), out, ctl_ + 2);
  hip_check(hipGetLastError(), "probe_pingpong launch");
}

}  // namespace mxar
