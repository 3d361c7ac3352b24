// SdmaComm: a bucket allreduce whose cross-rank data movement runs on the copy engines
// (SDMA), not on CU workgroups - the MI355X-native form of SURVEY §2.4 K2's
// "hipMemcpyPeerAsync writes the source slice into the owner's scatter slot", for DP buckets
// that run beside backward's GEMMs (BASELINE config 5). Same direct two-shot as XgmiComm
// (the reference's ScatterBlock / ReduceBlock, AllreduceWorker.scala:194-238):
//
//   phase 1  ScatterBlock   block j of the input -> rank j's SD slot [r], in K pipeline
//                           pieces: piece k is split over the `engines_per_peer` engines,
//                           and a 4-byte SDMA copy of the epoch into rank j's FS[r][k] flag
//                           follows its parts (HSA completion-signal dependencies)
//   reduce                  ONE small-grid kernel (grid_ workgroups, every local rank) walks
//                           the pieces in order: wait for FS[*][k], sum piece k of the own
//                           block from the input and the P-1 SD slots, and the piece's last
//                           workgroup releases the signal its phase-2 copies wait on - so
//                           the engines copy piece k + 1 while the CUs reduce piece k
//   phase 2  ReduceBlock    reduced piece k -> every peer's RD slot [r] + FR[r][k] (SDMA)
//   gather                  ONE small-grid kernel copies each peer's RD piece into the
//                           output as soon as its FR flag shows the epoch
//
// Stream ordering without the host: HIP's hipMemcpyAsync runs device-to-device copies as
// blit KERNELS (profiles/round4/README.md, tools/sdma_probe.cc in git history), so the copies are submitted
// with hsa_amd_memory_async_copy_on_engine(force_copy_on_sdma). Each call's copies are
// queued at call time but depend on an HSA signal that a one-lane kernel on the caller's
// stream releases (after a system-scope release event, so the engines read what earlier
// kernels wrote); the engines themselves wait on it. Flag waits are one-wave kernels with a
// wall-clock deadline (error word, never a hang). SD / RD slots are double-buffered by the
// call epoch's parity: a rank can be at most one call ahead of any peer still reading.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "xgmi_comm.h"

namespace mxar {

constexpr int kSdmaMaxPieces = 8;  // pipeline pieces per block at most
constexpr int kSdmaMaxLocal = 8;   // local ranks one reduce / gather launch serves

struct SdmaStats {
  uint64_t calls = 0, copies = 0, bytes = 0, host_waits = 0;
};

class SdmaComm {
 public:
  // slot_bytes: capacity of one SD / RD slot (one block of one peer); calls reduce up to
  // world * slot_bytes bytes (larger tensors are processed in segments).
  // engines_per_peer: SDMA engines one peer's block is split over; 0 = the device's engines
  // (this rank's share of them with connect_local) spread over the world - 1 peers
  SdmaComm(int rank, int world, int device, int64_t slot_bytes, int grid = 32, int engines_per_peer = 0,
           double timeout_s = 20.0);
  ~SdmaComm();
  SdmaComm(const SdmaComm&) = delete;
  SdmaComm& operator=(const SdmaComm&) = delete;

  // IPC handle of the slab + the device's PCI location (peers map the slab and pick the
  // SDMA engines towards this GPU from it).
  std::string handle() const;
  void connect(const std::vector<std::string>& handles);
  // ranks of ONE process (the one-GPU rehearsal): slabs shared directly
  void connect_local(const std::vector<SdmaComm*>& comms);

  // out = scale * sum over ranks of in (out may alias in), enqueued on `stream`.
  void allreduce(const void* in, void* out, int64_t n, DType dt, hipStream_t stream, float scale = 1.f);
  // every rank of this process (connect_local) in one stream-ordered schedule
  static void allreduce_local(const std::vector<SdmaComm*>& comms, const std::vector<const void*>& ins,
                              const std::vector<void*>& outs, int64_t n, DType dt, hipStream_t stream,
                              float scale = 1.f);

  uint32_t error() const;
  void clear_error();
  std::string debug_state() const;  // signals of the calls in flight, flag words (bring-up)
  int rank() const { return rank_; }
  int world() const { return world_; }
  int grid() const { return grid_; }
  void set_grid(int g) { grid_ = g > 0 ? g : 1; }
  // pipeline pieces per block (0 = by size: one per 64 MiB of the block, 2..kSdmaMaxPieces;
  // profiles/round6/sdma_pipe_*.jsonl: 2 pieces at 32-128 MiB blocks, grid 128)
  int pieces() const { return pieces_; }
  void set_pieces(int k) { pieces_ = k < 0 ? 0 : k; }
  int engines() const { return static_cast<int>(local_engines_.size()); }
  int engines_per_peer() const { return epp_; }
  int64_t slot_bytes() const { return slot_bytes_; }
  const SdmaStats& stats() const { return st_; }

 private:
  struct Impl;
  struct Plan {
    const char* in = nullptr;
    char* out = nullptr;
    int64_t n = 0, block = 0, pe = 0;  // pe: elements per pipeline piece
    int K = 1;                         // pipeline pieces of a block
    DType dt = DType::F32;
    uint32_t epoch = 0;
    int par = 0, slot = 0;
  };
  // one segment: wait for the slot, arm its signals, queue both phases' copies (host)
  Plan plan(const char* in, char* out, int64_t n, DType dt);
  int rank_, world_, device_;
  int64_t slot_bytes_;
  int grid_;
  int epp_;
  int pieces_ = 0;
  uint32_t* cnt_ = nullptr;  // device: per-piece workgroup tickets of the reduce kernel
  double timeout_s_;
  char* slab_ = nullptr;
  int64_t slab_bytes_ = 0;
  uint32_t* err_ = nullptr;  // device error word
  std::vector<char*> peers_;
  std::vector<bool> opened_;
  std::vector<uint32_t> local_engines_;
  uint64_t epoch_ = 0;
  bool connected_ = false;
  SdmaStats st_;
  std::unique_ptr<Impl> impl_;
};

// HSA view of the machine (agents, PCI locations, SDMA engine masks): bring-up diagnostics
std::string sdma_diagnose(int device);
// ms per engine copy of `bytes` (src -> dst on `device`, engine index into its mask)
double sdma_copy_probe(int device, uint64_t dst, uint64_t src, int64_t bytes, int engine, int iters,
                       int nengines = 1);
// PCI location of a HIP device ((domain << 32) | bdf): which GPU a rank's SDMA slab lives on,
// known before anything is allocated (SdmaCommunicator's cross-GPU check).
uint64_t pci_location(int device);

}  // namespace mxar
