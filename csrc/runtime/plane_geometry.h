// The kernel geometry of a protocol round (block, kernel chunk, chunks per block) as a pure
// function of the membership - InitWorkers alone. Every worker of a job must run the SAME
// chunking: peers store into each other's slots at chunk offsets and raise per-chunk flags,
// so two workers that disagree on the chunk size write where the other never reads (wrong
// sums or gather timeouts). Every input here is job-wide: the reference's geometry
// (dataSize, peers, maxChunkSize; AllreduceWorker.scala:56-57,211-214), the thresholds, and
// what each worker's plane descriptor announces (its grid and geometry knobs, its process and
// device) - never the calling worker's own placement. csrc/hip/xgmi_plane.cc configure() runs
// it; tests/test_plane_loopback.py checks mixed placements on the CPU.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "round_plane.h"

namespace mxar {

// One worker's xGMI plane descriptor: "xgmi1 pid=<pid> dev=<device> bytes=<arena bytes>
// id=<arena id> grid=<workgroups> wgc=<chunks per workgroup cap> coarsen=<0|1> h=<hex handle>"
struct PlaneDesc {
  long pid = 0;
  int device = 0;
  int64_t bytes = 0;
  uint64_t id = 0;
  int grid = 0;         // the plane's effective workgroups per round (0: not announced)
  int wg_chunks = 1;    // kernel chunks per workgroup at most for co-located workers (0: no cap)
  bool coarsen = true;  // full-threshold rounds may run multiples of maxChunkSize
  std::string handle;   // raw IPC handle bytes
};
PlaneDesc parse_plane_desc(const std::string& s);

struct PlaneGeometry {
  int64_t block = 0;   // elements per block: ceil(dataSize / P) in float32
  int64_t chunk = 0;   // kernel chunk (elements): maxChunkSize x coarse
  int nch = 0;         // kernel chunks per block
  int nch_ref = 0;     // reference chunks per block: ceil(block / maxChunkSize)
  int coarse = 1;      // reference chunks per kernel chunk
  bool coarsened_for_flags = false;  // maxChunkSize finer than the flag table (thresholds 1)
  int colocation = 1;  // most workers of the job in one process on one device
  int grid = 0;        // the job-wide grid the coarsening used (smallest announced)
};

// flag_maxch: kernel chunks per block the arena's flag table holds (XgmiComm::layout().maxch);
// es: element size. Throws ProtocolError where the reference semantics cannot be kept
// (maxChunkSize finer than the flag table at thresholds < 1).
PlaneGeometry plane_geometry(const PlaneConfig& cfg, int64_t flag_maxch, int64_t es);

}  // namespace mxar
