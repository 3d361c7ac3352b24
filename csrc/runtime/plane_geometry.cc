#include "plane_geometry.h"

#include <algorithm>
#include <sstream>

#include "../core/data_buffer.h"
#include "../core/protocol.h"

namespace mxar {

namespace {
int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

std::string from_hex(const std::string& h) {
  std::string out;
  out.reserve(h.size() / 2);
  for (size_t i = 0; i + 1 < h.size(); i += 2) out.push_back(static_cast<char>(std::stoi(h.substr(i, 2), nullptr, 16)));
  return out;
}
}  // namespace

PlaneDesc parse_plane_desc(const std::string& s) {
  std::istringstream is(s);
  std::string tag;
  is >> tag;
  if (tag != "xgmi1") throw ProtocolError("not an xGMI plane descriptor: '" + s.substr(0, 40) + "'");
  PlaneDesc d;
  std::string kv;
  while (is >> kv) {
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    const std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
    if (k == "pid") d.pid = std::stol(v);
    else if (k == "dev") d.device = std::stoi(v);
    else if (k == "bytes") d.bytes = std::stoll(v);
    else if (k == "id") d.id = std::stoull(v);
    else if (k == "grid") d.grid = std::stoi(v);
    else if (k == "wgc") d.wg_chunks = std::stoi(v);
    else if (k == "coarsen") d.coarsen = std::stoi(v) != 0;
    else if (k == "h") d.handle = from_hex(v);
  }
  return d;
}

PlaneGeometry plane_geometry(const PlaneConfig& cfg, int64_t flag_maxch, int64_t es) {
  PlaneGeometry g;
  const int P = cfg.peers;
  if (P <= 0 || cfg.maxChunkSize <= 0) throw ProtocolError("plane geometry: peers and maxChunkSize must be > 0");
  // job-wide knobs: the smallest announced grid / cap, coarsening only if every plane allows it,
  // and the largest co-location of any (process, device) of the membership
  int grid = 0, wgc = 1 << 30;
  bool coarsen = true;
  std::map<std::pair<long, int>, int> places;
  for (int k = 0; k < P; ++k) {
    auto it = cfg.descriptors.find(k);
    if (it == cfg.descriptors.end() || it->second.empty()) continue;
    const PlaneDesc d = parse_plane_desc(it->second);
    if (d.grid > 0) grid = grid == 0 ? d.grid : std::min(grid, d.grid);
    wgc = std::min(wgc, d.wg_chunks);
    coarsen = coarsen && d.coarsen;
    g.colocation = std::max(g.colocation, ++places[{d.pid, d.device}]);
  }
  if (grid <= 0) grid = 512;
  if (wgc == (1 << 30)) wgc = 1;
  g.grid = grid;
  // the reference's geometry: blocks of step = ceil(N / P) (float32 division,
  // AllreduceWorker.scala:211-214), chunks of maxChunkSize elements (:56-57)
  g.block = static_cast<int64_t>(f32_ceil_div(cfg.dataSize, P));
  g.chunk = cfg.maxChunkSize;
  int64_t nch = std::max<int64_t>(1, ceil_div(g.block, g.chunk));
  g.nch_ref = static_cast<int>(nch);
  if (nch > flag_maxch) {
    // More reference chunks than the flag table holds (maxChunkSize below the plane's flag
    // granularity). At thresholds 1 every contribution and every chunk is taken whatever the
    // granularity, so the kernel runs whole multiples of maxChunkSize and the counts are
    // reported per reference chunk. Below 1 the threshold decisions ARE per reference chunk
    // (DataBuffer.scala:28-29,69-75): coarser units would change which data a round keeps.
    if (cfg.thReduce < 1.f || cfg.thComplete < 1.f)
      throw ProtocolError("maxChunkSize " + std::to_string(cfg.maxChunkSize) + " at thReduce " +
                          std::to_string(cfg.thReduce) + " / thComplete " + std::to_string(cfg.thComplete) +
                          " needs one flag per chunk: build the plane with min_chunk <= " +
                          std::to_string(cfg.maxChunkSize) + " (PlaneJob(min_chunk=...), mxar.plane.min_chunk)");
    const int64_t m = ceil_div(nch, flag_maxch);
    g.chunk *= m;
    g.coarse = static_cast<int>(m);
    nch = ceil_div(g.block, g.chunk);
    g.coarsened_for_flags = true;
  }
  // Full thresholds: every contribution and every chunk is taken whatever the chunking, so the
  // kernel may also run whole multiples of maxChunkSize for speed (counts still reported per
  // reference chunk). Every kernel chunk costs a flag hand-off and a release per hop, so 2 KiB
  // chunks spend more time on hand-offs than on bytes: kernel chunks of >= 32 KiB, while
  // every fourth workgroup still gets a reduce unit. Same-box A/B (plane_probe --units):
  // 8 workers x 16 MiB, 8 -> 32 KiB chunks 0.350 / 0.358 -> 0.307 / 0.272 ms per round; 2 x 1 MiB,
  // 2 -> 8 KiB 0.069 / 0.057 -> 0.061 / 0.049 ms. MXAR_PLANE_COARSEN=0 keeps maxChunkSize.
  if (cfg.thReduce >= 1.f && cfg.thComplete >= 1.f && coarsen) {
    const int64_t want = ceil_div(int64_t{32} << 10, g.chunk * es);
    const int64_t room = std::max<int64_t>(1, nch / std::max(1, grid / 4));
    // ...and, when any workers of the job share one group kernel, at most one kernel chunk per
    // workgroup: a workgroup that reduces two chunks pays the second chunk's hand-offs after the
    // first one's, on the round's critical path. 2 co-located workers x 128 workgroups, bf16
    // (profiles/round5/protocol_grid_chunk.jsonl): 64 MiB 159-164 -> 145-149 us per round,
    // 16 MiB 86-95 -> 74-75, 256 MiB 441-474 -> 426-454. The condition is the JOB's largest
    // co-location, not this worker's: a lone worker of a mixed placement chunks like its
    // co-located peers (their slots and flags are laid out by the same chunk).
    int64_t m = std::min(want, room);
    if (wgc > 0 && g.colocation > 1) m = std::max(m, ceil_div(nch, static_cast<int64_t>(std::max(1, grid)) * wgc));
    // a block of at most 32 KiB is ONE kernel chunk: one hand-off per peer instead of one per
    // chunk (the reference's default job, 10 floats in 2-float chunks: 3 chunks per block -> 1)
    if (g.block * es <= (int64_t{32} << 10)) m = nch;
    if (m > 1) {
      g.chunk *= m;
      g.coarse *= static_cast<int>(m);
      nch = ceil_div(g.block, g.chunk);
    }
  }
  g.nch = static_cast<int>(nch);
  return g;
}

}  // namespace mxar
