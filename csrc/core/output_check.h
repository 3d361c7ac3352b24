// Consistency check of one round output against its per-chunk counts when every worker's
// source holds a distinct power of two everywhere (the straggler bench's sources): chunk c of
// block j must hold ONE value v everywhere, v an integer whose set bits name the contributors,
// and popcount(v) must equal the chunk's count (0: zeros). Any torn, mixed or double-counted
// chunk fails - the outputs equal the counted sums (AllReduceOutput.count).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "data_buffer.h"

namespace mxar {

struct OutputCheck {
  bool ok = true;
  int64_t chunks = 0, bad_chunks = 0, count_sum = 0;
  // the first bad chunk: block, chunk, its count, the value at its first element and the
  // number of distinct values in it
  int first_block = -1, first_chunk = -1, first_count = 0, first_distinct = 0;
  float first_value = 0.f;
};

inline OutputCheck check_power_of_two_output(const std::vector<float>& data, const std::vector<int>& count,
                                             int peers, int max_chunk) {
  OutputCheck r;
  const int n = static_cast<int>(data.size());
  if (peers <= 0 || max_chunk <= 0 || count.empty() || count.size() % static_cast<size_t>(peers) != 0) {
    r.ok = false;
    return r;
  }
  const BlockLayout lay(n, peers, max_chunk);
  const int nch = static_cast<int>(count.size() / static_cast<size_t>(peers));
  for (int j = 0; j < peers; ++j) {
    for (int c = 0; c < nch; ++c) {
      const int lo = lay.start[j] + c * max_chunk;
      const int hi = std::min(lay.end[j], lo + max_chunk);
      if (lo >= hi) continue;
      const int cnt = count[static_cast<size_t>(j) * nch + c];
      ++r.chunks;
      r.count_sum += cnt;
      const float v = data[lo];
      bool good = v >= 0.f && v == std::floor(v) && v < 4294967296.f &&
                  __builtin_popcountll(static_cast<uint64_t>(v)) == cnt;
      for (int i = lo + 1; good && i < hi; ++i) good = data[i] == v;
      if (!good) {
        if (r.bad_chunks == 0) {
          r.first_block = j, r.first_chunk = c, r.first_count = cnt, r.first_value = v;
          std::vector<float> seen;
          for (int i = lo; i < hi && seen.size() < 8; ++i)
            if (std::find(seen.begin(), seen.end(), data[i]) == seen.end()) seen.push_back(data[i]);
          r.first_distinct = static_cast<int>(seen.size());
        }
        ++r.bad_chunks;
        r.ok = false;
      }
    }
  }
  return r;
}

}  // namespace mxar
