// Tile packing of the HBM token stream: see tiles.h.
#include "tiles.h"

#include <algorithm>
#include <cstring>
#include <thread>

#include "common.h"

namespace shred {

size_t layout_entries(const WordTable& wt, Layout layout) {
  return layout == Layout::kStream ? wt.occurrence_rank.size() : wt.num_words();
}

void shard_range(const WordTable& wt, Layout layout, int rank, int world, size_t* begin, size_t* end) {
  const bool stream = layout == Layout::kStream;
  const size_t n = layout_entries(wt, layout);
  if (world <= 1) {
    *begin = 0;
    *end = n;
    return;
  }
  std::vector<uint64_t> prefix(n + 1, 0);
  for (size_t e = 0; e < n; ++e) {
    const uint32_t r = stream ? wt.occurrence_rank[e] : (uint32_t)e;
    prefix[e + 1] = prefix[e] + (wt.offset[r + 1] - wt.offset[r]) + 1;
  }
  auto cut = [&](int k) -> size_t {
    if (k <= 0) return 0;
    if (k >= world) return n;
    const uint64_t target = (uint64_t)((long double)prefix.back() * k / world);
    return (size_t)(std::lower_bound(prefix.begin(), prefix.end(), target) - prefix.begin());
  };
  *begin = std::min(cut(rank), n);
  *end = std::min(cut(rank + 1), n);
}

void pack_tiles(const WordTable& wt, Layout layout, size_t begin, size_t end, TiledStream* out) {
  const bool stream = layout == Layout::kStream;
  const size_t nent = layout_entries(wt, layout);
  if (stream && nent == 0 && wt.total_occurrences > 0) fatal("stream layout requested without occurrence ranks");
  end = std::min(end, nent);
  begin = std::min(begin, end);
  auto rank_of = [&](size_t e) -> uint32_t { return stream ? wt.occurrence_rank[e] : (uint32_t)e; };
  auto len_of = [&](uint32_t r) -> uint64_t { return wt.offset[r + 1] - wt.offset[r]; };

  TiledStream& ts = *out;
  ts = TiledStream();
  std::vector<size_t> first;
  uint64_t pos = 0, fill = 0;
  for (size_t e = begin; e < end; ++e) {
    const uint64_t need = len_of(rank_of(e)) + 1;
    if (need >= (1ull << 31)) fatal("word longer than 2^31 tokens");
    if (fill > 0 && fill + need > (uint64_t)kTileTokens) {
      ts.len.push_back((uint32_t)fill);
      pos += (fill + 3) & ~3ull;
      fill = 0;
    }
    if (fill == 0) {
      ts.off.push_back(pos);
      first.push_back(e);
    }
    fill += need;
  }
  if (fill > 0) {
    ts.len.push_back((uint32_t)fill);
    pos += (fill + 3) & ~3ull;
  }
  first.push_back(end);
  ts.elems = pos;
  ts.entries = end - begin;
  ts.tok.assign(pos + 4, kHeaderBase);
  const size_t nt = ts.len.size();
  auto fill_tiles = [&](size_t t0, size_t t1) {
    for (size_t t = t0; t < t1; ++t) {
      int32_t* dst = ts.tok.data() + ts.off[t];
      for (size_t e = first[t]; e < first[t + 1]; ++e) {
        const uint32_t r = rank_of(e);
        *dst++ = (int32_t)((uint32_t)kHeaderBase + r);
        const uint64_t o = wt.offset[r], l = len_of(r);
        std::memcpy(dst, wt.symbols.data() + o, l * sizeof(int32_t));
        dst += l;
      }
    }
  };
  const int threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (nt < 4096 || threads == 1) {
    fill_tiles(0, nt);
  } else {
    std::vector<std::thread> pool;
    for (int k = 0; k < threads; ++k)
      pool.emplace_back(fill_tiles, nt * k / threads, nt * (k + 1) / threads);
    for (auto& th : pool) th.join();
  }
  for (uint32_t l : ts.len) ts.live += l;
}

}  // namespace shred
