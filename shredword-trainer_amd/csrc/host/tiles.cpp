// Tile packing of the HBM token stream: see tiles.h.
#include "tiles.h"

#include <algorithm>
#include <cstring>
#include <functional>
#include <iterator>
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
  const size_t n = end - begin;
  // Stream layout: the first occurrence of every word type in [begin, end) is packed first, in
  // corpus order, and that block ends on a tile boundary (ft_tiles); the other occurrences follow
  // in corpus order.  Pair counts and merges are sums over occurrences (order-free), and every
  // occurrence of a type has the same first touch (rank, position), so K1 takes first touch from
  // the ft tiles alone and the bulk of the stream only has to be counted.
  std::vector<uint32_t> order;
  size_t nfirst = n;
  if (stream && n > 0) {
    order.resize(n);
    std::vector<uint8_t> seen(wt.num_words(), 0);
    size_t k = 0;
    for (size_t e = begin; e < end; ++e) {
      const uint32_t r = wt.occurrence_rank[e];
      if (!seen[r]) {
        seen[r] = 1;
        order[k++] = r;
      }
    }
    nfirst = k;
    std::fill(seen.begin(), seen.end(), 0);
    for (size_t e = begin; e < end; ++e) {
      const uint32_t r = wt.occurrence_rank[e];
      if (!seen[r]) {
        seen[r] = 1;
        continue;
      }
      order[k++] = r;
    }
  }
  auto rank_of = [&](size_t i) -> uint32_t { return stream ? order[i] : (uint32_t)(begin + i); };
  auto len_of = [&](uint32_t r) -> uint64_t { return wt.offset[r + 1] - wt.offset[r]; };

  TiledStream& ts = *out;
  ts = TiledStream();
  std::vector<size_t> first;
  uint64_t pos = 0, fill = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t need = len_of(rank_of(i)) + 1;
    if (need >= (1ull << 31)) fatal("word longer than 2^31 tokens");
    if (fill > 0 && (fill + need > (uint64_t)kTileTokens || i == nfirst)) {
      ts.len.push_back((uint32_t)fill);
      pos += (fill + 3) & ~3ull;
      fill = 0;
    }
    if (i == nfirst) ts.ft_tiles = ts.len.size();
    if (fill == 0) {
      ts.off.push_back(pos);
      first.push_back(i);
    }
    fill += need;
  }
  if (fill > 0) {
    ts.len.push_back((uint32_t)fill);
    pos += (fill + 3) & ~3ull;
  }
  if (nfirst == n) ts.ft_tiles = ts.len.size();
  first.push_back(n);
  ts.elems = pos;
  ts.entries = end - begin;
  ts.tok.assign(pos + 4, kHeaderBase);
  const size_t nt = ts.len.size();
  auto fill_tiles = [&](size_t t0, size_t t1) {
    for (size_t t = t0; t < t1; ++t) {
      int32_t* dst = ts.tok.data() + ts.off[t];
      for (size_t i = first[t]; i < first[t + 1]; ++i) {
        const uint32_t r = rank_of(i);
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

namespace shred {

void TileIndex::make(Set* s, std::vector<uint32_t>&& sorted) const {
  s->size = sorted.size();
  s->list.clear();
  s->bits.clear();
  if ((uint64_t)sorted.size() * 32 > ntiles_) {  // a bitmap is smaller
    s->bits.assign((ntiles_ + 63) / 64, 0);
    for (uint32_t t : sorted) s->bits[t >> 6] |= 1ull << (t & 63);
  } else {
    s->list = std::move(sorted);
  }
}

void TileIndex::build(const TiledStream& ts) {
  ntiles_ = (uint32_t)ts.num_tiles();
  // Threads over contiguous tile ranges; each lists (key, tile) once per tile where the key occurs,
  // in tile order, and a counting pass per key concatenates the ranges in order, so every key's
  // tile list comes out sorted without a sort (C5 at 100 GB: 70 M tokens in 68,905 tiles).
  //   ids: key = the token id (>= 0); pairs: key = x * 256 + y for adjacent ids x, y < 256
  const size_t T = ntiles_;
  const int P = (int)std::max<size_t>(1, std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()),
                                                          T / 64 + 1}));
  auto par = [&](const std::function<void(int)>& f) {
    if (P == 1) return f(0);
    std::vector<std::thread> pool;
    for (int k = 0; k < P; ++k) pool.emplace_back(f, k);
    for (auto& th : pool) th.join();
  };
  struct Part {
    std::vector<uint64_t> ids, pairs;  // key << 32 | tile, in tile order
    std::vector<uint32_t> nid, npair;  // entries per key
  };
  std::vector<Part> part((size_t)P);
  par([&](int k) {
    Part& pt = part[(size_t)k];
    const size_t t0 = T * (size_t)k / (size_t)P, t1 = T * (size_t)(k + 1) / (size_t)P;
    std::vector<uint32_t> seen(256, UINT32_MAX), last(256 * 256, UINT32_MAX);
    pt.nid.assign(256, 0);
    pt.npair.assign(256 * 256, 0);
    for (size_t t = t0; t < t1; ++t) {
      const int32_t* p = ts.tok.data() + ts.off[t];
      const uint32_t len = ts.len[t];
      for (uint32_t i = 0; i < len; ++i) {
        const int32_t id = p[i];
        if (id < 0) continue;  // headers, negative unk
        if ((size_t)id >= seen.size()) {
          seen.resize((size_t)id + 1, UINT32_MAX);
          pt.nid.resize((size_t)id + 1, 0);
        }
        if (seen[id] != (uint32_t)t) {
          seen[id] = (uint32_t)t;
          pt.ids.push_back((uint64_t)id << 32 | t);
          ++pt.nid[id];
        }
        if (i + 1 < len) {
          const uint32_t x = (uint32_t)id, y = (uint32_t)p[i + 1];
          if (x >= 256 || y >= 256) continue;  // headers, unk outside the byte range, merged ids
          const uint32_t key = x * 256 + y;
          if (last[key] != (uint32_t)t) {
            last[key] = (uint32_t)t;
            pt.pairs.push_back((uint64_t)key << 32 | t);
            ++pt.npair[key];
          }
        }
      }
    }
  });
  size_t nids = 256;
  for (const Part& pt : part) nids = std::max(nids, pt.nid.size());
  // per key: the ranges' entries back to back, range by range (so in tile order); then one Set each
  auto gather = [&](size_t nkeys, std::vector<uint64_t> Part::*ent, std::vector<uint32_t> Part::*num,
                    std::vector<Set>* out) {
    std::vector<uint64_t> at((size_t)P * nkeys);  // [part][key]: where the part's entries of key go
    std::vector<uint64_t> off(nkeys + 1, 0);
    uint64_t run = 0;
    for (size_t key = 0; key < nkeys; ++key) {
      off[key] = run;
      for (int k = 0; k < P; ++k) {
        const std::vector<uint32_t>& n = part[(size_t)k].*num;
        at[(size_t)k * nkeys + key] = run;
        run += key < n.size() ? n[key] : 0;
      }
    }
    off[nkeys] = run;
    std::vector<uint32_t> flat(run);
    par([&](int k) {
      uint64_t* a = at.data() + (size_t)k * nkeys;
      for (uint64_t e : part[(size_t)k].*ent) flat[a[(size_t)(e >> 32)]++] = (uint32_t)e;
    });
    out->assign(nkeys, Set());
    par([&](int k) {
      for (size_t key = nkeys * (size_t)k / (size_t)P; key < nkeys * (size_t)(k + 1) / (size_t)P; ++key)
        if (off[key + 1] > off[key])
          make(&(*out)[key], std::vector<uint32_t>(flat.begin() + (long)off[key], flat.begin() + (long)off[key + 1]));
    });
  };
  gather(nids, &Part::ids, &Part::nid, &ids_);
  ids0_ = ids_;
  gather(256 * 256, &Part::pairs, &Part::npair, &base_pairs_);
}

void TileIndex::reset() { ids_ = ids0_; }

void TileIndex::set_tiles(int32_t id, const uint32_t* tiles, size_t n) {
  if (id < 0) return;
  if ((size_t)id >= ids_.size()) ids_.resize(id + 1);
  std::vector<uint32_t> v(tiles, tiles + n);
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  make(&ids_[id], std::move(v));
}

void TileIndex::set_tiles_bits(int32_t id, const uint32_t* words, size_t n) {
  if (id < 0) return;
  if ((size_t)id >= ids_.size()) ids_.resize(id + 1);
  Set& s = ids_[id];
  s.size = n;
  s.list.clear();
  s.bits.clear();
  const size_t nw = (ntiles_ + 31) / 32;
  if ((uint64_t)n * 32 > ntiles_) {  // dense: the bitmap as is (two u32 words per u64, low first)
    s.bits.assign((ntiles_ + 63) / 64, 0);
    size_t pop = 0;  // the set's size is the bitmap's popcount, not the caller's entry count
    for (size_t w = 0; w < nw; ++w) {
      s.bits[w >> 1] |= (uint64_t)words[w] << (32 * (w & 1));
      pop += (size_t)__builtin_popcount(words[w]);
    }
    s.size = pop;
  } else {
    s.list.reserve(n);
    for (size_t w = 0; w < nw; ++w)
      for (uint32_t m = words[w]; m; m &= m - 1) s.list.push_back((uint32_t)(w * 32 + __builtin_ctz(m)));
    s.size = s.list.size();
  }
}

void TileIndex::set_all(int32_t id) {
  if (id < 0) return;
  if ((size_t)id >= ids_.size()) ids_.resize(id + 1);
  Set& s = ids_[id];
  s.list.clear();
  s.bits.assign((ntiles_ + 63) / 64, ~0ull);
  if (ntiles_ & 63) s.bits.back() = (1ull << (ntiles_ & 63)) - 1;
  s.size = ntiles_;
}

bool TileIndex::candidates(int32_t a, int32_t b, std::vector<uint32_t>* out) const {
  out->clear();
  const size_t limit = ntiles_ / 2;  // beyond this a full scan is as cheap
  if ((uint32_t)a < 256 && (uint32_t)b < 256 && !base_pairs_.empty()) {
    const Set& s = base_pairs_[(uint32_t)a * 256 + (uint32_t)b];
    if (s.size == 0 || s.size > limit) return false;
    if (!s.list.empty()) {
      *out = s.list;
    } else {
      for (size_t w = 0; w < s.bits.size(); ++w)
        for (uint64_t m = s.bits[w]; m; m &= m - 1) out->push_back((uint32_t)(w * 64 + __builtin_ctzll(m)));
    }
    return true;
  }
  const Set* sa = get(a);
  const Set* sb = get(b);
  if (!sa || !sb) return false;  // unknown id: be safe, scan everything
  return intersect(sa, sb, out) && out->size() <= limit;
}

bool TileIndex::intersect(const Set* sa, const Set* sb, std::vector<uint32_t>* out) const {
  if (sa->size > sb->size) std::swap(sa, sb);
  const size_t limit = ntiles_ / 2;
  if (sa->size > limit || sa->size == 0) return false;
  if (!sa->list.empty()) {
    if (!sb->bits.empty()) {
      for (uint32_t t : sa->list)
        if ((sb->bits[t >> 6] >> (t & 63)) & 1) out->push_back(t);
    } else {
      std::set_intersection(sa->list.begin(), sa->list.end(), sb->list.begin(), sb->list.end(),
                            std::back_inserter(*out));
    }
  } else {  // both dense
    for (size_t w = 0; w < sa->bits.size(); ++w) {
      uint64_t m = sa->bits[w] & sb->bits[w];
      while (m) {
        out->push_back((uint32_t)(w * 64 + __builtin_ctzll(m)));
        m &= m - 1;
      }
    }
  }
  return !out->empty();
}

void TileIndex::to_bits(const Set* s, std::vector<uint64_t>* bits) const {
  const size_t nw = (ntiles_ + 63) / 64;
  if (!s->bits.empty()) {
    *bits = s->bits;
    return;
  }
  bits->assign(nw, 0);
  for (uint32_t t : s->list) (*bits)[t >> 6] |= 1ull << (t & 63);
}

void TileIndex::owners(int32_t a, int32_t b, const std::vector<uint32_t>& first, std::vector<uint32_t>* out) const {
  out->clear();
  const size_t W = first.size() - 1;
  const size_t nw = (ntiles_ + 63) / 64;
  const Set* sa = nullptr;
  const Set* sb = nullptr;
  if ((uint32_t)a < 256 && (uint32_t)b < 256 && !base_pairs_.empty()) {
    sa = &base_pairs_[(uint32_t)a * 256 + (uint32_t)b];  // exact tiles of a pair of bytes
  } else {
    sa = get(a);
    sb = get(b);
  }
  if (!sa || (sb == nullptr && !((uint32_t)a < 256 && (uint32_t)b < 256 && !base_pairs_.empty()))) {
    for (size_t w = 0; w < W; ++w)  // unknown id: every owner
      if (first[w + 1] > first[w]) out->push_back((uint32_t)w);
    return;
  }
  to_bits(sa, &ba_);
  if (sb) {
    to_bits(sb, &bb_);
    for (size_t i = 0; i < nw; ++i) ba_[i] &= bb_[i];
  }
  for (size_t w = 0; w < W; ++w) {
    const uint32_t lo = first[w], hi = first[w + 1];  // [lo, hi)
    if (lo >= hi) continue;
    bool any = false;
    for (uint32_t i = lo >> 6; i <= (hi - 1) >> 6 && !any; ++i) {
      uint64_t m = ba_[i];
      if (i == lo >> 6) m &= ~0ull << (lo & 63);
      if (i == (hi - 1) >> 6 && ((hi - 1) & 63) != 63) m &= (2ull << ((hi - 1) & 63)) - 1;
      any = m != 0;
    }
    if (any) out->push_back((uint32_t)w);
  }
}

}  // namespace shred
