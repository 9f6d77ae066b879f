// Exact merge selection: see selector.h for the rules and reference citations.
#include "selector.h"

#include <immintrin.h>

#include <algorithm>
#include <cstring>

#include "common.h"

namespace shred {

namespace {
// First touch descending for one bucket's changes (the reference applies a bucket's chain head
// first: the latest first touch).  Buckets above a few entries (a merge's (p, a) and (p, X)
// changes share a's and X's buckets: about a quarter of its changes each) are radix-sorted on the
// bits of ft that vary inside the bucket (pext), inverted, with the change's index below them --
// no compare branches; first touches are distinct, so the order is the comparison sort's.
__attribute__((target("bmi2"))) bool sort_ft_desc_radix(Selector::Change* c, size_t m, std::vector<uint64_t>& ka,
                                                        std::vector<uint64_t>& kb, std::vector<Selector::Change>& tmp) {
  uint64_t orv = 0, andv = ~0ull;
  for (size_t i = 0; i < m; ++i) {
    orv |= c[i].ft;
    andv &= c[i].ft;
  }
  const uint64_t live = orv & ~andv;
  const int bits = __builtin_popcountll(live);
  const int ib = 64 - __builtin_clzll((uint64_t)m);
  if (bits + ib > 64) return false;
  const uint64_t fm = bits == 64 ? ~0ull : (1ull << bits) - 1;
  ka.resize(m);
  kb.resize(m);
  for (size_t i = 0; i < m; ++i) ka[i] = ((~_pext_u64(c[i].ft, live) & fm) << ib) | i;
  uint64_t* src = ka.data();
  uint64_t* dst = kb.data();
  for (int sh = ib; sh < ib + bits; sh += 8) {
    uint32_t cnt[257];
    std::memset(cnt, 0, sizeof cnt);
    for (size_t i = 0; i < m; ++i) cnt[((src[i] >> sh) & 255u) + 1]++;
    for (int k = 0; k < 256; ++k) cnt[k + 1] += cnt[k];
    for (size_t i = 0; i < m; ++i) dst[cnt[(src[i] >> sh) & 255u]++] = src[i];
    std::swap(src, dst);
  }
  tmp.assign(c, c + m);
  const uint64_t im = (1ull << ib) - 1;
  for (size_t i = 0; i < m; ++i) c[i] = tmp[src[i] & im];
  return true;
}
const bool kHaveBmi2 = __builtin_cpu_supports("bmi2");
}  // namespace

namespace {
inline uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  k *= 0xC4CEB9FE1A85EC53ull;
  k ^= k >> 33;
  return k;
}
}  // namespace

void Selector::reset(int32_t unk_id, uint64_t min_pair_freq) {
  unk_ = unk_id;
  min_freq_ = min_pair_freq;
  ctr_ = Counters();
  // at least 1 M slots (16 MB: no rehash below 512 k pairs), and as many as the previous
  // training grew to: a repeated train() (benchmarks, sweeps) rehashes nothing and reuses the
  // mapped pages (a 4 M -> 16 M slot grow costs ~12 ms mid-training at C3)
  const size_t want = std::max<size_t>(size_t(1) << 20, table_.size());
  table_.assign(want, Info{kEmptyKey, 0});
  created_.clear();
  mask_ = table_.size() - 1;
  count_ = 0;
  heap_.assign(1, HeapNode{0, 0, 0});
  exact_ = true;  // an empty map and an empty heap: nothing is popped before a count
  truth_live_ = false;
  truth_.clear();
}

void Selector::reset_info() {
  std::fill(table_.begin(), table_.end(), Info{kEmptyKey, 0});
  created_.clear();
  count_ = 0;
  exact_ = false;  // the kept heap's entries meet a map that has not counted the new corpus
  truth_live_ = false;
  truth_.clear();
}

void Selector::set_truth(const std::vector<PairCount>& pairs) {
  truth_.clear();
  truth_.reserve(pairs.size() * 2);
  for (const PairCount& p : pairs)
    if (p.a != unk_ && p.b != unk_) truth_[pack_pair(p.a, p.b)] = p.count;
  truth_live_ = true;
}

uint64_t Selector::recount(int32_t a, int32_t b) const {
  if (a == unk_ || b == unk_) return 0;  // bpe.cpp:53
  if (!truth_live_) fatal("Selector: a rescan without the truth table");
  const auto it = truth_.find(pack_pair(a, b));
  return it == truth_.end() ? 0 : it->second;
}

void Selector::grow() {
  HugeVec<Info> old(table_.size() * 4, Info{kEmptyKey, 0});
  old.swap(table_);
  mask_ = table_.size() - 1;
  for (size_t i = 0; i < old.size(); ++i) {
    const Info& in = old[i];
    if (in.key == kEmptyKey) continue;
    uint64_t j = mix64(in.key) & mask_;
    while (table_[j].key != kEmptyKey) j = (j + 1) & mask_;
    table_[j] = in;
  }
}

void Selector::info_overflow() { fatal("pair info field overflow (pair count >= 2^40 or version >= 2^24)"); }

Selector::Info& Selector::get(int32_t a, int32_t b) {
  const uint64_t key = pack_pair(a, b);
  uint64_t j = mix64(key) & mask_;
  for (;;) {
    Info& in = table_[j];
    if (in.key == key) return in;
    if (in.key == kEmptyKey) break;
    j = (j + 1) & mask_;
  }
  if (2 * (count_ + 1) > table_.size()) {
    grow();
    j = mix64(key) & mask_;
    while (table_[j].key != kEmptyKey) j = (j + 1) & mask_;
  }
  table_[j] = Info{key, 0};
  created_.push_back(key);
  ++count_;
  return table_[j];
}

const Selector::Info* Selector::find(uint64_t key) const {
  uint64_t j = mix64(key) & mask_;
  for (;;) {
    const Info& in = table_[j];
    if (in.key == key) return &in;
    if (in.key == kEmptyKey) return nullptr;
    j = (j + 1) & mask_;
  }
}

size_t Selector::exact_mismatches(const std::vector<PairCount>& fresh) const {
  size_t bad = 0, seen = 0;
  for (const PairCount& p : fresh) {
    if (p.a == unk_ || p.b == unk_) continue;
    const Info* in = find(pack_pair(p.a, p.b));
    bad += !in || in->freq() != p.count;
    ++seen;
  }
  size_t live = 0;  // infos with a count, unk pairs aside: exactly the fresh count's pairs
  for (size_t j = 0; j < table_.size(); ++j) {
    const Info& in = table_[j];
    if (in.key == kEmptyKey || in.freq() == 0) continue;
    if (pair_first(in.key) == unk_ || pair_second(in.key) == unk_) continue;
    ++live;
  }
  return bad + (live > seen ? live - seen : 0);
}

bool Selector::lookup(int32_t a, int32_t b, uint64_t* freq, uint32_t* version) const {
  const Info* in = find(pack_pair(a, b));
  *freq = in ? in->freq() : 0;
  *version = in ? in->version() : 0;
  return in != nullptr;
}

void Selector::push(int32_t a, int32_t b, uint64_t freq, uint32_t version) {
  ++ctr_.pushes;
  if (freq >> 40 || version >> 24) fatal("heap node field overflow (pair count >= 2^40 or version >= 2^24)");
  HeapNode* h = heap_.data();
  heap_.push_back(HeapNode{0, 0, 0});
  h = heap_.data();
  size_t i = heap_.size() - 2;  // logical slot of the new node
  while (i > 0) {
    size_t p = (i - 1) >> 1;
    if (node_freq(h[p + 1]) >= freq) break;  // sift up only while parent < child (heap.cpp:76)
    h[i + 1] = h[p + 1];
    i = p;
  }
  h[i + 1] = HeapNode{freq << 24 | version, a, b};
}

Selector::HeapEnt Selector::pop() {
  ++ctr_.pops;
  HeapNode* h = heap_.data();
  const HeapEnt top{h[1].a, h[1].b, node_freq(h[1]), node_version(h[1])};
  const HeapNode x = heap_.back();
  heap_.pop_back();
  const size_t n = heap_.size() - 1;
  if (n == 0) return top;
  const uint64_t xf = node_freq(x);
  size_t i = 0;
  // The reference's sift-down (heap.cpp:101-106): left child if strictly greater than x, then
  // right if strictly greater than that.  With both children present this is "the larger
  // child, left on a tie, while it is strictly greater than x", so the child is chosen without
  // a branch (the choice is a coin flip to the predictor); only the stop test branches, and it
  // almost always goes the same way.
  while (2 * i + 2 < n) {
    const size_t l = 2 * i + 1;
    if (4 * i + 3 < n) __builtin_prefetch(h + 4 * i + 4);  // the four grandchildren: one line
    if (8 * i + 7 < n) {                                  // their eight children: two lines
      __builtin_prefetch(h + 8 * i + 8);
      __builtin_prefetch(h + 8 * i + 12);
    }
    if (16 * i + 15 < n) {  // and their sixteen: four lines
      __builtin_prefetch(h + 16 * i + 16);
      __builtin_prefetch(h + 16 * i + 20);
      __builtin_prefetch(h + 16 * i + 24);
      __builtin_prefetch(h + 16 * i + 28);
    }
    const uint64_t lf = node_freq(h[l + 1]), rf = node_freq(h[l + 2]);
    const bool right = rf > lf;
    const size_t c = l + right;
    if ((right ? rf : lf) <= xf) break;
    h[i + 1] = h[c + 1];
    i = c;
  }
  if (2 * i + 2 == n && node_freq(h[2 * i + 2]) > xf) {  // a lone left child (the last slot)
    h[i + 1] = h[2 * i + 2];
    i = 2 * i + 1;
  }
  h[i + 1] = x;
  return top;
}

void Selector::add_counts(std::vector<PairCount> pairs) {
  // A count on a map that already holds pairs adds to them (bpe.cpp:206-211): the map is then
  // no longer the corpus's count.  On a fresh map it is exactly the count.
  if (count_ != 0 && !pairs.empty()) exact_ = false;
  else if (count_ == 0) exact_ = true;
  // bimap_get is reached in (word rank, position) order, so that is creation order.
  std::sort(pairs.begin(), pairs.end(), [](const PairCount& x, const PairCount& y) { return x.ft < y.ft; });
  for (const PairCount& p : pairs) {
    Info& in = get(p.a, p.b);
    if (in.freq() == 0) in.set_version(0);  // bpe.cpp:207-210
    in.set_freq(in.freq() + p.count);
  }
  // Heap build: bucket 0..4095, chain (creation) order, freq >= min (bpe.cpp:218-225), over every
  // pair of the map (those the merges created included).
  std::vector<std::pair<uint64_t, uint64_t>> order;  // ((bucket << 32) | creation, key)
  order.reserve(created_.size());
  for (size_t c = 0; c < created_.size(); ++c) {
    const uint64_t key = created_[c];
    const Info* in = find(key);
    if (in && in->freq() >= min_freq_) {
      const uint32_t bk = pair_fnv(pair_first(key), pair_second(key)) & (kPairBuckets - 1);
      order.push_back({((uint64_t)bk << 32) | c, key});
    }
  }
  std::sort(order.begin(), order.end());
  for (auto& o : order) {
    const Info* in = find(o.second);
    push(pair_first(o.second), pair_second(o.second), in->freq(), in->version());
  }
}

bool Selector::predict_next(int32_t a, int32_t b, size_t window, int32_t* pa, int32_t* pb) const {
  const int32_t used[2] = {a, b};
  return predict_avoid(used, 2, window, pa, pb);
}

bool Selector::predict_avoid(const int32_t* used, size_t n_used, size_t window, int32_t* pa, int32_t* pb) const {
  // The best valid entry sharing no token with `used` among the first `window` heap slots, by a
  // walk from the root that skips every subtree whose root is below the best found so far (the
  // heap property bounds the whole subtree), so it touches a handful of entries.  Ties: the
  // lowest heap slot, as a scan in slot order would pick.
  const size_t n = std::min(window, heap_size());
  const HeapNode* h = heap_.data() + 1;  // logical slots
  uint64_t best_f = 0;
  size_t best = SIZE_MAX;
  size_t stack[64];
  int sp = 0;
  if (n) stack[sp++] = 0;
  while (sp) {
    const size_t i = stack[--sp];
    const uint64_t f = node_freq(h[i]);
    if (f < best_f || f < min_freq_ || (best != SIZE_MAX && f == best_f && i > best)) continue;
    const size_t l = 2 * i + 1;
    if (l + 1 < n && sp < 63) stack[sp++] = l + 1;
    if (l < n && sp < 63) stack[sp++] = l;
    const HeapNode& e = h[i];
    if (e.a == unk_ || e.b == unk_) continue;
    bool clash = false;
    for (size_t k = 0; k < n_used; ++k) clash |= e.a == used[k] || e.b == used[k];
    if (clash) continue;
    const Info* in = find(pack_pair(e.a, e.b));
    if (!in || in->version() != node_version(e) || in->freq() != f) continue;
    if (f > best_f || best == SIZE_MAX || i < best) {
      best_f = f;
      best = i;
    }
  }
  if (best == SIZE_MAX) return false;
  *pa = h[best].a;
  *pb = h[best].b;
  if (simulate_pops_) simulate_select(used, n_used, best_f, pa, pb);
  return true;
}

bool Selector::simulate_select(const int32_t* used, size_t n_used, uint64_t floor, int32_t* pa, int32_t* pb) const {
  // Among entries of one frequency the exact pop order decides, and a slot-order guess misses
  // it (late merges are mostly ties).  So the coming select() is replayed on a copy-on-write
  // overlay of the heap as it stands, with tokens in `used` counted as stale (the merge in
  // flight changes their pairs).  Only entries >= floor (a valid entry exists there) can come
  // out first, and they move exactly as in the real heap while every element sifted down from
  // the end is below floor: a child >= floor always beats it, and which entries < floor sit
  // where never decides between entries >= floor.  So a sift stops where both children are
  // below floor.  Any other case (an end element >= floor, the overlay full, too many pops)
  // keeps the caller's guess.
  ++ov_gen_;
  if (ov_gen_ == 0) {  // generation wrap: clear the stamps
    std::fill(ov_stamp_.begin(), ov_stamp_.end(), 0u);
    ov_gen_ = 1;
  }
  constexpr size_t kCap = 1024, kMask = kCap - 1;
  if (ov_stamp_.size() != kCap) {
    ov_stamp_.assign(kCap, 0u);
    ov_pos_.assign(kCap, 0);
    ov_node_.assign(kCap, HeapNode{0, 0, 0});
  }
  size_t used_slots = 0;
  const HeapNode* h = heap_.data() + 1;  // logical slots
  auto slot_of = [&](size_t pos) -> size_t {
    size_t j = (pos * 0x9E3779B97F4A7C15ull >> 40) & kMask;
    while (ov_stamp_[j] == ov_gen_ && ov_pos_[j] != pos) j = (j + 1) & kMask;
    return j;
  };
  auto rd = [&](size_t pos) -> const HeapNode& {
    const size_t j = slot_of(pos);
    return ov_stamp_[j] == ov_gen_ ? ov_node_[j] : h[pos];
  };
  auto wr = [&](size_t pos, const HeapNode& v) -> bool {
    const size_t j = slot_of(pos);
    if (ov_stamp_[j] != ov_gen_) {
      if (++used_slots > kCap / 2) return false;
      ov_stamp_[j] = ov_gen_;
      ov_pos_[j] = pos;
    }
    ov_node_[j] = v;
    return true;
  };
  size_t n = heap_size();
  for (int k = 0; k < 256 && n > 0; ++k) {
    const HeapNode top = rd(0);
    const uint64_t f = node_freq(top);
    if (f < floor) return false;
    bool skip = top.a == unk_ || top.b == unk_;
    for (size_t u = 0; u < n_used && !skip; ++u) skip = top.a == used[u] || top.b == used[u];
    if (!skip) {
      const Info* in = find(pack_pair(top.a, top.b));
      if (in && in->version() == node_version(top) && in->freq() == f) {
        *pa = top.a;
        *pb = top.b;
        return true;
      }
    }
    const HeapNode x = rd(n - 1);  // pop: the last element sifts down from the root
    --n;
    if (n == 0) return false;
    if (node_freq(x) >= floor) return false;
    size_t i = 0;
    for (;;) {
      const size_t l = 2 * i + 1;
      if (l >= n) break;
      const uint64_t lf = node_freq(rd(l));
      const uint64_t rf = l + 1 < n ? node_freq(rd(l + 1)) : 0;
      const bool right = l + 1 < n && rf > lf;
      if ((right ? rf : lf) < floor) break;
      const size_t c = l + right;
      if (!wr(i, rd(c))) return false;
      i = c;
    }
    if (!wr(i, x)) return false;
  }
  return false;
}

size_t Selector::predict_chain(int32_t a, int32_t b, size_t window, size_t k, int32_t* out) const {
  const size_t n = std::min(window, heap_size());
  const HeapNode* h = heap_.data() + 1;
  std::vector<std::pair<uint64_t, size_t>> cand;  // (freq, heap slot) of the valid entries
  for (size_t i = 0; i < n; ++i) {
    const HeapEnt e{h[i].a, h[i].b, node_freq(h[i]), node_version(h[i])};
    if (e.freq < min_freq_ || e.a == unk_ || e.b == unk_) continue;
    const Info* in = find(pack_pair(e.a, e.b));
    if (!in || in->version() != e.version || in->freq() != e.freq) continue;
    cand.push_back({e.freq, i});
  }
  std::stable_sort(cand.begin(), cand.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
  std::vector<int32_t> used = {a, b};
  size_t m = 0;
  for (const auto& c : cand) {
    if (m == k) break;
    const HeapNode& e = h[c.second];
    bool clash = false;
    for (int32_t u : used) clash |= e.a == u || e.b == u;
    if (clash) continue;
    out[2 * m] = e.a;
    out[2 * m + 1] = e.b;
    used.push_back(e.a);
    used.push_back(e.b);
    ++m;
  }
  return m;
}

bool Selector::select(int32_t* a, int32_t* b, uint64_t* freq) {
  while (!heap_empty()) {
    HeapEnt top = pop();
    if (!heap_empty())  // the next top's pair info, fetched while this one is checked
      __builtin_prefetch(&table_[mix64(pack_pair(heap_[1].a, heap_[1].b)) & mask_]);
    Info& in = get(top.a, top.b);
    if (top.version != in.version()) {  // stale entry
      ++ctr_.stale;
      continue;
    }
    // recompute_freq (bpe.cpp:251): info.freq while the map is exact, else the truth table
    uint64_t actual = exact_ ? ((top.a == unk_ || top.b == unk_) ? 0 : in.freq()) : recount(top.a, top.b);
    if (actual != in.freq()) {
      in.set_freq(actual);
      in.bump_version();
      if (actual >= min_freq_) push(top.a, top.b, actual, in.version());
      continue;
    }
    if (actual < min_freq_) continue;
    *a = top.a;
    *b = top.b;
    *freq = actual;
    return true;
  }
  return false;
}

void Selector::apply(int32_t a, int32_t b, int32_t X, const DeltaRecord* recs, size_t n) {
  apply_combine(a, b, X, recs, n);
  apply_finish(a, b, X);
}

void Selector::prepare(int32_t a, int32_t b, int32_t X, const DeltaRecord* recs, size_t n, Prepared* p,
                       const void* prefetch_base, uint64_t prefetch_mask) const {
  const uint64_t c0 = __builtin_ia32_rdtsc();
  p->a = a;
  p->b = b;
  p->X = X;
  p->records = n;
  // 1. records -> FreqChange entries keyed exactly like the reference's pair_hash.
  std::vector<Change>& changes = p->changes;
  changes.clear();
  size_t cap = 64;
  while (cap < 2 * n + 2) cap <<= 1;
  p->index.assign(cap, 0);
  uint32_t* index = p->index.data();
  const uint64_t cm = cap - 1;
  const Info* pt = static_cast<const Info*>(prefetch_base);
  for (size_t i = 0; i < n; ++i) {
    const uint32_t cat = recs[i].key & 3u;
    const uint32_t slot = recs[i].key >> 2;
    const int32_t id = slot == 0 ? unk_ : (int32_t)(slot - 1);
    int32_t first, second;
    switch (cat) {
      case kOldLeft: first = id; second = a; break;
      case kNewLeft: first = id; second = X; break;
      case kOldRight: first = b; second = id; break;
      default: first = X; second = id; break;
    }
    const uint64_t hk = ((uint64_t)(int64_t)first << 32) | (uint64_t)(int64_t)second;
    const int64_t d = (cat == kOldLeft || cat == kOldRight) ? -(int64_t)recs[i].sum : (int64_t)recs[i].sum;
    uint64_t j = mix64(hk) & cm;
    for (;;) {
      uint32_t s = index[j];
      if (!s) {
        // the pair's info line, requested now: the combine and the ordering hide its miss
        if (pt) __builtin_prefetch(&pt[mix64(pack_pair((int32_t)(hk >> 32), (int32_t)hk)) & prefetch_mask]);
        changes.push_back({hk, d, recs[i].ft});
        index[j] = (uint32_t)changes.size();
        break;
      }
      Change& c = changes[s - 1];
      if (c.hk == hk) {
        c.delta += d;
        if (recs[i].ft < c.ft) c.ft = recs[i].ft;
        break;
      }
      j = (j + 1) & cm;
    }
  }
  const uint64_t c1 = __builtin_ia32_rdtsc();
  p->cyc_combine = c1 - c0;
  // 2. reference application order: bucket (hk % 1024) ascending, latest first touch first.
  //    Two stable 5-bit counting passes by bucket (the usual ~100 changes never pay for a
  //    1024-entry prefix), then a sort by first touch inside each bucket.
  static_assert(kDeltaBuckets == 1024, "two 5-bit passes");
  const size_t nc = changes.size();
  std::vector<Change>& staged = p->staged;
  std::vector<Change>& ordered = p->ordered;
  staged.resize(nc);
  ordered.resize(nc);
  {
    uint32_t cnt[33] = {};
    for (const Change& c : changes) cnt[(c.hk & 31u) + 1]++;
    for (int k = 0; k < 32; ++k) cnt[k + 1] += cnt[k];
    for (const Change& c : changes) staged[cnt[c.hk & 31u]++] = c;
  }
  {
    uint32_t cnt[33] = {};
    for (const Change& c : staged) cnt[((c.hk >> 5) & 31u) + 1]++;
    for (int k = 0; k < 32; ++k) cnt[k + 1] += cnt[k];
    for (const Change& c : staged) ordered[cnt[(c.hk >> 5) & 31u]++] = c;
  }
  // Inside a bucket, first touch descending (unique per change, so any sort gives the same
  // order).  Buckets are not small: every (p, a) change lands in a's bucket and every (p, X)
  // change in X's (the bucket is the second id's low bits), so each holds about a quarter of
  // the merge's changes -- sorted, not insertion-sorted.
  for (size_t i = 0; i < nc;) {
    const uint64_t bk = ordered[i].hk % kDeltaBuckets;
    size_t e = i + 1;
    while (e < nc && ordered[e].hk % kDeltaBuckets == bk) ++e;
    if (e - i > 16 && kHaveBmi2) {
      static thread_local std::vector<uint64_t> ka, kb;
      static thread_local std::vector<Change> tmp;
      if (sort_ft_desc_radix(ordered.data() + i, e - i, ka, kb, tmp)) {
        i = e;
        continue;
      }
    }
    if (e - i > 1) std::sort(ordered.begin() + i, ordered.begin() + e, [](const Change& x, const Change& y) { return x.ft > y.ft; });
    i = e;
  }
  p->cyc_order = __builtin_ia32_rdtsc() - c1;
}

void Selector::apply_combine(int32_t a, int32_t b, int32_t X, const DeltaRecord* recs, size_t n) {
  prepare(a, b, X, recs, n, &own_, table_.data(), mask_);
  ctr_.records += n;
  ctr_.changes += own_.changes.size();
  ctr_.cyc_combine += own_.cyc_combine;
  ctr_.cyc_order += own_.cyc_order;
}

void Selector::apply_changes(int32_t a, int32_t b, int32_t X, const Change* c, size_t n) {
  own_.a = a;
  own_.b = b;
  own_.X = X;
  own_.records = n;
  own_.ordered.assign(c, c + n);
  own_.cyc_combine = own_.cyc_order = 0;
  // the walk's info lines, requested together so their misses overlap
  for (size_t i = 0; i < n; ++i)
    __builtin_prefetch(&table_[mix64(pack_pair((int32_t)(c[i].hk >> 32), (int32_t)c[i].hk)) & mask_]);
  ctr_.records += n;
  ctr_.changes += n;
}

void Selector::adopt(Prepared* p) {
  std::swap(own_, *p);
  // the lines the other core requested are in the shared L3: bring them closer for the walk
  for (const Change& c : own_.ordered)
    __builtin_prefetch(&table_[mix64(pack_pair((int32_t)(c.hk >> 32), (int32_t)c.hk)) & mask_]);
  ctr_.records += own_.records;
  ctr_.changes += own_.changes.size();
  ctr_.cyc_combine += own_.cyc_combine;
  ctr_.cyc_order += own_.cyc_order;
}

bool Selector::predict_after(int32_t X, uint64_t above, int32_t* pa, int32_t* pb, uint64_t* pf) const {
  // Pairs holding X are new: their count after this merge is their combined delta, exactly.
  uint64_t best_f = above;
  bool found = false;
  for (const Change& c : own_.ordered) {
    const int32_t f = (int32_t)(uint32_t)(c.hk >> 32), s = (int32_t)(uint32_t)c.hk;
    if ((f != X && s != X) || f == unk_ || s == unk_ || c.delta <= 0) continue;
    const uint64_t v = (uint64_t)c.delta;
    if (v > best_f && v >= min_freq_) {
      best_f = v;
      *pa = f;
      *pb = s;
      found = true;
    }
  }
  if (found) *pf = best_f;
  return found;
}

void Selector::apply_finish(int32_t a, int32_t b, int32_t X) {
  const uint64_t c2 = __builtin_ia32_rdtsc();
  const std::vector<Change>& ordered_ = own_.ordered;
  // (the table lines this merge touches were requested by apply_combine)
  if (2 * (count_ + ordered_.size() + 1) > table_.size()) grow();
  // The pair-info updates first, then the heap pushes in the same order: the pushes read nothing
  // the updates write, so this is the reference's interleaved loop exactly, and the info lines'
  // misses overlap each other instead of waiting behind sift-ups.
  pushes_.clear();
  for (const Change& c : ordered_) {
    const int32_t f = (int32_t)(uint32_t)(c.hk >> 32), s = (int32_t)(uint32_t)c.hk;
    if (f == a && s == b) continue;
    Info& in = get(f, s);
    if (c.delta < 0) {
      const uint64_t m = (uint64_t)(-c.delta);
      in.set_freq(in.freq() >= m ? in.freq() - m : 0);
    } else {
      in.set_freq(in.freq() + (uint64_t)c.delta);
    }
    if (in.freq() >= min_freq_) {
      in.bump_version();
      pushes_.push_back(HeapNode{in.fv, f, s});
    }
  }
  Info& merged = get(a, b);
  merged.set_freq(0);
  merged.bump_version();
  if (truth_live_) {  // the corpus's counts follow the same exact deltas (pairs holding unk: none)
    for (const Change& c : ordered_) {
      const int32_t f = (int32_t)(uint32_t)(c.hk >> 32), s = (int32_t)(uint32_t)c.hk;
      if ((f == a && s == b) || f == unk_ || s == unk_) continue;
      uint64_t& v = truth_[pack_pair(f, s)];
      v = c.delta < 0 ? (v >= (uint64_t)(-c.delta) ? v - (uint64_t)(-c.delta) : 0) : v + (uint64_t)c.delta;
    }
    truth_[pack_pair(a, b)] = 0;
  }
  const uint64_t c3 = __builtin_ia32_rdtsc();
  ctr_.cyc_walk += c3 - c2;
  for (const HeapNode& p : pushes_) push(p.a, p.b, node_freq(p), node_version(p));
  ctr_.cyc_push += __builtin_ia32_rdtsc() - c3;
}

}  // namespace shred
