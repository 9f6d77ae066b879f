// Corpus loading: see corpus.h for the normative rules and reference citations.
#include "corpus.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstring>
#include <thread>

#include "common.h"

namespace shred {
namespace {

inline bool is_delim(uint8_t c) { return c == '\t' || c == '\r' || c == '\n' || c == ' '; }

struct Range { uint64_t begin, end; };

// fgets(buf, size) on the file from `pos`: reads until size-1 bytes or a '\n' is stored.
inline uint64_t fgets_end(const uint8_t* d, uint64_t n, uint64_t pos, uint64_t size) {
  uint64_t lim = std::min<uint64_t>(n, pos + size - 1);
  const void* nl = std::memchr(d + pos, '\n', lim - pos);
  return nl ? (uint64_t)((const uint8_t*)nl - d) + 1 : lim;
}

// The byte ranges the reference's strtok actually sees (bpe.cpp:131-153).  Without NUL bytes
// every line is read whole, so the visible text is the whole file.
std::vector<Range> visible_ranges(const uint8_t* d, uint64_t n) {
  std::vector<Range> out;
  if (n == 0) return out;
  if (!std::memchr(d, 0, n)) { out.push_back({0, n}); return out; }
  uint64_t pos = 0, cap = 4096;  // INITIAL_STR_BUFFER; the buffer never shrinks (bpe.cpp:133-140)
  while (pos < n) {
    uint64_t start = pos;
    pos = fgets_end(d, n, pos, cap);
    auto strlen_from = [&](uint64_t end) {
      const void* z = std::memchr(d + start, 0, end - start);
      return z ? (uint64_t)((const uint8_t*)z - (d + start)) : end - start;
    };
    uint64_t len = strlen_from(pos);
    while (len == cap - 1 && d[start + len - 1] != '\n') {
      cap *= 2;
      if (pos >= n) break;                   // fgets returns NULL at EOF
      pos = fgets_end(d, n, pos, cap - len);  // appends at line + len == start + len == pos
      len = strlen_from(pos);
    }
    if (len) out.push_back({start, start + len});
  }
  return out;
}

// Cuts the visible ranges into pieces of about `target` bytes, only at delimiters.
std::vector<Range> split_pieces(const uint8_t* d, const std::vector<Range>& rs, uint64_t target) {
  std::vector<Range> out;
  for (const Range& r : rs) {
    uint64_t s = r.begin;
    while (s < r.end) {
      uint64_t e = std::min(r.end, s + target);
      while (e < r.end && !is_delim(d[e])) ++e;
      out.push_back({s, e});
      s = e;
    }
  }
  return out;
}

inline uint64_t word_hash(const uint8_t* p, uint32_t len) {
  uint64_t h = 0x84222325CBF29CE4ull ^ len;
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t w;
    std::memcpy(&w, p + i, 8);
    h = (h ^ w) * 0x100000001B3ull;
    h ^= h >> 29;
  }
  for (; i < len; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
  h ^= h >> 32;
  h *= 0xD6E8FEB86659FD93ull;
  h ^= h >> 32;
  return h;
}

struct Entry {
  uint64_t hash;
  uint64_t first;  // file offset of the first occurrence
  uint64_t count;
  uint64_t sp;     // where the spelling lives in the bytes the entry is read against (the file, or
                   // the spellings a sharded load gathered)
  uint32_t len;
  uint32_t pad;
};
static_assert(sizeof(Entry) == 40, "the sharded load ships entries as bytes");

constexpr int kPartBits = 6;
constexpr int kParts = 1 << kPartBits;

// Open-addressing word counter (one per thread and hash partition).
struct Counter {
  std::vector<Entry> ents;
  std::vector<uint32_t> slots;  // index + 1, 0 = empty
  uint64_t mask = 0;

  void grow() {
    uint64_t ns = slots.empty() ? 1024 : 2 * slots.size();
    std::vector<uint32_t> s(ns, 0);
    for (uint32_t i = 0; i < ents.size(); ++i) {
      uint64_t j = ents[i].hash & (ns - 1);
      while (s[j]) j = (j + 1) & (ns - 1);
      s[j] = i + 1;
    }
    slots.swap(s);
    mask = ns - 1;
  }
  // Adds `cnt` occurrences of the word spelled at d[sp, sp+len), first seen at file offset `first`.
  void add(const uint8_t* d, uint64_t hash, uint64_t sp, uint32_t len, uint64_t cnt, uint64_t first) {
    if (2 * (ents.size() + 1) > slots.size()) grow();
    uint64_t j = hash & mask;
    for (;;) {
      uint32_t s = slots[j];
      if (!s) break;
      Entry& e = ents[s - 1];
      if (e.hash == hash && e.len == len && std::memcmp(d + e.sp, d + sp, len) == 0) {
        e.count += cnt;
        if (first < e.first) e.first = first;  // spelling is identical, keep the earliest
        return;
      }
      j = (j + 1) & mask;
    }
    ents.push_back({hash, first, cnt, sp, len, 0});
    slots[j] = (uint32_t)ents.size();
  }
  const Entry* find(const uint8_t* d, uint64_t hash, uint64_t off, uint32_t len) const {
    uint64_t j = hash & mask;
    for (;;) {
      uint32_t s = slots[j];
      if (!s) return nullptr;
      const Entry& e = ents[s - 1];
      if (e.hash == hash && e.len == len && std::memcmp(d + e.sp, d + off, len) == 0) return &e;
      j = (j + 1) & mask;
    }
  }
};

template <class F>
void parallel_for(int threads, size_t n, F&& f) {
  if (threads <= 1 || n <= 1) {
    for (size_t i = 0; i < n; ++i) f(i, 0);
    return;
  }
  std::vector<std::thread> pool;
  std::atomic<size_t> next{0};
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (size_t i; (i = next.fetch_add(1)) < n;) f(i, t);
    });
  for (auto& th : pool) th.join();
}

template <class F>
void scan_words(const uint8_t* d, Range r, F&& f) {
  uint64_t i = r.begin;
  while (i < r.end) {
    while (i < r.end && is_delim(d[i])) ++i;
    uint64_t s = i;
    while (i < r.end && !is_delim(d[i])) ++i;
    if (i > s) f(s, (uint32_t)(i - s));
  }
}

// The word table from the distinct words in reference word order (rank order): spellings,
// counts, the coverage cut and the symbols (bpe.cpp:156-172, histogram.cpp:7-53).
// spell: the spellings already packed in rank order (the device gathered them), else from d.
void finish_table(const uint8_t* d, const std::vector<WordRec>& recs, const LoadOptions& opt, int threads,
                  WordTable* out, std::vector<uint8_t>* spell = nullptr) {
  const size_t W = recs.size();
  if (W > (size_t)kMaxRank) fatal("corpus has more than 2^30 distinct words");
  WordTable& wt = *out;
  wt = WordTable();
  wt.offset.resize(W + 1);
  wt.count.resize(W);
  uint64_t S = 0;
  for (size_t r = 0; r < W; ++r) {
    wt.offset[r] = S;
    wt.count[r] = recs[r].count;
    S += recs[r].len;
  }
  wt.offset[W] = S;
  if (spell) {
    if (spell->size() != S) fatal("device spellings disagree with the word lengths");
    wt.bytes.swap(*spell);
  } else {
    wt.bytes.resize(S);
    parallel_for(threads, (W + 4095) / 4096, [&](size_t blk, int) {
      size_t r1 = std::min(W, (blk + 1) * 4096);
      for (size_t r = blk * 4096; r < r1; ++r) std::memcpy(wt.bytes.data() + wt.offset[r], d + recs[r].first, recs[r].len);
    });
  }
  uint64_t occ = 0;
  for (uint64_t c : wt.count) occ += c;
  wt.total_occurrences = occ;

  // Coverage (bpe.cpp:156-172): unweighted histogram over distinct words.
  std::vector<std::array<uint64_t, 256>> hist(threads);
  for (auto& h : hist) h.fill(0);
  const size_t chunk = 1 << 20;
  parallel_for(threads, (S + chunk - 1) / chunk, [&](size_t c, int t) {
    size_t e = std::min<size_t>(S, (c + 1) * chunk);
    for (size_t i = c * chunk; i < e; ++i) hist[t][wt.bytes[i]]++;
  });
  uint64_t cnt[256] = {};
  for (auto& h : hist)
    for (int c = 0; c < 256; ++c) cnt[c] += h[c];
  std::vector<std::pair<int, uint64_t>> cand;
  for (int bk = 0; bk < 256; ++bk) {
    int c = (bk - 165) & 255;  // StrMap(256) bucket of the 1-byte key c is (5381*33 + c) & 255
    if (cnt[c]) cand.push_back({c, cnt[c]});
  }
  std::stable_sort(cand.begin(), cand.end(),
                   [](const std::pair<int, uint64_t>& a, const std::pair<int, uint64_t>& b) { return a.second > b.second; });
  wt.distinct_bytes = cand.size();
  wt.kept_bytes = (size_t)((float)cand.size() * opt.coverage);
  for (size_t i = 0; i < wt.kept_bytes && i < cand.size(); ++i) wt.keep[cand[i].first] = true;

  int32_t map[256];
  for (int c = 0; c < 256; ++c) map[c] = wt.keep[c] ? c : opt.unk_id;
  wt.symbols.resize(S);
  parallel_for(threads, (S + chunk - 1) / chunk, [&](size_t c, int) {
    size_t e = std::min<size_t>(S, (c + 1) * chunk);
    for (size_t i = c * chunk; i < e; ++i) wt.symbols[i] = map[wt.bytes[i]];
  });
}

// Thread-local counting of the words of `pieces`, partitioned by hash, then merged per partition.
std::vector<Counter> count_pieces(const uint8_t* d, const std::vector<Range>& pieces, int threads,
                                  std::vector<uint64_t>* piece_words) {
  std::vector<std::vector<Counter>> local(threads, std::vector<Counter>(kParts));
  piece_words->assign(pieces.size(), 0);
  parallel_for(threads, pieces.size(), [&](size_t p, int t) {
    auto& parts = local[t];
    uint64_t nw = 0;
    scan_words(d, pieces[p], [&](uint64_t off, uint32_t len) {
      uint64_t h = word_hash(d + off, len);
      parts[h >> (64 - kPartBits)].add(d, h, off, len, 1, off);
      ++nw;
    });
    (*piece_words)[p] = nw;
  });
  std::vector<Counter> merged(kParts);
  parallel_for(threads, kParts, [&](size_t part, int) {
    Counter& m = merged[part];
    for (int t = 0; t < threads; ++t)
      for (const Entry& e : local[t][part].ents) m.add(d, e.hash, e.sp, e.len, e.count, e.first);
  });
  return merged;
}

struct OrderKey { uint64_t order; uint32_t part, idx; };

// Reference word order (djb2 & 4095, first occurrence) over the merged counters, then the table.
// d: the bytes the entries' spellings live in (Entry::sp).
void order_and_finish(const uint8_t* d, const std::vector<Counter>& merged, const LoadOptions& opt, int threads,
                      WordTable* out, std::vector<OrderKey>* keys_out) {
  std::vector<size_t> part_base(kParts + 1, 0);
  for (int p = 0; p < kParts; ++p) part_base[p + 1] = part_base[p] + merged[p].ents.size();
  const size_t W = part_base[kParts];
  if (W > (size_t)kMaxRank) fatal("corpus has more than 2^30 distinct words");
  std::vector<OrderKey>& keys = *keys_out;
  keys.resize(W);
  parallel_for(threads, kParts, [&](size_t p, int) {
    for (uint32_t i = 0; i < merged[p].ents.size(); ++i) {
      const Entry& e = merged[p].ents[i];
      uint64_t h = 5381;
      for (uint32_t k = 0; k < e.len; ++k) h = h * 33 + d[e.sp + k];
      if (e.first >= (1ull << 52)) fatal("corpus larger than 2^52 bytes");
      keys[part_base[p] + i] = {((h & 4095) << 52) | e.first, (uint32_t)p, i};
    }
  });
  {
    // by the 12-bit bucket (the key's top bits) into place, then each bucket sorted on its own
    // thread: one std::sort of 4 M keys was 0.4 s of a C4 merge
    std::vector<size_t> at(4097, 0);
    for (const OrderKey& k : keys) ++at[(k.order >> 52) + 1];
    for (int b = 0; b < 4096; ++b) at[b + 1] += at[b];
    std::vector<OrderKey> tmp(W);
    std::vector<size_t> pos(at.begin(), at.end() - 1);
    for (const OrderKey& k : keys) tmp[pos[k.order >> 52]++] = k;
    parallel_for(threads, 4096, [&](size_t b, int) {
      std::sort(tmp.begin() + at[b], tmp.begin() + at[b + 1],
                [](const OrderKey& x, const OrderKey& y) { return x.order < y.order; });
    });
    keys.swap(tmp);
  }
  std::vector<WordRec> recs(W);
  std::vector<uint64_t> at(W + 1, 0);
  for (size_t r = 0; r < W; ++r) {
    const Entry& e = merged[keys[r].part].ents[keys[r].idx];
    recs[r] = WordRec{e.first, e.count, e.len, 0};
    at[r + 1] = at[r] + e.len;
  }
  std::vector<uint8_t> spell(at[W]);
  parallel_for(threads, (W + 4095) / 4096, [&](size_t blk, int) {
    const size_t r1 = std::min(W, (blk + 1) * 4096);
    for (size_t r = blk * 4096; r < r1; ++r) {
      const Entry& e = merged[keys[r].part].ents[keys[r].idx];
      std::memcpy(spell.data() + at[r], d + e.sp, e.len);
    }
  });
  finish_table(nullptr, recs, opt, threads, out, &spell);
}

// First position >= x after a delimiter (0 and n stay): the words starting before it end before it.
uint64_t shard_cut(const uint8_t* d, uint64_t n, uint64_t x) {
  if (x == 0 || x >= n) return std::min(x, n);
  while (x < n && !is_delim(d[x - 1])) ++x;
  return x;
}

// The distinct words starting in rank r's byte range (of W): entries with their hashes and file
// offsets, their spellings packed in *blob (Entry::sp indexes it), and whether the range holds a
// NUL byte (*nul; the load then falls back to the host's line semantics on every rank).
std::vector<Entry> shard_entries(const uint8_t* d, size_t n, int fd, const LoadOptions& opt, uint64_t r, uint64_t W,
                                 int threads, bool* on_gpu, std::vector<uint8_t>* blob, bool* nul) {
  const uint64_t b = shard_cut(d, n, (uint64_t)((unsigned __int128)n * r / W));
  const uint64_t e = shard_cut(d, n, (uint64_t)((unsigned __int128)n * (r + 1) / W));
  std::vector<Entry> mine;
  blob->clear();
  *on_gpu = false;
  *nul = false;
  if (opt.gpu_device >= 0 && e > b && e - b >= opt.gpu_min_bytes) {
    std::vector<WordRec> recs;
    std::string why;
    // the range straight from the file (reader threads + pinned buffers), the spellings from the
    // device; without a file (in-memory bytes), from the mapping through pinned buffers
    const bool ok = fd >= 0 ? gpu_count_file(opt.gpu_device, fd, b, e - b, &recs, blob, nul, &why)
                            : gpu_count_words(opt.gpu_device, d + b, e - b, &recs, &why, /*staged=*/b > 0 || e < n);
    if (*nul) return mine;
    if (ok) {
      *on_gpu = true;
      const double th = now_seconds();
      std::vector<uint64_t> at(recs.size() + 1, 0);
      for (size_t i = 0; i < recs.size(); ++i) {
        if (fd < 0) recs[i].first += b;
        at[i + 1] = at[i] + recs[i].len;
      }
      if (fd < 0) {
        blob->resize(at[recs.size()]);
        for (size_t i = 0; i < recs.size(); ++i) std::memcpy(blob->data() + at[i], d + recs[i].first, recs[i].len);
      }
      mine.resize(recs.size());
      parallel_for(threads, (recs.size() + 4095) / 4096, [&](size_t blk, int) {
        const size_t i1 = std::min(recs.size(), (blk + 1) * 4096);
        for (size_t i = blk * 4096; i < i1; ++i)
          mine[i] = Entry{word_hash(blob->data() + at[i], recs[i].len), recs[i].first, recs[i].count, at[i],
                          recs[i].len, 0};
      });
      if (std::getenv("SHREDWORD_LOAD_REPORT"))
        std::fprintf(stderr, "[LOAD] range %llu/%llu: %zu word hashes %.1f ms\n", (unsigned long long)r,
                     (unsigned long long)W, recs.size(), 1e3 * (now_seconds() - th));
      return mine;
    }
    std::fprintf(stderr, "[WARNING]\t GPU word count unavailable (%s): counting on the host\n", why.c_str());
  }
  if (e > b) {
    if (std::memchr(d + b, 0, e - b)) {
      *nul = true;
      return mine;
    }
    const uint64_t target = std::max<uint64_t>(1 << 20, (e - b) / (uint64_t)(threads * 8) + 1);
    std::vector<uint64_t> pw;
    std::vector<Counter> c = count_pieces(d, split_pieces(d, {{b, e}}, target), threads, &pw);
    uint64_t at = 0;
    for (const Counter& k : c)
      for (const Entry& x : k.ents) {
        mine.push_back(x);
        mine.back().sp = at;
        at += x.len;
      }
    blob->resize(at);
    for (const Entry& x : mine) std::memcpy(blob->data() + x.sp, d + x.first, x.len);
  }
  return mine;
}

// Every rank's word list merged (counts summed, first occurrence min; equal hashes must spell
// the same word: Counter::add compares the bytes), then the table in reference order.  `blob`
// holds every entry's spelling (Entry::sp).
void merge_entries(const uint8_t* blob, const Entry* all, size_t total, const LoadOptions& opt, int threads,
                   WordTable* out) {
  const double t0 = now_seconds();
  // 64-bit indices: Σ over ranks of distinct words per rank can pass 2^32 even when the merged
  // table stays small
  std::vector<std::vector<uint64_t>> by_part(kParts);
  for (size_t i = 0; i < total; ++i) by_part[all[i].hash >> (64 - kPartBits)].push_back((uint64_t)i);
  std::vector<Counter> merged(kParts);
  parallel_for(threads, kParts, [&](size_t p, int) {
    for (uint64_t i : by_part[p]) merged[p].add(blob, all[i].hash, all[i].sp, all[i].len, all[i].count, all[i].first);
  });
  const double t1 = now_seconds();
  std::vector<OrderKey> keys;
  order_and_finish(blob, merged, opt, threads, out, &keys);
  if (std::getenv("SHREDWORD_LOAD_REPORT"))
    std::fprintf(stderr, "[LOAD] merge of %zu listed words: %.1f ms combine, %.1f ms order + table (%zu distinct)\n",
                 total, 1e3 * (t1 - t0), 1e3 * (now_seconds() - t1), keys.size());
}

// A rank's words as one gather buffer: [u64 entries][u64 blob bytes][u64 nul][entries][blob].
void pack_shard(const std::vector<Entry>& ents, const std::vector<uint8_t>& blob, bool nul, std::vector<uint8_t>* out) {
  const uint64_t h[3] = {ents.size(), blob.size(), nul ? 1ull : 0ull};
  out->resize(sizeof(h) + ents.size() * sizeof(Entry) + blob.size());
  std::memcpy(out->data(), h, sizeof(h));
  if (!ents.empty()) std::memcpy(out->data() + sizeof(h), ents.data(), ents.size() * sizeof(Entry));
  if (!blob.empty()) std::memcpy(out->data() + sizeof(h) + ents.size() * sizeof(Entry), blob.data(), blob.size());
}

// Appends one rank's buffer to (all, blob), its spellings' offsets moved past the blob so far.
// False for a malformed buffer; *used = its size.
bool unpack_shard(const uint8_t* p, size_t avail, std::vector<Entry>* all, std::vector<uint8_t>* blob, bool* nul,
                  size_t* used) {
  uint64_t h[3];
  if (avail < sizeof(h)) return false;
  std::memcpy(h, p, sizeof(h));
  const size_t need = sizeof(h) + h[0] * sizeof(Entry) + h[1];
  if (h[0] > avail / sizeof(Entry) || h[1] > avail || need > avail) return false;
  const uint64_t base = blob->size();
  const size_t e0 = all->size();
  all->resize(e0 + h[0]);
  if (h[0]) std::memcpy(all->data() + e0, p + sizeof(h), h[0] * sizeof(Entry));
  for (size_t i = e0; i < all->size(); ++i) (*all)[i].sp += base;
  blob->insert(blob->end(), p + sizeof(h) + h[0] * sizeof(Entry), p + need);
  *nul = *nul || h[2] != 0;
  *used = need;
  return true;
}

// The sharded load (LoadOptions::shard_world > 1): this rank's words, then every rank's merged.
// SHREDWORD_LOAD_SIM_SHARDS=k (tests, one process): the k ranges counted in turn, merged the same way.
// Returns 0, -1 on a failed gather (*err), or 1 when some range holds a NUL byte (the caller loads
// without sharding: the reference's line semantics need the whole file in order).
int load_sharded(const uint8_t* d, size_t n, int fd, const LoadOptions& opt, int threads, WordTable* out, int sim,
                 std::string* err) {
  bool on_gpu = false, nul = false;
  std::vector<Entry> all;
  std::vector<uint8_t> blob;
  if (sim > 1) {
    for (int r = 0; r < sim && !nul; ++r) {
      bool g = false, z = false;
      std::vector<uint8_t> b;
      std::vector<Entry> m = shard_entries(d, n, fd, opt, (uint64_t)r, (uint64_t)sim, threads, &g, &b, &z);
      on_gpu = on_gpu || g;
      nul = nul || z;
      std::vector<uint8_t> buf;
      pack_shard(m, b, z, &buf);
      size_t used = 0;
      unpack_shard(buf.data(), buf.size(), &all, &blob, &nul, &used);
    }
  } else {
    std::vector<uint8_t> b;
    bool z = false;
    std::vector<Entry> mine = shard_entries(d, n, fd, opt, (uint64_t)opt.shard_rank, (uint64_t)opt.shard_world, threads,
                                            &on_gpu, &b, &z);
    std::vector<uint8_t> buf;
    pack_shard(mine, b, z, &buf);
    size_t got = 0;
    const double tg = now_seconds();
    const uint8_t* g = (const uint8_t*)opt.gather(opt.gather_ctx, buf.data(), buf.size(), &got);
    if (std::getenv("SHREDWORD_LOAD_REPORT"))
      std::fprintf(stderr, "[LOAD] rank %d: word-list all-gather %.1f ms (%zu bytes sent, %zu received)\n",
                   opt.shard_rank, 1e3 * (now_seconds() - tg), buf.size(), got);
    // A failed gather (the caller's callback raised, a peer left) must not become an empty
    // table: every rank would then train on nothing without an error.
    bool ok = g != nullptr && got >= buf.size();
    size_t pos = 0, ranks = 0;
    while (ok && pos < got) {
      size_t used = 0;
      ok = unpack_shard(g + pos, got - pos, &all, &blob, &nul, &used);
      pos += used;
      ++ranks;
    }
    if (!ok || ranks != (size_t)opt.shard_world) {
      if (err)
        *err = "sharded load: the word-list all-gather failed (" + std::to_string(got) + " bytes returned for " +
               std::to_string(buf.size()) + " sent)";
      return -1;
    }
  }
  if (nul) return 1;
  merge_entries(blob.data(), all.data(), all.size(), opt, threads, out);
  out->counted_on_gpu = on_gpu;
  return 0;
}

}  // namespace

int load_corpus_bytes(const uint8_t* d, size_t n, const LoadOptions& opt, WordTable* out, std::string* err, int fd) {
  int threads = opt.threads > 0 ? opt.threads : (int)std::thread::hardware_concurrency();
  threads = std::max(1, std::min(threads, 32));
  const char* sim_env = std::getenv("SHREDWORD_LOAD_SIM_SHARDS");
  const int sim = sim_env ? std::atoi(sim_env) : 0;
  if (((opt.shard_world > 1 && opt.gather) || sim > 1) && !opt.want_stream && n > 0) {
    const int r = load_sharded(d, n, fd, opt, threads, out, sim, err);
    if (r <= 0) return r;
    // a NUL byte in some rank's range: every rank loads the whole file the reference's way
  }
  // the device count (types layout, NUL-free files: every line is read whole, so the words are
  // the maximal runs of non-delimiters of the whole file)
  const bool report = std::getenv("SHREDWORD_LOAD_REPORT") != nullptr;
  const double tz = now_seconds();
  const bool nul_free = opt.gpu_device >= 0 && !opt.want_stream && n >= opt.gpu_min_bytes && !std::memchr(d, 0, n);
  if (report && opt.gpu_device >= 0) std::fprintf(stderr, "[LOAD] phase nul_scan %.1f ms (host memchr, page-in)\n",
                                                   1e3 * (now_seconds() - tz));
  if (nul_free) {
    std::vector<WordRec> recs;
    std::string why;
    const double t0 = now_seconds();
    if (gpu_count_words(opt.gpu_device, d, n, &recs, &why)) {
      const double t1 = now_seconds();
      finish_table(d, recs, opt, threads, out);
      out->counted_on_gpu = true;
      if (std::getenv("SHREDWORD_LOAD_REPORT"))
        std::fprintf(stderr, "[LOAD] device count %.1f ms, host table %.1f ms\n", 1e3 * (t1 - t0),
                     1e3 * (now_seconds() - t1));
      return 0;
    }
    std::fprintf(stderr, "[WARNING]\t GPU word count unavailable (%s): counting on the host\n", why.c_str());
  }
  std::vector<Range> vis = visible_ranges(d, n);
  uint64_t vis_bytes = 0;
  for (auto& r : vis) vis_bytes += r.end - r.begin;
  uint64_t target = std::max<uint64_t>(1 << 20, vis_bytes / (uint64_t)(threads * 8) + 1);
  std::vector<Range> pieces = split_pieces(d, vis, target);
  std::vector<uint64_t> piece_words;
  std::vector<Counter> merged = count_pieces(d, pieces, threads, &piece_words);
  std::vector<OrderKey> keys;
  order_and_finish(d, merged, opt, threads, out, &keys);
  WordTable& wt = *out;

  if (opt.want_stream) {
    const size_t W = keys.size();
    // rank of every distinct word, addressable through the merged counters
    std::vector<std::vector<uint32_t>> rank_of(kParts);
    for (int p = 0; p < kParts; ++p) rank_of[p].resize(merged[p].ents.size());
    for (size_t r = 0; r < W; ++r) rank_of[keys[r].part][keys[r].idx] = (uint32_t)r;
    std::vector<uint64_t> base(pieces.size() + 1, 0);
    for (size_t p = 0; p < pieces.size(); ++p) base[p + 1] = base[p] + piece_words[p];
    wt.occurrence_rank.resize(base[pieces.size()]);
    parallel_for(threads, pieces.size(), [&](size_t p, int) {
      uint64_t k = base[p];
      scan_words(d, pieces[p], [&](uint64_t off, uint32_t len) {
        uint64_t h = word_hash(d + off, len);
        int part = (int)(h >> (64 - kPartBits));
        const Entry* e = merged[part].find(d, h, off, len);
        wt.occurrence_rank[k++] = rank_of[part][(uint32_t)(e - merged[part].ents.data())];
      });
    });
  }
  return 0;
}

int load_corpus(const char* path, const LoadOptions& opt, WordTable* out, std::string* err) {
  int fd = ::open(path, O_RDONLY);
  if (fd < 0) {
    if (err) *err = std::string("Couldn't open file: ") + path;
    return -1;
  }
  struct stat st;
  if (::fstat(fd, &st) != 0) {
    ::close(fd);
    if (err) *err = std::string("Couldn't stat file: ") + path;
    return -1;
  }
  size_t n = (size_t)st.st_size;
  if (n == 0) {
    ::close(fd);
    return load_corpus_bytes(nullptr, 0, opt, out, err);
  }
  // The device path reads the file itself (no mapping): the whole-file count of a types-layout
  // load.  A NUL byte sends the file to the host's fgets/strlen path below.
  LoadOptions o2 = opt;
  const char* sim_env = std::getenv("SHREDWORD_LOAD_SIM_SHARDS");
  const bool sharded = (opt.shard_world > 1 && opt.gather) || (sim_env && std::atoi(sim_env) > 1);
  if (opt.gpu_device >= 0 && !opt.want_stream && !sharded && n >= opt.gpu_min_bytes) {
    std::vector<WordRec> recs;
    std::vector<uint8_t> spell;
    std::string why;
    bool nul = false;
    const double t0 = now_seconds();
    if (gpu_count_file(opt.gpu_device, fd, 0, n, &recs, &spell, &nul, &why)) {
      ::close(fd);
      const double t1 = now_seconds();
      int threads = opt.threads > 0 ? opt.threads : (int)std::thread::hardware_concurrency();
      threads = std::max(1, std::min(threads, 32));
      finish_table(nullptr, recs, opt, threads, out, &spell);
      out->counted_on_gpu = true;
      if (std::getenv("SHREDWORD_LOAD_REPORT"))
        std::fprintf(stderr, "[LOAD] phase device_count %.1f ms (file -> HBM, count, order, spellings), host_table "
                     "%.1f ms (coverage, symbols)\n", 1e3 * (t1 - t0), 1e3 * (now_seconds() - t1));
      return 0;
    }
    if (!nul) std::fprintf(stderr, "[WARNING]\t GPU word count unavailable (%s): counting on the host\n", why.c_str());
    o2.gpu_device = -1;  // the host path (NUL bytes: the reference's line semantics)
  }
  void* m = ::mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
  if (m == MAP_FAILED) {
    ::close(fd);
    if (err) *err = std::string("Couldn't map file: ") + path;
    return -1;
  }
  ::madvise(m, n, MADV_SEQUENTIAL);
  const int rc = load_corpus_bytes((const uint8_t*)m, n, o2, out, err, sharded ? fd : -1);
  ::munmap(m, n);
  ::close(fd);
  return rc;
}

}  // namespace shred
