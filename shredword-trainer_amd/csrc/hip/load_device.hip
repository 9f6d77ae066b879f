// GPU word count of the corpus load (replaces the O(tokens · W / 4096) word
// counting of reference bpe.cpp:110-153 / hash.cpp:29-72 on the device).
//
// The file's bytes are uploaded once; then, on gfx950:
//   k_word_count   per 16 KB tile staged in LDS (coalesced 16-B loads: the text is read from HBM
//                  once), one thread per 64-byte chunk takes the words that START in its chunk
//                  (maximal runs of bytes outside "\t\r\n "), hashes each (64-bit FNV-1a + length
//                  mix) with its djb2 & 4095 (the reference StrMap bucket), and counts it in a
//                  per-workgroup LDS table (count, min first offset) that spills to, and is
//                  flushed into, one open-addressing HBM table with 64-bit atomics.  Every
//                  occurrence is compared byte for byte with an earlier occurrence of its key
//                  (the one atomicMin hands back), so a 64-bit key collision is detected (the
//                  count is then repeated with another seed) and the table is exact;
//   k_word_compact entries -> (bucket << 52 | first offset) keys, radix-sorted (hipCUB): the
//                  reference word order, since first offsets are distinct;
//   k_word_gather  rank -> {first, count, length} records for the host.
// The host keeps the fgets/strlen path for files with NUL bytes (corpus.cpp) and builds the word
// table (spellings, coverage, symbols) from the records.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <sched.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../host/corpus.h"

namespace shred {
namespace {

typedef unsigned long long u64;

#define LOAD_OK(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) {                                                                     \
      if (why) *why = std::string(#expr) + ": " + hipGetErrorString(e_);                        \
      return false;                                                                             \
    }                                                                                           \
  } while (0)

constexpr int kChunkBytes = 64;      // bytes whose word starts one thread owns
constexpr int kTileStride = kChunkBytes + 4;  // LDS bytes per chunk: the lanes' chunks start in distinct banks
// Two workgroup shapes (36 B an LDS slot; the tile is kChunkBytes per thread, staged at kTileStride):
//   narrow: 256 threads, 16 KB tiles, 1536 slots (54 KB + 17 KB): two workgroups per CU;
//   wide:   512 threads, 32 KB tiles, 3072 slots (108 KB + 34 KB): one workgroup per CU, a table
//           twice the size over twice the range (fewer words spill to HBM: 16.5% -> 12.3% of
//           occurrences at C3 by a host simulation of the table).
constexpr int kNarrowThreads = 256, kNarrowSlots = 1536;
constexpr int kWideThreads = 512, kWideSlots = 3072;
// xwide (round 5): 768 threads, 48 KB tiles, the same 3072 slots (108 KB + 51 KB): 12 waves a CU
// instead of 8, more HBM spill chains in flight (the count is bound by them, not by its bytes)
constexpr int kXWideThreads = 768;
constexpr int kLdsProbes = 8;
constexpr int kSpell = 16;           // leading bytes of a word an LDS slot keeps
constexpr size_t kPadBytes = (size_t)kChunkBytes * kXWideThreads + 256;  // ' ' past the corpus: every tile load and word scan stays inside
// HBM table probes before the table counts as too full (it is grown 4x and the count rerun); with
// the 3/4 fill flag the usual probe run is a few slots
constexpr u64 kTableProbes = 512;
constexpr uint32_t kLoadEvictPctDefault = 0;  // LDS eviction off by default (A/B: SHREDWORD_LOAD_EVICT)
constexpr int kLoadShapeDefault = 2;  // xwide: C3 load 1.09-1.12 s -> 0.92-0.95 s (round 5 A/B on one box)

__device__ __forceinline__ bool delim(uint32_t c) { return c == 9u || c == 13u || c == 10u || c == 32u; }
__device__ __forceinline__ uint32_t has_zero(uint32_t v) { return (v - 0x01010101u) & ~v & 0x80808080u; }

// One 32-byte HBM slot per distinct word (a probe and its atomics touch one cache line).
struct Slot {
  u64 key;     // 0 = empty; else mix(hash, len, seed) | 1
  u64 cnt;
  u64 nfirst;  // ~(min first offset): 0 = none yet, so the table clears with one memset
  uint32_t len;
  uint32_t bkt;  // djb2 & 4095
};
static_assert(sizeof(Slot) == 32, "slot layout");

struct Table {
  Slot* slot;
  u64 mask;         // capacity - 1
  uint32_t* nkeys;
  uint32_t* flags;  // [0] table too full, [1] key collision, [2] a NUL byte in the text, [3] a word
                    // past a segment's landed bytes
  u64* stats;       // [0] words, [1] counted straight in HBM (LDS table full / slot being made),
                    // [2] words longer than the LDS spelling that hit an LDS slot, [3] LDS slots evicted
};

// kmask keeps all 64 bits (tests narrow it, SHREDWORD_LOAD_KEY_BITS, to force key collisions).
__device__ __forceinline__ u64 word_key(u64 h, uint32_t len, u64 seed, u64 kmask) {
  h ^= (u64)len * 0x9E3779B97F4A7C15ull ^ seed;
  h ^= h >> 31;
  h *= 0xD6E8FEB86659FD93ull;
  h ^= h >> 32;
  return (h & kmask) | 1ull;
}

// Byte p of the workgroup's tile (p may run past the tile: then from HBM).
template <int kTileBytes>
__device__ __forceinline__ uint32_t tile_byte(const uint8_t* s, const uint8_t* d, u64 base, uint32_t p) {
  return p < (uint32_t)kTileBytes ? s[(p / kChunkBytes) * kTileStride + (p % kChunkBytes)] : d[base + p];
}

// True when the words at d[a] and d[b] (a's length len) spell the same bytes.  The bytes are
// loaded 16 at a time, every load of a batch issued before the first compare (one HBM round trip
// per 16 bytes instead of one per byte); reads past a word stay inside the text's ' ' padding.
__device__ __forceinline__ bool same_global(const uint8_t* d, u64 a, u64 b, uint32_t len) {
  uint32_t diff = delim(d[b + len]) ? 0u : 1u;
  for (uint32_t k = 0; k < len; k += 16) {
    uint32_t x[16], y[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      x[j] = d[a + k + j];
      y[j] = d[b + k + j];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) diff |= k + j < len ? x[j] ^ y[j] : 0u;
  }
  return diff == 0;
}
// djb2 (32 bits) of the len bytes at d[a], 16 loads in flight at a time.
__device__ __forceinline__ uint32_t djb2_global(const uint8_t* d, u64 a, uint32_t len) {
  uint32_t dj = 5381u;
  for (uint32_t k = 0; k < len; k += 16) {
    uint32_t x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = d[a + k + j];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (k + j < len) dj = dj * 33u + x[j];
  }
  return dj;
}

// Adds (cnt, first) to key's slot.  Exactness: every add but the slot's very first compares its
// occurrence with the offset the atomic hands back — an occurrence some earlier add stored — so
// all the occurrences behind one key are linked by byte-equal pairs, or flags[1] is raised (a
// 64-bit key collision: the count is repeated with another seed).
__device__ __forceinline__ void table_add(const uint8_t* d, const Table& t, u64 key, uint32_t bkt, uint32_t len,
                                          u64 cnt, u64 first) {
  u64 s = key & t.mask;
  for (u64 probe = 0; probe < kTableProbes; ++probe) {
    Slot& e = t.slot[s];
    u64 prev = e.key;
    if (prev == 0ull) {
      prev = atomicCAS(&e.key, 0ull, key);
      if (prev == 0ull) {
        e.len = len;
        e.bkt = bkt;
        if (atomicAdd(t.nkeys, 1u) > (uint32_t)((t.mask + 1) / 4 * 3)) atomicOr(&t.flags[0], 1u);
        prev = key;
      }
    }
    if (prev == key) {
      atomicAdd(&e.cnt, cnt);
      const u64 link = ~atomicMax(&e.nfirst, ~first);  // ~0: none yet (this is the key's first add)
      if (link != ~0ull && !same_global(d, first, link, len)) atomicOr(&t.flags[1], 1u);
      return;
    }
    s = (s + 1) & t.mask;
  }
  atomicOr(&t.flags[0], 1u);
}

// One pass over the corpus.  Workgroup w owns a contiguous range of tiles (kChunkBytes per thread); each tile is
// staged in LDS with coalesced 16-B loads (the text is read from HBM once), and each thread takes
// the words that START in its 64-byte chunk (maximal runs of bytes outside "\t\r\n "), hashes each
// (64-bit FNV-1a + length mix) and counts it in the workgroup's LDS table (count, min first
// offset relative to the range, length, the first kSpell bytes of its creator's spelling), which
// spills to, and at the end is flushed into, one open-addressing HBM table.
// Exactness without a second pass: an LDS hit compares its bytes with the slot's kSpell-byte
// spelling (LDS) and its length with the slot's; bytes past kSpell with the occurrence the
// slot's atomicMin hands back (the same linking argument as table_add), and the flush and every
// spill compare with the HBM slot's occurrence.  A slot is used once its length is published
// (0 = being created: the occurrence then goes to HBM directly).  The reference StrMap bucket
// (djb2 & 4095) is computed at the flush, from the slot's first occurrence.
template <int kLoadThreads, int kLdsSlots>
__global__ __launch_bounds__(kLoadThreads) void k_word_count(const uint8_t* d, u64 n, Table t, u64 seed, u64 kmask,
                                                             u64 tiles_per_wg, u64 tile0, u64 tile1, u64 safe_end,
                                                             uint32_t evict_at) {
  constexpr int kTileBytes = kChunkBytes * kLoadThreads;
  __shared__ u64 s_key[kLdsSlots];
  __shared__ uint32_t s_first[kLdsSlots];
  __shared__ uint32_t s_cnt[kLdsSlots];
  __shared__ uint32_t s_len[kLdsSlots];
  __shared__ uint4 s_spell[kLdsSlots];
  __shared__ uint32_t s_tile32[kLoadThreads * kTileStride / 4];
  const uint8_t* s_tile = reinterpret_cast<const uint8_t*>(s_tile32);
  const int tid = threadIdx.x;
  for (int i = tid; i < kLdsSlots; i += kLoadThreads) {
    s_key[i] = 0;
    s_first[i] = ~0u;
    s_cnt[i] = 0;
    s_len[i] = 0;
  }
  // tiles [tile0, tile1) of the text (a segment counted while later ones are still uploading:
  // bytes at or past safe_end may not have landed yet)
  const u64 t0 = tile0 + (u64)blockIdx.x * tiles_per_wg;
  const u64 t1 = t0 + tiles_per_wg < tile1 ? t0 + tiles_per_wg : tile1;
  const u64 range = t0 * kTileBytes;  // LDS first offsets are relative to it (< 2^32: host-checked)
  __shared__ uint32_t s_full, s_nul, s_used, s_thr;
  if (tid == 0) {
    s_nul = 0;
    s_used = 0;
    s_thr = 1;
  }
  uint32_t n_words = 0, n_hbm = 0, n_long = 0, n_evict = 0;
  for (u64 tile = t0; tile < t1; ++tile) {
    const u64 base = tile * kTileBytes;
    if (tid == 0) s_full = __hip_atomic_load(&t.flags[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();  // the previous tile's scans are done
    if (s_full) return;  // the table is too full: this count is rerun on a bigger one
    // Eviction (evict_at > 0): once the LDS table holds more than evict_at slots, the words it met
    // at most s_thr times go to the HBM table (counts, first offsets and links as at the final
    // flush) and their slots are freed, so words that keep coming get slots instead of the rare
    // words of the first tiles.  A key may then hold two slots (a probe run broken by a freed
    // slot): both are flushed, and the HBM table adds them up.
    if (evict_at && s_used > evict_at) {
      uint32_t freed = 0;
      for (int i = tid; i < kLdsSlots; i += kLoadThreads) {
        if (!s_key[i] || s_cnt[i] > s_thr) continue;
        const u64 first = range + s_first[i];
        const uint32_t len = s_len[i];
        table_add(d, t, s_key[i], djb2_global(d, first, len) & 4095u, len, s_cnt[i], first);
        s_key[i] = 0;
        s_first[i] = ~0u;
        s_cnt[i] = 0;
        s_len[i] = 0;
        ++freed;
      }
      n_evict += freed;
      if (freed) atomicSub(&s_used, freed);
      __syncthreads();
      if (tid == 0 && s_used > evict_at - evict_at / 4) s_thr = s_thr < (1u << 30) ? 2u * s_thr : s_thr;  // freed too little
      __syncthreads();
    }
    const int4* g = reinterpret_cast<const int4*>(d + base);
#pragma unroll
    for (int j = 0; j < kTileBytes / 16 / kLoadThreads; ++j) {
      const int q = j * kLoadThreads + tid;  // 16-B piece q of the tile
      const int4 v = g[q];
      // a NUL byte anywhere (the reference's fgets/strlen cuts lines there: those files take the
      // host path; bytes past the corpus are the ' ' padding)
      const uint32_t z = has_zero((uint32_t)v.x) | has_zero((uint32_t)v.y) | has_zero((uint32_t)v.z) |
                         has_zero((uint32_t)v.w);
      if (z && base + (u64)q * 16 < n) s_nul = 1u;
      uint32_t* dst = s_tile32 + (q / (kChunkBytes / 16)) * (kTileStride / 4) + (q % (kChunkBytes / 16)) * 4;
      dst[0] = (uint32_t)v.x;
      dst[1] = (uint32_t)v.y;
      dst[2] = (uint32_t)v.z;
      dst[3] = (uint32_t)v.w;
    }
    __syncthreads();
    uint32_t p = (uint32_t)tid * kChunkBytes;
    const uint32_t end = p + kChunkBytes;
    const uint32_t prev = p ? tile_byte<kTileBytes>(s_tile, d, base, p - 1) : (base ? d[base - 1] : 32u);
    if (!delim(prev))  // a word running in from the previous chunk belongs to that chunk
      while (p < end && !delim(tile_byte<kTileBytes>(s_tile, d, base, p))) ++p;
    for (;;) {
      while (p < end && delim(tile_byte<kTileBytes>(s_tile, d, base, p))) ++p;
      if (p >= end || base + p >= n) break;
      u64 h = 0xCBF29CE484222325ull ^ seed;
      uint32_t w[kSpell / 4] = {0, 0, 0, 0};  // the leading bytes, packed
      uint32_t len = 0;
      for (;; ++len) {
        if (base + p + len >= safe_end) {  // a word running past the landed bytes: count again later
          atomicOr(&t.flags[3], 1u);
          break;
        }
        const uint32_t c = tile_byte<kTileBytes>(s_tile, d, base, p + len);
        if (delim(c)) break;
        h = (h ^ c) * 0x100000001B3ull;
        if (len < (uint32_t)kSpell) w[len / 4] |= c << (8 * (len % 4));
      }
      const u64 key = word_key(h, len, seed, kmask), off = base + p;
      const uint32_t rel = (uint32_t)(off - range);
      uint32_t s = (uint32_t)(((key >> 32) * (u64)kLdsSlots) >> 32);
      bool done = false;
      for (int probe = 0; probe < kLdsProbes && !done; ++probe) {
        u64 k = s_key[s];
        bool mine = false;
        if (k == 0ull) {
          k = atomicCAS(&s_key[s], 0ull, key);
          if (k == 0ull) {  // created: spelling and first offset, then the length publishes it
            mine = true;
            if (evict_at) atomicAdd(&s_used, 1u);
            k = key;
            s_spell[s] = make_uint4(w[0], w[1], w[2], w[3]);
            atomicMin(&s_first[s], rel);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __hip_atomic_store(&s_len[s], len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            atomicAdd(&s_cnt[s], 1u);
            done = true;
          }
        }
        if (!mine && k == key) {
          const uint32_t sl = __hip_atomic_load(&s_len[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (sl == 0u) break;  // being created: count this one in HBM
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          const uint4 sp = s_spell[s];
          uint32_t diff = (sl != len) | (sp.x ^ w[0]) | (sp.y ^ w[1]) | (sp.z ^ w[2]) | (sp.w ^ w[3]);
          uint32_t link = s_first[s];
          if (rel < link) link = atomicMin(&s_first[s], rel);
          if (len > (uint32_t)kSpell && link != ~0u && !diff) {
            ++n_long;
            const u64 rep = range + link;
            for (uint32_t q = kSpell; q < len; q += 16) {  // the representative's bytes: 16 loads in flight
              uint32_t r[16];
#pragma unroll
              for (int j = 0; j < 16; ++j) r[j] = d[rep + q + j];
#pragma unroll
              for (int j = 0; j < 16; ++j)
                if (q + j < len) diff |= tile_byte<kTileBytes>(s_tile, d, base, p + q + j) ^ r[j];
            }
          }
          if (diff) atomicOr(&t.flags[1], 1u);
          atomicAdd(&s_cnt[s], 1u);
          done = true;
        } else if (!done) {
          s = s + 1 == (uint32_t)kLdsSlots ? 0u : s + 1;
        }
      }
      ++n_words;
      if (!done) {
        ++n_hbm;
        uint32_t dj = 5381u;  // djb2 in 32 bits: its & 4095 equals the reference's 64-bit value's
        for (uint32_t q = 0; q < len; ++q) dj = dj * 33u + tile_byte<kTileBytes>(s_tile, d, base, p + q);
        table_add(d, t, key, dj & 4095u, len, 1ull, off);
      }
      p += len;
    }
  }
  __syncthreads();
  if (tid == 0 && s_nul) atomicOr(&t.flags[2], 1u);
  if (n_words) atomicAdd(&t.stats[0], (u64)n_words);
  if (n_hbm) atomicAdd(&t.stats[1], (u64)n_hbm);
  if (n_long) atomicAdd(&t.stats[2], (u64)n_long);
  if (n_evict) atomicAdd(&t.stats[3], (u64)n_evict);
  for (int i = tid; i < kLdsSlots; i += kLoadThreads) {
    if (!s_key[i]) continue;
    const u64 first = range + s_first[i];
    const uint32_t len = s_len[i];
    table_add(d, t, s_key[i], djb2_global(d, first, len) & 4095u, len, s_cnt[i], first);
  }
}

__global__ void k_word_compact(Table t, u64* okey, uint32_t* oslot, uint32_t* nout) {
  for (u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x; s <= t.mask; s += (u64)gridDim.x * blockDim.x) {
    const Slot& e = t.slot[s];
    if (!e.key) continue;
    const uint32_t i = atomicAdd(nout, 1u);
    okey[i] = ((u64)e.bkt << 52) | ~e.nfirst;
    oslot[i] = (uint32_t)s;
  }
}

__global__ void k_word_gather(Table t, const uint32_t* slot, uint32_t W, WordRec* out) {
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < W; r += gridDim.x * blockDim.x) {
    const Slot& e = t.slot[slot[r]];
    WordRec w;
    w.first = ~e.nfirst;
    w.count = e.cnt;
    w.len = e.len;
    w.pad = 0;
    out[r] = w;
  }
}

// rank r's length, for the offsets of the packed spellings
__global__ void k_word_lens(const WordRec* rec, uint32_t W, u64* len) {
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < W; r += gridDim.x * blockDim.x) len[r] = rec[r].len;
}
// The spellings packed in rank order (the host word table's byte array): a wave per 64 words, a
// lane per word.
__global__ void k_word_spell(const uint8_t* d, const WordRec* rec, const u64* off, uint32_t W, uint8_t* out) {
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < W; r += gridDim.x * blockDim.x) {
    const uint8_t* src = d + rec[r].first;
    uint8_t* dst = out + off[r];
    for (uint32_t k = 0; k < rec[r].len; ++k) dst[k] = src[k];
  }
}

struct DevBuf {
  void* p = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace

// The pinned host ring of the streamed load, kept for the process (a later load of the same
// shape reuses it: pinning 4 x 64 MiB costs 50-90 ms on the box, unpinning as much again).  The
// first load allocates it on a helper thread while the device buffer is being set up; the readers
// wait per buffer (ready[k]: 0 pending, 1 ready, 2 failed).
struct PinRing {
  std::mutex mu;  // one streamed load at a time owns the ring
  std::vector<void*> buf;
  size_t chunk = 0;
  std::unique_ptr<std::atomic<int>[]> ready;
};
static PinRing& pin_ring() {
  static PinRing* r = new PinRing();  // never destroyed: the runtime may already be down at exit
  return *r;
}

static double wall() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The count kernel's geometry for n bytes: workgroup shape, tiles per workgroup.
struct CountShape {
  int kind;   // 0 narrow (256 threads, 2 a CU), 1 wide (512), 2 xwide (768)
  bool wide;  // one workgroup a CU
  int threads;
  u64 tile_bytes, ntiles, per;
};
static CountShape count_shape(size_t n, int cus) {
  const char* wenv = std::getenv("SHREDWORD_LOAD_WIDE");
  CountShape c;
  c.kind = wenv ? std::max(0, std::min(2, std::atoi(wenv))) : kLoadShapeDefault;
  c.wide = c.kind != 0;
  c.threads = c.kind == 2 ? kXWideThreads : c.kind == 1 ? kWideThreads : kNarrowThreads;
  c.tile_bytes = (u64)kChunkBytes * (u64)c.threads;
  c.ntiles = (n + c.tile_bytes - 1) / c.tile_bytes;
  u64 grid = std::min<u64>(std::max<u64>(c.ntiles, 1), (u64)cus * (c.wide ? 1 : 2));
  c.per = (c.ntiles + grid - 1) / grid;
  while (c.per * c.tile_bytes >= (1ull << 32)) {  // LDS first offsets are 32-bit range-relative
    grid *= 2;
    c.per = (c.ntiles + grid - 1) / grid;
  }
  if (c.per == 0) c.per = 1;
  return c;
}
// k_word_count over tiles [tile0, tile1).
// per: tiles per workgroup (0: the whole-text shape's).
static void count_launch(const CountShape& c, const uint8_t* db, size_t n, const Table& t, u64 seed, u64 kmask,
                         u64 tile0, u64 tile1, u64 safe_end, hipStream_t st, u64 per = 0) {
  if (tile1 <= tile0) return;
  if (!per) per = c.per;
  const u64 grid = (tile1 - tile0 + per - 1) / per;
  // LDS eviction trigger (slots in use); SHREDWORD_LOAD_EVICT=<percent of the slots>, 0 = off
  uint32_t evict_pct = kLoadEvictPctDefault;
  if (const char* e = std::getenv("SHREDWORD_LOAD_EVICT")) evict_pct = (uint32_t)std::max(0, std::min(100, std::atoi(e)));
  const uint32_t slots = c.kind == 0 ? kNarrowSlots : kWideSlots;
  const uint32_t evict_at = evict_pct ? std::max<uint32_t>(1, slots * evict_pct / 100) : 0u;
  if (c.kind == 2)
    k_word_count<kXWideThreads, kWideSlots><<<(unsigned)grid, kXWideThreads, 0, st>>>(db, n, t, seed, kmask, per, tile0,
                                                                                      tile1, safe_end, evict_at);
  else if (c.wide)
    k_word_count<kWideThreads, kWideSlots><<<(unsigned)grid, kWideThreads, 0, st>>>(db, n, t, seed, kmask, per, tile0,
                                                                                    tile1, safe_end, evict_at);
  else
    k_word_count<kNarrowThreads, kNarrowSlots><<<(unsigned)grid, kNarrowThreads, 0, st>>>(db, n, t, seed, kmask, per,
                                                                                          tile0, tile1, safe_end, evict_at);
}
static u64 count_table_slots(size_t n) {
  // a power of two >= 1 M and >= n / 8192 (grown 4x while it is over 3/4 full): a small table
  // keeps the slots the spills touch in L2 / MALL
  u64 cap = 1ull << 20;
  while (cap < (u64)(n / 8192) && cap < (1ull << 29)) cap <<= 1;
  if (const char* e = std::getenv("SHREDWORD_LOAD_TABLE_SLOTS")) {  // tests: a table that must grow
    const u64 want = std::strtoull(e, nullptr, 10);
    if (want >= 1024) {
      cap = 1024;
      while (cap < want && cap < (1ull << 29)) cap <<= 1;
    }
  }
  return cap;
}
static u64 count_key_mask() {
  u64 kmask = ~0ull;
  if (const char* e = std::getenv("SHREDWORD_LOAD_KEY_BITS")) {
    const int bits = std::atoi(e);
    if (bits > 0 && bits < 64) kmask = (1ull << bits) - 1;
  }
  return kmask;
}
static u64 count_seed(int attempt) { return 0x51ED270B27A1F4A3ull * (u64)(attempt + 1); }

// A count's device table (slots + meta) that outlives one attempt (the segmented count of
// gpu_count_file hands its table to count_on_device).
struct CountTable {
  DevBuf slot, meta;
  u64 cap = 0;
  Table t{};
};
static bool count_table_alloc(CountTable* ct, u64 cap, hipStream_t st, std::string* why) {
  if (ct->slot.p) (void)hipFree(ct->slot.p);
  if (ct->meta.p) (void)hipFree(ct->meta.p);
  ct->slot.p = ct->meta.p = nullptr;
  LOAD_OK(hipMalloc(&ct->slot.p, cap * sizeof(Slot)));
  LOAD_OK(hipMalloc(&ct->meta.p, 64));
  LOAD_OK(hipMemsetAsync(ct->slot.p, 0, cap * sizeof(Slot), st));
  LOAD_OK(hipMemsetAsync(ct->meta.p, 0, 64, st));
  ct->cap = cap;
  ct->t.slot = (Slot*)ct->slot.p;
  ct->t.mask = cap - 1;
  ct->t.nkeys = (uint32_t*)ct->meta.p;
  ct->t.flags = (uint32_t*)ct->meta.p + 4;
  ct->t.stats = (u64*)ct->meta.p + 4;
  return true;
}

// The count of text already in HBM (db[0, n), ' ' padding after it): records in reference word
// order, and (spell) the spellings packed in that order.  *nul: the text holds a NUL byte (the
// records are then not made).  pre: a table already counted (attempt 0, seed 0) or nullptr.
static bool count_on_device(uint8_t* db, size_t n, hipStream_t st, int cus, bool report, double t0, double t1,
                            std::vector<WordRec>* out, std::vector<uint8_t>* spell, bool* nul, std::string* why,
                            CountTable* pre = nullptr, size_t table_n = 0) {
  u64 cap = count_table_slots(std::max(n, table_n));
  const u64 kmask = count_key_mask();
  const CountShape shape = count_shape(n, cus);
  if (nul) *nul = false;
  CountTable own;
  for (int attempt = 0; attempt < 6; ++attempt) {
    const u64 seed = count_seed(attempt);
    CountTable* ct = nullptr;
    if (attempt == 0 && pre) {
      ct = pre;
      cap = pre->cap;
    } else {
      if (!count_table_alloc(&own, cap, st, why)) return false;
      ct = &own;
      count_launch(shape, db, n, ct->t, seed, kmask, 0, shape.ntiles, ~0ull, st);
      LOAD_OK(hipGetLastError());
    }
    const Table& t = ct->t;
    uint32_t meta[16];
    LOAD_OK(hipMemcpyAsync(meta, ct->meta.p, 64, hipMemcpyDeviceToHost, st));
    LOAD_OK(hipStreamSynchronize(st));
    const double t2 = wall();
    const uint32_t W = meta[0];
    if (meta[6]) {  // a NUL byte: the reference reads such lines only up to it (host path)
      if (nul) *nul = true;
      if (why) *why = "the text holds NUL bytes";
      return false;
    }
    if (report) {
      const u64* ms = reinterpret_cast<const u64*>(meta) + 4;
      std::fprintf(stderr, "[LOAD] count attempt %d: %llu words, %.2f%% counted straight in HBM, %.2f%% long words "
                   "compared in HBM, %llu LDS slots evicted\n", attempt, (unsigned long long)ms[0],
                   100.0 * (double)ms[1] / (double)std::max<u64>(1, ms[0]),
                   100.0 * (double)ms[2] / (double)std::max<u64>(1, ms[0]), (unsigned long long)ms[3]);
    }
    if (report && (meta[4] || meta[5] || meta[7]))
      std::fprintf(stderr, "[LOAD] count attempt %d over %zu bytes repeated:%s%s%s (%.1f ms)\n", attempt, n,
                   meta[4] ? " table too full" : "", meta[5] ? " key collision" : "",
                   meta[7] ? " a word past a segment's landed bytes" : "", 1e3 * (t2 - t1));
    if (meta[4]) {  // too full: a bigger table
      if (cap >= (1ull << 29)) break;
      cap <<= 2;
      continue;
    }
    if (meta[5] || meta[7]) continue;  // a 64-bit key collision (another seed), or a segment's word past its bytes
    // reference word order: (djb2 & 4095, first offset); the keys are distinct
    DevBuf bk, bs, bk2, bs2, bn, btmp, brec;
    LOAD_OK(hipMalloc(&bk.p, (size_t)W * 8 + 8));
    LOAD_OK(hipMalloc(&bs.p, (size_t)W * 4 + 4));
    LOAD_OK(hipMalloc(&bk2.p, (size_t)W * 8 + 8));
    LOAD_OK(hipMalloc(&bs2.p, (size_t)W * 4 + 4));
    LOAD_OK(hipMalloc(&bn.p, 4));
    LOAD_OK(hipMemsetAsync(bn.p, 0, 4, st));
    k_word_compact<<<cus * 4, 256, 0, st>>>(t, (u64*)bk.p, (uint32_t*)bs.p, (uint32_t*)bn.p);
    LOAD_OK(hipGetLastError());
    size_t tmp_bytes = 0, tb2 = 0;
    LOAD_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, (u64*)bk.p, (u64*)bk2.p, (uint32_t*)bs.p,
                                               (uint32_t*)bs2.p, (int)W, 0, 64, st));
    LOAD_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, (u64*)bk.p, (u64*)bk2.p, (int)W + 1, st));
    tmp_bytes = std::max(tmp_bytes, tb2);
    LOAD_OK(hipMalloc(&btmp.p, tmp_bytes + 16));
    LOAD_OK(hipcub::DeviceRadixSort::SortPairs(btmp.p, tmp_bytes, (u64*)bk.p, (u64*)bk2.p, (uint32_t*)bs.p,
                                               (uint32_t*)bs2.p, (int)W, 0, 64, st));
    LOAD_OK(hipMalloc(&brec.p, (size_t)W * sizeof(WordRec) + sizeof(WordRec)));
    k_word_gather<<<cus * 4, 256, 0, st>>>(t, (const uint32_t*)bs2.p, W, (WordRec*)brec.p);
    LOAD_OK(hipGetLastError());
    out->resize(W);
    if (W) LOAD_OK(hipMemcpyAsync(out->data(), brec.p, (size_t)W * sizeof(WordRec), hipMemcpyDeviceToHost, st));
    if (spell) {  // the spellings in rank order: lengths -> offsets (bk: lengths, bk2: offsets) -> bytes
      LOAD_OK(hipMemsetAsync(bk.p, 0, (size_t)W * 8 + 8, st));
      k_word_lens<<<cus * 4, 256, 0, st>>>((const WordRec*)brec.p, W, (u64*)bk.p);
      LOAD_OK(hipGetLastError());
      LOAD_OK(hipcub::DeviceScan::ExclusiveSum(btmp.p, tb2, (u64*)bk.p, (u64*)bk2.p, (int)W + 1, st));
      u64 S = 0;
      LOAD_OK(hipMemcpyAsync(&S, (u64*)bk2.p + W, 8, hipMemcpyDeviceToHost, st));
      LOAD_OK(hipStreamSynchronize(st));
      DevBuf bsp;
      LOAD_OK(hipMalloc(&bsp.p, S + 16));
      k_word_spell<<<cus * 4, 256, 0, st>>>(db, (const WordRec*)brec.p, (const u64*)bk2.p, W, (uint8_t*)bsp.p);
      LOAD_OK(hipGetLastError());
      spell->resize(S);
      if (S) LOAD_OK(hipMemcpyAsync(spell->data(), bsp.p, S, hipMemcpyDeviceToHost, st));
      LOAD_OK(hipStreamSynchronize(st));
    }
    LOAD_OK(hipStreamSynchronize(st));
    if (report)
      std::fprintf(stderr, "[LOAD] %zu bytes: upload %.1f ms, count %.1f ms%s, order+gather%s %.1f ms, %u words\n", n,
                   1e3 * (t1 - t0), 1e3 * (t2 - t1), attempt == 0 && pre ? " (past the overlapped upload)" : "",
                   spell ? "+spellings" : "", 1e3 * (wall() - t2), W);
    return true;
  }
  if (why) *why = "the device word table did not converge";
  return false;
}

// The allowed CPUs on the GPU's NUMA node (its PCI device's local_cpulist), empty when unknown:
// the reader threads run there, so their pinned buffers and copies stay on the GPU's socket.
static std::vector<int> gpu_local_cpus(int device) {
  std::vector<int> out;
  char bus[64] = {};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return out;
  for (char* c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
  const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist";
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return out;
  char buf[4096] = {};
  const size_t got = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[got] = 0;
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return out;
  for (char* tok = std::strtok(buf, ",\n"); tok; tok = std::strtok(nullptr, ",\n")) {
    int lo = 0, hi = 0;
    if (std::sscanf(tok, "%d-%d", &lo, &hi) == 2) {
    } else if (std::sscanf(tok, "%d", &lo) == 1) {
      hi = lo;
    } else {
      continue;
    }
    for (int c = lo; c <= hi && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) out.push_back(c);
  }
  return out;
}

static bool device_setup(int device, hipStream_t* st, int* cus, std::string* why) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
    if (why) *why = "no HIP device";
    return false;
  }
  LOAD_OK(hipSetDevice(device));
  LOAD_OK(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
  hipDeviceProp_t prop;
  LOAD_OK(hipGetDeviceProperties(&prop, device));
  *cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  return true;
}

struct StreamGuard {
  hipStream_t s = nullptr;
  ~StreamGuard() {
    if (!s) return;
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
  }
};

bool gpu_count_words(int device, const uint8_t* d, size_t n, std::vector<WordRec>* out, std::string* why,
                     bool staged) {
  out->clear();
  const bool report = std::getenv("SHREDWORD_LOAD_REPORT") != nullptr;
  const double t0 = wall();
  if (n == 0) return true;
  if (n >= (1ull << 52)) {
    if (why) *why = "corpus larger than 2^52 bytes";
    return false;
  }
  StreamGuard sg;
  int cus = 256;
  if (!device_setup(device, &sg.s, &cus, why)) return false;
  hipStream_t st = sg.s;
  if (report) std::fprintf(stderr, "[LOAD] range of %zu bytes at %p: device setup %.1f ms\n", n, (const void*)d,
                           1e3 * (wall() - t0));
  DevBuf dd;
  LOAD_OK(hipMalloc(&dd.p, n + kPadBytes));
  uint8_t* db = static_cast<uint8_t*>(dd.p);
  LOAD_OK(hipMemsetAsync(db + n, ' ', kPadBytes, st));
  if (staged) {
    // A byte range inside the mapped file (a sharded load): the runtime's pageable copy of such a
    // range measured ~35 MB/s on MI355X boxes (the whole mapping from its start: ~20 GB/s), so
    // the range goes through two pinned 64 MiB buffers, filled by the CPU in turn.
    constexpr size_t kChunk = 64u << 20;
    void* pin[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool ok = true;
    for (int k = 0; k < 2 && ok; ++k)
      ok = hipHostMalloc(&pin[k], kChunk, hipHostMallocDefault) == hipSuccess &&
           hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) == hipSuccess;
    int k = 0;
    for (size_t off = 0; ok && off < n; off += kChunk, k ^= 1) {
      if (off >= 2 * kChunk) ok = hipEventSynchronize(ev[k]) == hipSuccess;  // buffer k is free again
      const size_t len = std::min(kChunk, n - off);
      std::memcpy(pin[k], d + off, len);
      ok = ok && hipMemcpyAsync(db + off, pin[k], len, hipMemcpyHostToDevice, st) == hipSuccess &&
           hipEventRecord(ev[k], st) == hipSuccess;
    }
    ok = hipStreamSynchronize(st) == hipSuccess && ok;
    for (int j = 0; j < 2; ++j) {
      if (ev[j]) (void)hipEventDestroy(ev[j]);
      if (pin[j]) (void)hipHostFree(pin[j]);
    }
    if (!ok) {
      if (why) *why = "staged upload failed";
      return false;
    }
  } else {
    LOAD_OK(hipMemcpyAsync(db, d, n, hipMemcpyHostToDevice, st));
  }
  if (report) LOAD_OK(hipStreamSynchronize(st));
  return count_on_device(db, n, st, cus, report, t0, wall(), out, nullptr, nullptr, why);
}

bool gpu_count_file(int device, int fd, uint64_t base, size_t n, std::vector<WordRec>* out,
                    std::vector<uint8_t>* spell, bool* nul, std::string* why) {
  out->clear();
  spell->clear();
  *nul = false;
  const bool report = std::getenv("SHREDWORD_LOAD_REPORT") != nullptr;
  const double t0 = wall();
  if (n == 0) return true;
  if (n >= (1ull << 52)) {
    if (why) *why = "corpus larger than 2^52 bytes";
    return false;
  }
  // 32 MiB chunks: the ring pins in half the time of 64 MiB ones and one stream still moves them
  // at full rate (round 5 A/B, 3 loads each: C3 0.52-0.56 s against 0.53-0.63 s; C5 100 GB
  // 2.85-2.90 against 2.84-2.85 s; profiles/r05_load_chunk_ab.txt)
  size_t chunk = (size_t)32 << 20;
  if (const char* e = std::getenv("SHREDWORD_LOAD_CHUNK_MB")) chunk = std::max<size_t>(1, std::strtoull(e, nullptr, 10)) << 20;
  const size_t nchunks = (n + chunk - 1) / chunk;
  int NB = 4;  // chunks in flight: read, queued for DMA, in DMA
  if (const char* e = std::getenv("SHREDWORD_LOAD_BUFS")) NB = std::max(2, std::min(16, std::atoi(e)));
  NB = (int)std::min<size_t>((size_t)NB, nchunks);
  // the pinned ring: reused, or (re)allocated on a helper thread meanwhile
  PinRing& ring = pin_ring();
  std::unique_lock<std::mutex> ring_lock(ring.mu);
  std::thread pin_thread;
  if (ring.chunk != chunk || ring.buf.size() < (size_t)NB) {
    for (void* q : ring.buf)
      if (q) (void)hipHostFree(q);
    ring.buf.assign((size_t)NB, nullptr);
    ring.chunk = chunk;
    ring.ready.reset(new std::atomic<int>[(size_t)NB]);
    for (int k = 0; k < NB; ++k) ring.ready[k].store(0);
    pin_thread = std::thread([&ring, device, NB, chunk] {
      bool ok = hipSetDevice(device) == hipSuccess;
      for (int k = 0; k < NB; ++k) {
        ok = ok && hipHostMalloc(&ring.buf[(size_t)k], chunk, hipHostMallocDefault) == hipSuccess;
        if (!ok) ring.buf[(size_t)k] = nullptr;
        ring.ready[k].store(ok ? 1 : 2, std::memory_order_release);
      }
    });
  }
  struct JoinGuard {
    std::thread& t;
    PinRing& r;
    ~JoinGuard() {
      if (!t.joinable()) return;
      t.join();
      for (size_t k = 0; k < r.buf.size(); ++k)  // a failed allocation: the next load starts over
        if (r.ready[k].load() != 1) r.chunk = 0;
    }
  } pin_join{pin_thread, ring};
  StreamGuard sg;
  int cus = 256;
  if (!device_setup(device, &sg.s, &cus, why)) return false;
  hipStream_t st = sg.s;
  DevBuf dd;
  LOAD_OK(hipMalloc(&dd.p, n + kPadBytes));
  uint8_t* db = static_cast<uint8_t*>(dd.p);
  LOAD_OK(hipMemsetAsync(db + n, ' ', kPadBytes, st));
  LOAD_OK(hipStreamSynchronize(st));
  const double t_buf = wall();
  // The file straight into HBM (round 5): a ring of NB pinned buffers of `chunk` bytes; T reader
  // threads fill each chunk together (a slice each, pread) and one copy thread sends the full
  // chunks, in order, over ONE stream.  Measured on the box (tools/h2d_probe.py): 32 MiB copies
  // reach 44 GB/s on one stream but 29 GB/s spread over 8, and pread from the page cache scales
  // to 52 GB/s at 8 threads -- round 4's reader-per-stream design sat at 12-14 GB/s.  No mapping of
  // the file (the page-ins of an mmap and the runtime's pageable staging bound that).  Overlap:
  // the count runs on segments (whole tiles) as they land -- segment k once every chunk up to the
  // end of segment k + 1 is in HBM (a word may run into the next segment; one running further is
  // flagged and the whole count is repeated after the upload).
  // 16 readers: the same rate as 8 once the file's pages are local (C3 0.51-0.55 s, C5 2.81-2.84 s
  // either way), and 18% faster on the first read of freshly written tmpfs pages (C5 100 GB right
  // after the generator: 4.99 s against 5.89 s; profiles/r05_load_readers_ab.txt)
  int T = 16;
  if (const char* e = std::getenv("SHREDWORD_LOAD_READERS")) T = std::max(1, std::min(64, std::atoi(e)));
  // readers on the GPU's NUMA node (SHREDWORD_LOAD_NUMA=0: wherever the scheduler puts them)
  std::vector<int> local;
  {
    const char* e = std::getenv("SHREDWORD_LOAD_NUMA");
    if (!(e && e[0] == '0')) local = gpu_local_cpus(device);
  }
  const CountShape shape = count_shape(n, cus);
  // 512 MiB segments (round 6; 2 GiB before): the count of the last segment is what follows the
  // upload, 73-112 ms -> 18-49 ms at C3 (profiles/r06_load_ab.json).  (Round 6 also tried the
  // word's spelling in 64-B HBM slots, compared in place instead of at a linked occurrence: 12-16%
  // more count traffic, profiles/r06_count_pmc_ab.json; not kept.)
  u64 seg_bytes = (u64)512 << 20;
  if (const char* e = std::getenv("SHREDWORD_LOAD_SEGMENT_MB")) seg_bytes = std::max<u64>(1, std::strtoull(e, nullptr, 10)) << 20;
  const char* oenv = std::getenv("SHREDWORD_LOAD_OVERLAP");
  const u64 seg_tiles = std::max<u64>(1, seg_bytes / shape.tile_bytes);
  const u64 nseg = (shape.ntiles + seg_tiles - 1) / seg_tiles;
  const bool overlap = !(oenv && oenv[0] == '0') && nseg > 1;
  // A byte range of a larger file (a sharded load) holds about as many distinct words as the whole
  // file (Heaps' law: a 5 GB half of C3 has all of its 1.25 M): its table is sized by the file,
  // not by the range, or it overflows and the count runs twice.
  size_t table_n = n;
  {
    struct stat sb;
    if (fstat(fd, &sb) == 0 && sb.st_size > 0) table_n = std::max(n, (size_t)sb.st_size);
  }
  std::vector<hipEvent_t> ev(nchunks, nullptr);
  for (size_t c = 0; c < nchunks; ++c) LOAD_OK(hipEventCreateWithFlags(&ev[c], hipEventDisableTiming));
  struct EventsGuard {
    std::vector<hipEvent_t>& v;
    ~EventsGuard() {
      for (hipEvent_t e : v)
        if (e) (void)hipEventDestroy(e);
    }
  } eg{ev};
  std::vector<void*>& pin = ring.buf;
  StreamGuard cs;
  LOAD_OK(hipStreamCreateWithFlags(&cs.s, hipStreamNonBlocking));
  const double t_pin = wall();
  // recorded[c]: 1 once chunk c's copy is queued behind ev[c] (2: failed); filled[c]: readers done
  std::unique_ptr<std::atomic<int>[]> recorded(new std::atomic<int>[nchunks]);
  std::unique_ptr<std::atomic<int>[]> filled(new std::atomic<int>[nchunks]);
  for (size_t c = 0; c < nchunks; ++c) {
    recorded[c].store(0);
    filled[c].store(0);
  }
  std::vector<std::thread> pool;
  std::atomic<int> failed{0};
  std::atomic<uint64_t> read_ns{0};
  const size_t slice = ((chunk + (size_t)T - 1) / (size_t)T + 4095) & ~(size_t)4095;
  for (int ti = 0; ti < T; ++ti)
    pool.emplace_back([&, ti] {
      if (!local.empty()) {
        cpu_set_t cpus;
        CPU_ZERO(&cpus);
        for (int c : local) CPU_SET(c, &cpus);
        (void)sched_setaffinity(0, sizeof(cpus), &cpus);
      }
      bool ok = hipSetDevice(device) == hipSuccess;
      for (size_t c = 0; c < nchunks; ++c) {
        const size_t off = c * chunk, len = std::min(chunk, n - off);
        const size_t s0 = std::min(len, (size_t)ti * slice), s1 = std::min(len, s0 + slice);
        if (ok && !failed.load(std::memory_order_relaxed) && s1 > s0) {
          if (c >= (size_t)NB) {  // the buffer is free once chunk c - NB's copy is done
            int r;
            while ((r = recorded[c - NB].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
            ok = r == 1 && hipEventSynchronize(ev[c - NB]) == hipSuccess;
          } else {  // the buffer's first use: pinned yet?
            int r;
            while ((r = ring.ready[c].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
            ok = r == 1;
          }
          uint8_t* dst = static_cast<uint8_t*>(pin[c % (size_t)NB]);
          const double tr = wall();
          size_t got = s0;
          while (ok && got < s1) {
            const ssize_t r = ::pread(fd, dst + got, s1 - got, (off_t)(base + off + got));
            if (r <= 0) ok = false;
            else got += (size_t)r;
          }
          read_ns.fetch_add((uint64_t)(1e9 * (wall() - tr)), std::memory_order_relaxed);
        }
        if (!ok) failed.store(1);
        filled[c].fetch_add(1, std::memory_order_acq_rel);
      }
    });
  // the copy thread: every full chunk, in order, on one stream
  pool.emplace_back([&] {
    bool ok = hipSetDevice(device) == hipSuccess;
    for (size_t c = 0; c < nchunks; ++c) {
      while (filled[c].load(std::memory_order_acquire) < T) std::this_thread::yield();
      ok = ok && !failed.load(std::memory_order_relaxed);
      const size_t off = c * chunk, len = std::min(chunk, n - off);
      ok = ok && hipMemcpyAsync(db + off, pin[c % (size_t)NB], len, hipMemcpyHostToDevice, cs.s) == hipSuccess &&
           hipEventRecord(ev[c], cs.s) == hipSuccess;
      if (!ok) failed.store(1);
      recorded[c].store(ok ? 1 : 2, std::memory_order_release);
    }
    if (hipStreamSynchronize(cs.s) != hipSuccess) failed.store(1);
  });
  // the segmented count on this thread's stream, behind the chunks' events
  CountTable pre;
  bool pre_ok = false;
  if (overlap) {
    pre_ok = count_table_alloc(&pre, count_table_slots(table_n), st, why);
    size_t waited = 0;  // chunks [0, waited) are behind an event wait on st
    for (u64 k = 0; pre_ok && k < nseg; ++k) {
      const u64 tile0 = k * seg_tiles, tile1 = std::min(shape.ntiles, tile0 + seg_tiles);
      const u64 reach = std::min<u64>(n, std::min(shape.ntiles, tile1 + seg_tiles) * shape.tile_bytes);
      const size_t need = k + 1 == nseg ? nchunks : (size_t)((reach + chunk - 1) / chunk);
      for (; waited < need; ++waited) {
        int r;
        while ((r = recorded[waited].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
        if (r != 1) {
          pre_ok = false;
          break;
        }
        if (hipStreamWaitEvent(st, ev[waited], 0) != hipSuccess) pre_ok = false;
      }
      if (!pre_ok) break;
      const u64 safe_end = k + 1 == nseg ? ~0ull : (u64)need * chunk;
      // a segment over the whole chip (a workgroup per CU: shape.per would leave most idle)
      const u64 per_seg = std::max<u64>(1, (tile1 - tile0 + (u64)cus * (shape.wide ? 1 : 2) - 1) /
                                               ((u64)cus * (shape.wide ? 1 : 2)));
      count_launch(shape, db, n, pre.t, count_seed(0), count_key_mask(), tile0, tile1, safe_end, st, per_seg);
      if (hipGetLastError() != hipSuccess) pre_ok = false;
    }
  }
  for (auto& th : pool) th.join();
  if (failed.load()) {
    if (why) *why = "reading / uploading the file failed";
    return false;
  }
  const double t1 = wall();
  if (report)
    std::fprintf(stderr, "[LOAD] file_to_hbm setup: device + text buffer %.1f ms (the pinned ring meanwhile), events + copy stream "
                 "%.1f ms\n",
                 1e3 * (t_buf - t0), 1e3 * (t_pin - t_buf));
  if (report)
    std::fprintf(stderr, "[LOAD] phase file_to_hbm %.1f ms (%d readers, %d pinned %zu MiB chunks, one copy stream, readers "
                 "on %zu GPU-local CPUs, pread %.1f ms summed over readers): %.1f GB/s%s\n", 1e3 * (t1 - t0), T, NB,
                 chunk >> 20, local.size(), 1e-6 * (double)read_ns.load(), (double)n / (t1 - t0) / 1e9,
                 overlap ? "; the count ran on segments meanwhile" : "");
  if (!count_on_device(db, n, st, cus, report, t0, t1, out, spell, nul, why, pre_ok ? &pre : nullptr, table_n))
    return false;
  if (base)
    for (WordRec& w : *out) w.first += base;  // file offsets
  if (report) std::fprintf(stderr, "[LOAD] file count done at %.1f ms (teardown follows)\n", 1e3 * (wall() - t0));
  return true;
}

}  // namespace shred
