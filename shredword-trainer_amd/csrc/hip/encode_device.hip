// BPE encoder on gfx950 (C ABI include/shredword_encode.h).
//
// Applies a trained merge list to text.  The replay the trainer performs (merge m over every word
// left to right, reference bpe.cpp:265-296, for m = 0, 1, ...) equals, per word, "merge the
// leftmost adjacent pair of lowest rank until no pair has a rank": a pair created by merge m
// involves the new id 256 + m, so its rank is > m, and no earlier rank can reappear.  The
// kernels therefore encode every word independently:
//
//   k_encode_words  one thread per 32-byte span takes the words that START in it (maximal runs
//                   outside "\t\r\n ", found with a 32-bit delimiter mask of the span), maps
//                   bytes through the byte map, and runs the lowest-rank loop on a per-thread
//                   LDS strip of tokens and cached pair ranks (words <= 32 bytes), or in global
//                   scratch (longer words, <= kEncMaxWord).  Pair ranks come from a read-only
//                   open-addressing table of u64 slots (L2-resident: 16 K slots = 128 KB for
//                   8 K merges).  A thread packs its words' ids at its first word start, so the
//                   spans of different threads never overlap; per-thread and per-block counts.
//   hipCUB scan     inclusive block sums (the last is the total).
//   k_encode_emit   one workgroup per block copies its threads' runs to the output in text
//                   order: each output slot finds its thread by binary search over the block's
//                   inclusive scan, so the stores are coalesced.
// Traffic per text byte: 1 B read + 4 B x (ids / byte) x 3 (pack write, emit read, emit write)
// + 0.125 B of counts; algorithmic: 1 B + 4 B x ids / byte.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../host/encoder.h"

namespace shred {
namespace {

typedef uint64_t u64;

constexpr int kThreads = 128;              // threads per workgroup
constexpr int kSpan = 32;                  // bytes whose word starts one thread owns
constexpr int kChunk = kThreads * kSpan;   // bytes per workgroup
constexpr int kStrip = 32;                 // tokens a word keeps in LDS (32 KB per workgroup)
constexpr int kInf = 0x7fffffff;

__device__ __forceinline__ uint32_t is_delim(uint32_t c) { return c == 9u || c == 13u || c == 10u || c == 32u; }

__device__ __forceinline__ int pair_rank(const u64* __restrict__ tab, u64 mask, int a, int b) {
  if ((uint32_t)a >= (uint32_t)kEncIdLimit || (uint32_t)b >= (uint32_t)kEncIdLimit) return kInf;
  const u64 key = (u64)(uint32_t)a << 20 | (u64)(uint32_t)b;
  for (u64 i = ((key * 0x9E3779B97F4A7C15ull) >> 24) & mask;; i = (i + 1) & mask) {
    const u64 e = tab[i];
    if (e == kEncEmpty) return kInf;
    if ((e >> 20) == key) return (int)(e & 0xFFFFFu);
  }
}

// Lowest-rank merging of tok[0..m) with cached ranks rk[0..m-1) (LDS strip or global scratch).
// Returns the final length.
template <typename Tok>
__device__ __forceinline__ int merge_word(Tok tok, Tok rk, int m, const u64* __restrict__ tab, u64 mask) {
  for (int j = 0; j + 1 < m; ++j) rk(j) = pair_rank(tab, mask, tok(j), tok(j + 1));
  while (m > 1) {
    int best = kInf, p = -1;
    for (int j = 0; j + 1 < m; ++j) {
      const int r = rk(j);
      if (r < best) { best = r; p = j; }
    }
    if (best == kInf) break;
    tok(p) = 256 + best;
    for (int j = p + 1; j + 1 < m; ++j) tok(j) = tok(j + 1);
    for (int j = p + 1; j + 2 < m; ++j) rk(j) = rk(j + 1);
    --m;
    if (p > 0) rk(p - 1) = pair_rank(tab, mask, tok(p - 1), tok(p));
    if (p + 1 < m) rk(p) = pair_rank(tab, mask, tok(p), tok(p + 1));
  }
  return m;
}

// Packed form for vocabularies below 2^16 ids: LDS entry j = tok_j << 16 | rank of (tok_j, tok_j+1)
// (0xFFFF: none), one word per position, so a strip takes half the LDS (twice the occupancy) and
// a shift moves token and rank together.  e points at the thread's column (stride kThreads).
__device__ __forceinline__ uint32_t rank16(const u64* __restrict__ tab, u64 mask, uint32_t a, uint32_t b) {
  const int r = pair_rank(tab, mask, (int)a, (int)b);
  return r == kInf ? 0xFFFFu : (uint32_t)r;
}

__device__ __forceinline__ int merge_word_packed(uint32_t* e, int m, const u64* __restrict__ tab, u64 mask) {
#define E(j) e[(j) * kThreads]
  for (int j = 0; j + 1 < m; ++j) E(j) |= rank16(tab, mask, E(j) >> 16, E(j + 1) >> 16);
  E(m - 1) |= 0xFFFFu;
  while (m > 1) {
    uint32_t best = 0xFFFFu;
    int p = -1;
    for (int j = 0; j + 1 < m; ++j) {
      const uint32_t r = E(j) & 0xFFFFu;
      if (r < best) { best = r; p = j; }
    }
    if (p < 0) break;
    const uint32_t x = 256u + best;
    for (int j = p + 1; j + 1 < m; ++j) E(j) = E(j + 1);
    --m;
    E(p) = x << 16 | (p + 1 < m ? rank16(tab, mask, x, E(p + 1) >> 16) : 0xFFFFu);
    if (p > 0) E(p - 1) = (E(p - 1) & 0xFFFF0000u) | rank16(tab, mask, E(p - 1) >> 16, x);
  }
#undef E
  return m;
}

struct LdsRef {
  int* base;
  __device__ __forceinline__ int& operator()(int j) const { return base[j * kThreads]; }
};
struct GlobalRef {
  int* base;
  __device__ __forceinline__ int& operator()(int j) const { return base[j]; }
};

template <bool kAligned, bool kPacked>
__global__ __launch_bounds__(kThreads) void k_encode_words(const uint8_t* __restrict__ text, u64 n,
                                                           const int32_t* __restrict__ byte_map,
                                                           const u64* __restrict__ tab, u64 mask,
                                                           int32_t* __restrict__ pad, int32_t* __restrict__ rank,
                                                           uint32_t* __restrict__ tcnt, u64* __restrict__ bcnt,
                                                           u64* __restrict__ misc) {
  __shared__ int s_map[256];
  __shared__ int s_strip[(kPacked ? 1 : 2) * kStrip * kThreads];
  __shared__ uint32_t s_sum;
  const int tid = threadIdx.x;
  for (int i = tid; i < 256; i += kThreads) s_map[i] = byte_map[i];
  if (tid == 0) s_sum = 0;
  __syncthreads();

  const u64 base = (u64)blockIdx.x * kChunk + (u64)tid * kSpan;
  uint32_t cnt = 0, j0 = 0;
  if (base < n) {
    const u64 lim = n - base < (u64)kSpan ? n - base : (u64)kSpan;
    uint32_t dm = 0;  // bit k: byte base + k is a delimiter (or past the end)
    if (kAligned && lim == (u64)kSpan) {
      const uint4* p = reinterpret_cast<const uint4*>(text + base);
      const uint4 v0 = p[0], v1 = p[1];
      const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int k = 0; k < kSpan; ++k) dm |= is_delim((w[k >> 2] >> (8 * (k & 3))) & 255u) << k;
    } else {
      for (int k = 0; k < kSpan; ++k) dm |= ((u64)k < lim ? is_delim(text[base + k]) : 1u) << k;
    }
    const uint32_t prevd = base == 0 ? 1u : is_delim(text[base - 1]);
    uint32_t starts = ~dm & ((dm << 1) | prevd);
    if (starts) j0 = __ffs(starts) - 1;
    u64 wpos = base + j0;
    LdsRef tok{s_strip + tid}, rk{s_strip + kStrip * kThreads + tid};
    while (starts) {
      const int j = __ffs(starts) - 1;
      starts &= starts - 1;
      const u64 s = base + j;
      const uint32_t above = dm >> j;  // bit 0 is clear: s starts a word
      u64 L;
      if (above) {
        L = __ffs(above) - 1;
      } else {  // runs past the span
        u64 e = base + kSpan;
        while (e < n && e - s <= (u64)kEncMaxWord && !is_delim(text[e])) ++e;
        L = e - s;
      }
      if (L > (u64)kEncMaxWord) {
        atomicOr(reinterpret_cast<unsigned long long*>(misc + 1), 1ull);
        continue;
      }
      int m;
      if (L <= (u64)kStrip) {
        if (kPacked) {
          uint32_t* e = reinterpret_cast<uint32_t*>(s_strip) + tid;
          for (int k = 0; k < (int)L; ++k) e[k * kThreads] = (uint32_t)s_map[text[s + k]] << 16;
          m = merge_word_packed(e, (int)L, tab, mask);
          for (int k = 0; k < m; ++k) pad[wpos + k] = (int)(e[k * kThreads] >> 16);
        } else {
          for (int k = 0; k < (int)L; ++k) tok(k) = s_map[text[s + k]];
          m = merge_word(tok, rk, (int)L, tab, mask);
          for (int k = 0; k < m; ++k) pad[wpos + k] = tok(k);
        }
      } else {
        GlobalRef gt{pad + s}, gr{rank + s};
        for (int k = 0; k < (int)L; ++k) gt(k) = s_map[text[s + k]];
        m = merge_word(gt, gr, (int)L, tab, mask);
        for (int k = 0; k < m; ++k) pad[wpos + k] = gt(k);  // wpos <= s: ascending copy is safe
      }
      wpos += m;
      cnt += m;
    }
  }
  tcnt[(u64)blockIdx.x * kThreads + tid] = cnt << 5 | j0;
  if (cnt) atomicAdd(&s_sum, cnt);
  __syncthreads();
  if (tid == 0) bcnt[blockIdx.x] = s_sum;
}

// ---- word cache: every distinct word is encoded once -------------------------------------
// A corpus repeats its words (C3: 1.13 G occurrences of 1.25 M distinct words), so the default
// path encodes each distinct word once and copies its ids to every occurrence:
//   k_cache_insert  per occurrence: 64-bit hash of (bytes, length) into an open-addressing table
//                   of 64-byte slots (key, payload = the inserting occurrence's offset, then the
//                   short word's bytes and ids inline): a read that hits L2 for a hot word, a CAS
//                   only for an empty slot; a full probe window flags an overflow (the table then
//                   grows 4x);
//   k_cache_encode  per used slot: the lowest-rank loop on that occurrence; the ids, then the
//                   word's bytes, go to a dense arena (one entry per distinct word), and the
//                   payload becomes (arena offset, length, id count);
//   k_cache_words   per occurrence: the slot (key and payload in one 16-byte load), a byte compare
//                   with the slot's inline copy (words <= 16 bytes with <= 8 ids: no arena read)
//                   or the arena's (a 64-bit collision is flagged, never trusted); then the
//                   block's ids are written as one contiguous run from its first word start
//                   (per-block count + start);
//   k_block_emit    one workgroup per block copies its run to the output, coalesced.
// An arena overflow or a collision reruns the call on the direct path (k_encode_words): exact
// always.  HBM traffic per text byte: 2 B of text reads (insert, words) + 4 B x ids / byte x 3
// (run write, emit read, emit write); the slot table and arena stay in L2/MALL for a corpus of
// repeated words.
constexpr int kCacheProbes = 128;
// A word-cache slot is one 64-byte line of 8 u64: [0] key, [1] payload (first the inserting
// occurrence's offset), [2..3] the word's bytes and [4..7] its ids inline when it is short
// (<= kInlineBytes bytes, <= kInlineIds ids; most occurrences at any vocab size), so a hot word
// costs k_cache_words one line -- which stays in L2 -- and no arena read.
constexpr int kSlotU64 = 8;
constexpr int kInlineBytes = 16;
constexpr int kInlineIds = 8;
constexpr int kSpanWords = kSpan / 2 + 1;  // words starting in one span, at most

// The chunk's text staged in LDS (coalesced 4-byte loads), with a few bytes before it and
// kOverhang after: word scans, hashes and compares read LDS, and global memory only for bytes
// outside the staged window.
constexpr int kOverhang = 256;
constexpr int kStageBytes = 4 + kChunk + kOverhang;

struct TextView {
  const uint8_t* __restrict__ g;
  const uint8_t* l;  // LDS copy of [lo, hi)
  u64 lo, hi;
  __device__ __forceinline__ uint32_t operator[](u64 i) const { return (i >= lo && i < hi) ? l[i - lo] : g[i]; }
};

__device__ __forceinline__ TextView stage_chunk(const uint8_t* __restrict__ text, u64 n, u64 chunk, uint32_t* lds) {
  const u64 cbase = chunk * kChunk;
  const u64 lo = cbase >= 4 ? cbase - 4 : 0;
  u64 hi = lo + kStageBytes;
  if (hi > n) hi = n;
  const u64 words = (hi - lo) / 4;
  for (u64 w = threadIdx.x; w < words; w += kThreads) {
    const uint8_t* p = text + lo + 4 * w;  // lo is 4-aligned; the text base may not be
    lds[w] = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
  }
  __syncthreads();
  return TextView{text, reinterpret_cast<const uint8_t*>(lds), lo, lo + 4 * words};
}

template <typename T>
__device__ __forceinline__ u64 word_hash(const T& t, u64 s, uint32_t L) {
  u64 h = 1469598103934665603ull;
  for (uint32_t k = 0; k < L; ++k) h = (h ^ t[s + k]) * 1099511628211ull;
  h ^= (u64)L * 0x9E3779B97F4A7C15ull;
  // FNV's multiplier barely mixes the middle bits the slot index uses: murmur3's fmix64 does
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h | 1ull;  // 0 marks an empty slot
}

// Calls f(s, L, j) for every word starting in the span at `base` (L may exceed kEncMaxWord).
template <typename T, typename F>
__device__ __forceinline__ void for_each_word(const T& text, u64 n, u64 base, F f) {
  if (base >= n) return;
  const u64 lim = n - base < (u64)kSpan ? n - base : (u64)kSpan;
  uint32_t dm = 0;
  for (int k = 0; k < kSpan; ++k) dm |= ((u64)k < lim ? is_delim(text[base + k]) : 1u) << k;
  const uint32_t prevd = base == 0 ? 1u : is_delim(text[base - 1]);
  uint32_t starts = ~dm & ((dm << 1) | prevd);
  while (starts) {
    const int j = __ffs(starts) - 1;
    starts &= starts - 1;
    const u64 s = base + j;
    const uint32_t above = dm >> j;
    u64 L;
    if (above) {
      L = __ffs(above) - 1;
    } else {
      u64 e = base + kSpan;
      while (e < n && e - s <= (u64)kEncMaxWord && !is_delim(text[e])) ++e;
      L = e - s;
    }
    f(s, L, j);
  }
}

__device__ __forceinline__ void flag(u64* misc, u64 bit) {
  atomicOr(reinterpret_cast<unsigned long long*>(misc + 1), (unsigned long long)bit);
}

__global__ __launch_bounds__(kThreads) void k_cache_insert(const uint8_t* __restrict__ text, u64 n,
                                                           u64* __restrict__ slot, u64 cmask, u64* __restrict__ misc) {
  __shared__ uint32_t s_text[kStageBytes / 4];
  const TextView tv = stage_chunk(text, n, blockIdx.x, s_text);
  const u64 base = (u64)blockIdx.x * kChunk + (u64)threadIdx.x * kSpan;
  for_each_word(tv, n, base, [&](u64 s, u64 L, int) {
    if (L > (u64)kEncMaxWord) {
      flag(misc, 1);
      return;
    }
    const u64 h = word_hash(tv, s, (uint32_t)L);
    u64 i = (h >> 17) & cmask;
    for (int p = 0; p < kCacheProbes; ++p, i = (i + 1) & cmask) {
      u64 k = slot[kSlotU64 * i];  // hot words: a read that hits L2, no atomic
      if (k == 0) {
        k = atomicCAS(reinterpret_cast<unsigned long long*>(slot + kSlotU64 * i), 0ull, (unsigned long long)h);
        if (k == 0) {
          slot[kSlotU64 * i + 1] = s;  // any occurrence spells the word (k_cache_words checks them all)
          return;
        }
      }
      if (k == h) return;
    }
    flag(misc, 2);  // window full
  });
}

// Payload of an encoded slot: arena offset (int32 units) | length << 32 | id count << 48.  The arena
// entry at that offset: a header (id count | length << 16), the ids, the word's bytes.
__device__ __forceinline__ u64 pack_payload(u64 off, u64 L, u64 m) { return off | L << 32 | m << 48; }

template <bool kPacked>
__global__ __launch_bounds__(kThreads) void k_cache_encode(const uint8_t* __restrict__ text, u64 n,
                                                           const int32_t* __restrict__ byte_map,
                                                           const u64* __restrict__ tab, u64 mask,
                                                           u64* __restrict__ slot, u64 cap,
                                                           int32_t* __restrict__ arena, u64 arena_cap,
                                                           int32_t* __restrict__ rank, u64* __restrict__ misc) {
  __shared__ int s_map[256];
  __shared__ int s_strip[(kPacked ? 1 : 2) * kStrip * kThreads];
  const int tid = threadIdx.x;
  for (int i = tid; i < 256; i += kThreads) s_map[i] = byte_map[i];
  __syncthreads();
  const u64 i = (u64)blockIdx.x * kThreads + tid;
  if (i >= cap || slot[kSlotU64 * i] == 0) return;
  const u64 s = slot[kSlotU64 * i + 1];
  u64 e = s;
  while (e < n && !is_delim(text[e])) ++e;  // <= kEncMaxWord (insert checked)
  const int L = (int)(e - s);
  const u64 need = 1 + (u64)L + (u64)(L + 3) / 4;  // header (m | L << 16), ids (<= L), then the bytes
  const u64 off = atomicAdd(reinterpret_cast<unsigned long long*>(misc + 2), (unsigned long long)need);
  if (off + need > arena_cap) {
    flag(misc, 8);  // arena full
    return;
  }
  int32_t* ids = arena + off + 1;
  int m;
  if (L <= kStrip) {
    if (kPacked) {
      uint32_t* q = reinterpret_cast<uint32_t*>(s_strip) + tid;
      for (int k = 0; k < L; ++k) q[k * kThreads] = (uint32_t)s_map[text[s + k]] << 16;
      m = merge_word_packed(q, L, tab, mask);
      for (int k = 0; k < m; ++k) ids[k] = (int)(q[k * kThreads] >> 16);
    } else {
      LdsRef tok{s_strip + tid}, rk{s_strip + kStrip * kThreads + tid};
      for (int k = 0; k < L; ++k) tok(k) = s_map[text[s + k]];
      m = merge_word(tok, rk, L, tab, mask);
      for (int k = 0; k < m; ++k) ids[k] = tok(k);
    }
  } else {  // tokens in the arena entry, ranks in scratch at the word's own text offset
    GlobalRef gt{ids}, gr{rank + s};
    for (int k = 0; k < L; ++k) gt(k) = s_map[text[s + k]];
    m = merge_word(gt, gr, L, tab, mask);
  }
  uint32_t* bytes = reinterpret_cast<uint32_t*>(ids + m);
  for (int k = 0; k < L; k += 4) {
    uint32_t w = 0;
    for (int b = 0; b < 4 && k + b < L; ++b) w |= (uint32_t)text[s + k + b] << (8 * b);
    bytes[k / 4] = w;
  }
  arena[off] = m | L << 16;
  u64* sl = slot + kSlotU64 * i;
  if (L <= kInlineBytes && m <= kInlineIds) {  // the bytes and the ids inline (zero-padded)
    u64 b[2] = {0, 0};
    for (int k = 0; k < L; ++k) b[k >> 3] |= (u64)text[s + k] << (8 * (k & 7));
    sl[2] = b[0];
    sl[3] = b[1];
    u64 w[kInlineIds / 2] = {0, 0, 0, 0};
    for (int k = 0; k < m; ++k) w[k >> 1] |= (u64)(uint32_t)ids[k] << (32 * (k & 1));
    for (int k = 0; k < kInlineIds / 2; ++k) sl[4 + k] = w[k];
  }
  sl[1] = pack_payload(off, (u64)L, (u64)m);
}

// Per occurrence: its word's cached ids, written straight to the output at the chunk's place.
// The chunk's place is its exclusive sum over the chunks before it, found by a decoupled
// look-back: chunks are taken in ticket order (a block never waits for one that has not started),
// each publishes its id count, then walks back over the predecessors' published counts until one
// that also published its inclusive sum (status 2), and publishes its own.  The states are 8-B
// agent atomics on both sides (cross-XCD coherent).  No staging copy of the ids.
constexpr u64 kLbValue = (1ull << 62) - 1;
__global__ __launch_bounds__(kThreads) void k_cache_words(const uint8_t* __restrict__ text, u64 n,
                                                          const u64* __restrict__ slot, u64 cmask,
                                                          const int32_t* __restrict__ arena, int32_t* __restrict__ out,
                                                          u64 out_cap, u64* __restrict__ bcnt, u64* __restrict__ lb,
                                                          u64 nb, u64* __restrict__ misc) {
  __shared__ uint32_t s_text[kStageBytes / 4];
  __shared__ uint32_t s_list[kSpanWords * kThreads];  // this chunk's words: arena offsets, column per thread
  __shared__ uint32_t s_inc[kThreads];
  __shared__ u64 s_chunk, s_prefix;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_chunk = __hip_atomic_fetch_add(lb + nb, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ticket
  }
  __syncthreads();
  const u64 chunk = s_chunk;
  const TextView tv = stage_chunk(text, n, chunk, s_text);  // synchronises
  const u64 cbase = chunk * kChunk;
  const u64 base = cbase + (u64)tid * kSpan;
  uint32_t cnt = 0, nw = 0;
  for_each_word(tv, n, base, [&](u64 s, u64 L, int) {
    if (L > (u64)kEncMaxWord) return;  // flagged by k_cache_insert
    const u64 h = word_hash(tv, s, (uint32_t)L);
    u64 pay = 0, i = (h >> 17) & cmask;
    for (int p = 0; p < kCacheProbes; ++p, i = (i + 1) & cmask) {
      const ulonglong2 sl = *reinterpret_cast<const ulonglong2*>(slot + kSlotU64 * i);  // key and payload: one load
      if (sl.x == h) {
        pay = sl.y;
        break;
      }
      if (sl.x == 0) break;
    }
    if (!pay) return;  // not inserted: an overflow, flagged by k_cache_insert / k_cache_encode
    const uint32_t m = (uint32_t)(pay >> 48), pl = (uint32_t)(pay >> 32) & 0xFFFFu;
    uint32_t diff = pl != (uint32_t)L;
    uint32_t entry;
    if (pl <= (uint32_t)kInlineBytes && m <= (uint32_t)kInlineIds) {  // inline: the slot's own line
      const ulonglong2 sb = *reinterpret_cast<const ulonglong2*>(slot + kSlotU64 * i + 2);
      for (uint32_t k = 0; k < pl && !diff; ++k)
        diff |= (uint32_t)(((k < 8 ? sb.x : sb.y) >> (8 * (k & 7))) & 0xFFu) ^ tv[s + k];
      entry = 0x80000000u | (uint32_t)i;  // (slot indices < 2^31: the table is far smaller)
    } else {
      const uint8_t* ab = reinterpret_cast<const uint8_t*>(arena + (uint32_t)pay + 1 + m);
      for (uint32_t k = 0; k < pl && !diff; ++k) diff |= ab[k] ^ tv[s + k];
      entry = (uint32_t)pay;
    }
    if (diff) {
      flag(misc, 4);  // 64-bit collision
      return;
    }
    s_list[nw * kThreads + tid] = entry;
    ++nw;
    cnt += m;
  });
  // block-inclusive scan of the per-thread id counts
  s_inc[tid] = cnt;
  __syncthreads();
  for (int d = 1; d < kThreads; d <<= 1) {
    const uint32_t v = tid >= d ? s_inc[tid - d] : 0;
    __syncthreads();
    s_inc[tid] += v;
    __syncthreads();
  }
  if (tid == 0) {
    const u64 agg = s_inc[kThreads - 1];
    u64 prefix = 0;
    if (chunk == 0) {
      __hip_atomic_exchange(lb, (2ull << 62) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_exchange(lb + chunk, (1ull << 62) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (u64 j = chunk - 1;;) {
        const u64 v = __hip_atomic_fetch_add(lb + j, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const u64 status = v >> 62;
        if (status == 0) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        prefix += v & kLbValue;
        if (status == 2 || j == 0) break;
        --j;
      }
      __hip_atomic_exchange(lb + chunk, (2ull << 62) | (prefix + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_prefix = prefix;
    bcnt[chunk] = agg;
    if (prefix + agg > out_cap) flag(misc, 16);  // the output is too small: nothing of this chunk is written
  }
  __syncthreads();
  if (s_prefix + s_inc[kThreads - 1] > out_cap) return;
  int32_t* dst = out + s_prefix + (s_inc[tid] - cnt);
  for (uint32_t w = 0; w < nw; ++w) {
    const uint32_t e = s_list[w * kThreads + tid];
    if (e & 0x80000000u) {  // inline ids: the slot line the lookup just read
      const u64* sl = slot + kSlotU64 * (u64)(e & 0x7FFFFFFFu);
      const uint32_t m = (uint32_t)(sl[1] >> 48);
      const int32_t* src = reinterpret_cast<const int32_t*>(sl + 4);
      for (uint32_t k = 0; k < m; ++k) dst[k] = src[k];
      dst += m;
      continue;
    }
    const int32_t* src = arena + e;
    const uint32_t m = (uint32_t)src[0] & 0xFFFFu;
    ++src;
    for (uint32_t k = 0; k < m; ++k) dst[k] = src[k];
    dst += m;
  }
}

__global__ __launch_bounds__(kThreads) void k_encode_emit(const int32_t* __restrict__ pad, const uint32_t* __restrict__ tcnt,
                                                          const u64* __restrict__ bcnt, int32_t* __restrict__ out) {
  __shared__ uint32_t s_inc[kThreads];
  __shared__ int s_src[kThreads];  // pad offset of each thread's run (block-relative) minus its exclusive count
  const int tid = threadIdx.x;
  const uint32_t t = tcnt[(u64)blockIdx.x * kThreads + tid];
  const uint32_t cnt = t >> 5;
  s_inc[tid] = cnt;
  __syncthreads();
  for (int d = 1; d < kThreads; d <<= 1) {
    const uint32_t v = tid >= d ? s_inc[tid - d] : 0;
    __syncthreads();
    s_inc[tid] += v;
    __syncthreads();
  }
  s_src[tid] = tid * kSpan + (int)(t & 31u) - (int)(s_inc[tid] - cnt);
  __syncthreads();
  const uint32_t total = s_inc[kThreads - 1];
  const u64 base = (u64)blockIdx.x * kChunk;
  int32_t* dst = out + (bcnt[blockIdx.x] - total);  // bcnt: inclusive block sums
  for (uint32_t i = tid; i < total; i += kThreads) {
    int lo = 0, hi = kThreads - 1;  // first thread whose inclusive count exceeds i
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_inc[mid] > i) hi = mid; else lo = mid + 1;
    }
    dst[i] = pad[(int64_t)base + s_src[lo] + (int64_t)i];
  }
}

#define ENC_OK(expr)                                                                            \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "[ERROR]\t encoder: %s: %s\n", #expr, hipGetErrorString(e_));        \
      return -1;                                                                                \
    }                                                                                           \
  } while (0)

}  // namespace

EncodeDevice* EncodeDevice::create(int device, const std::vector<uint64_t>& table, const int32_t* byte_map,
                                   std::string* why) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    *why = "no HIP device visible";
    return nullptr;
  }
  if (device < 0 || device >= count) {
    *why = "device ordinal " + std::to_string(device) + " out of range";
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    *why = "hipSetDevice failed";
    return nullptr;
  }
  EncodeDevice* d = new EncodeDevice();
  d->device_ = device;
  d->mask_ = table.size() - 1;
  // 16-bit packing needs every id (bytes' symbols and 256 + rank) below 0xFFFF: decided from the
  // largest rank in the table (a merge list with repeated pairs has ranks past its distinct pairs)
  uint64_t max_rank = 0;
  for (uint64_t e : table)
    if (e != kEncEmpty) max_rank = std::max<uint64_t>(max_rank, e & 0xFFFFFu);
  d->packed_ = 256 + max_rank < 0xFFFFu;
  for (int b = 0; b < 256; ++b) d->packed_ = d->packed_ && byte_map[b] >= 0 && byte_map[b] < 0xFFFF;
  hipStream_t st = nullptr;
  bool ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
  d->stream_ = st;
  ok = ok && hipMalloc(&d->table_, table.size() * 8) == hipSuccess;
  ok = ok && hipMalloc(&d->byte_map_, 256 * 4) == hipSuccess;
  ok = ok && hipMalloc(&d->misc_, 32) == hipSuccess;
  ok = ok && hipHostMalloc(&d->host_misc_, 16, hipHostMallocDefault) == hipSuccess;
  ok = ok && hipMemcpy(d->table_, table.data(), table.size() * 8, hipMemcpyHostToDevice) == hipSuccess;
  ok = ok && hipMemcpy(d->byte_map_, byte_map, 256 * 4, hipMemcpyHostToDevice) == hipSuccess;
  for (int i = 0; i < 4 && ok; ++i) {
    hipEvent_t e;
    ok = hipEventCreate(&e) == hipSuccess;
    d->ev_[i] = e;
  }
  if (!ok) {
    *why = "device allocation failed";
    delete d;
    return nullptr;
  }
  return d;
}

EncodeDevice::~EncodeDevice() {
  (void)hipSetDevice(device_);
  if (stream_) (void)hipStreamSynchronize((hipStream_t)stream_);
  for (void* p : {(void*)table_, (void*)byte_map_, (void*)misc_, (void*)pad_, (void*)rank_, (void*)tcnt_,
                  (void*)bcnt_, (void*)dtext_, (void*)dout_, (void*)cslot_, scan_tmp_})
    if (p) (void)hipFree(p);
  if (host_misc_) (void)hipHostFree(host_misc_);
  for (void* e : ev_)
    if (e) (void)hipEventDestroy((hipEvent_t)e);
  if (stream_) (void)hipStreamDestroy((hipStream_t)stream_);
}

bool EncodeDevice::reserve(size_t n, std::string* why) {
  if (n <= cap_bytes_) return true;
  for (void* p : {(void*)pad_, (void*)rank_, (void*)tcnt_, (void*)bcnt_, (void*)cslot_, scan_tmp_})
    if (p) (void)hipFree(p);
  scan_tmp_ = nullptr;
  pad_ = rank_ = nullptr;
  cslot_ = nullptr;
  tcnt_ = nullptr;
  bcnt_ = nullptr;
  cap_bytes_ = 0;
  const size_t nb = (n + kChunk - 1) / kChunk, cap = nb * kChunk;  // every later n <= cap fits
  // word-cache slots: the table is allocated for one slot per 256 text bytes; a call starts with
  // one per 4096 (a small table keeps the probed lines cache-resident) and grows it 4x while a
  // probe window overflows, then takes the direct path
  ccap_ = 1 << 20;
  while (ccap_ < cap / 256) ccap_ <<= 1;
  ccap_min_ = 1 << 20;
  while (ccap_min_ < cap / 4096) ccap_min_ <<= 1;
  if (hipMalloc(&cslot_, ccap_ * kSlotU64 * 8) != hipSuccess) {
    *why = "word-cache allocation failed";
    return false;
  }
  if (hipMalloc(&pad_, cap * 4) != hipSuccess || hipMalloc(&rank_, cap * 4) != hipSuccess ||
      hipMalloc(&tcnt_, nb * kThreads * 4) != hipSuccess || hipMalloc(&bcnt_, (3 * nb + 1) * 8) != hipSuccess ||
      hipcub::DeviceScan::InclusiveSum(nullptr, scan_tmp_bytes_, bcnt_, bcnt_ + nb, (int)nb) != hipSuccess ||
      hipMalloc(&scan_tmp_, scan_tmp_bytes_ ? scan_tmp_bytes_ : 16) != hipSuccess) {
    *why = "scratch allocation failed";
    return false;
  }
  cap_bytes_ = cap;
  return true;
}

namespace {
// Restores the caller's current device when an encoder call returns.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
}  // namespace

int64_t EncodeDevice::encode(const uint8_t* text, size_t n, int32_t* out, size_t cap, void* stream, double* kernel_ms) {
  if (kernel_ms) *kernel_ms = 0;
  if (n == 0) return 0;
  if (!text || !out) return -1;
  DeviceGuard guard;
  ENC_OK(hipSetDevice(device_));
  std::string why;
  if (!reserve(n, &why)) {
    std::fprintf(stderr, "[ERROR]\t encoder: %s (%zu bytes)\n", why.c_str(), n);
    return -1;
  }
  hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)stream_;
  const u64 nb = (n + kChunk - 1) / kChunk;
  hipEvent_t* ev = reinterpret_cast<hipEvent_t*>(ev_);
  const char* env = std::getenv("SHREDWORD_ENCODE_CACHE");
  bool cached = !(env && env[0] == '0');
  ENC_OK(hipEventRecord(ev[0], st));
  size_t cc = ccap_min_;
  for (;;) {
    ENC_OK(hipMemsetAsync(misc_, 0, 32, st));
    if (cached) {
      ENC_OK(hipMemsetAsync(cslot_, 0, cc * kSlotU64 * 8, st));
      k_cache_insert<<<dim3((unsigned)nb), dim3(kThreads), 0, st>>>(text, n, cslot_, cc - 1, misc_);
      ENC_OK(hipGetLastError());
      auto enck = packed_ ? k_cache_encode<true> : k_cache_encode<false>;
      // arena offsets must stay below 2^31: bit 31 of a payload tags "ids inline in the slot", so
      // a larger arena flags "arena full" and the call reruns on the direct path
      const u64 arena_cap = std::min<u64>(cap_bytes_, (u64)1 << 31);
      enck<<<dim3((unsigned)(cc / kThreads)), dim3(kThreads), 0, st>>>(text, n, byte_map_, table_, mask_, cslot_, cc,
                                                                       rank_, arena_cap, pad_, misc_);
      ENC_OK(hipGetLastError());
      // look-back states and the ticket (bcnt_[2 nb, 3 nb], zero = "not published")
      ENC_OK(hipMemsetAsync(bcnt_ + 2 * nb, 0, (nb + 1) * 8, st));
      k_cache_words<<<dim3((unsigned)nb), dim3(kThreads), 0, st>>>(text, n, cslot_, cc - 1, rank_, out, (u64)cap, bcnt_,
                                                                   bcnt_ + 2 * nb, nb, misc_);
    } else {
      const bool aligned = (reinterpret_cast<uintptr_t>(text) & 15) == 0;
      auto kern = aligned ? (packed_ ? k_encode_words<true, true> : k_encode_words<true, false>)
                          : (packed_ ? k_encode_words<false, true> : k_encode_words<false, false>);
      kern<<<dim3((unsigned)nb), dim3(kThreads), 0, st>>>(text, n, byte_map_, table_, mask_, pad_, rank_, tcnt_,
                                                          bcnt_, misc_);
    }
    ENC_OK(hipGetLastError());
    // inclusive block sums into bcnt_[nb, 2 nb); the last one is the total
    ENC_OK(hipcub::DeviceScan::InclusiveSum(scan_tmp_, scan_tmp_bytes_, bcnt_, bcnt_ + nb, (int)nb, st));
    ENC_OK(hipMemcpyAsync(misc_, bcnt_ + 2 * nb - 1, 8, hipMemcpyDeviceToDevice, st));
    ENC_OK(hipMemcpyAsync(host_misc_, misc_, 16, hipMemcpyDeviceToHost, st));
    ENC_OK(hipStreamSynchronize(st));
    const uint64_t fl = host_misc_[1];
    if (fl & 1) return -3;
    if (fl & 16) return -2;  // the output capacity (the cached path writes it directly)
    if (!(fl & 14)) break;
    if (fl == 2 && cc < ccap_) {  // only a probe window overflowed: a bigger table
      cc = std::min(ccap_, cc * 4);
      continue;
    }
    cached = false;  // cache / arena overflow or a 64-bit word-hash collision: redo on the direct path
    if (std::getenv("SHREDWORD_ENCODE_DEBUG"))
      std::fprintf(stderr, "[DEBUG]\t encoder: word cache %s (%zu slots); direct path\n",
                   fl & 4 ? "hash collision" : fl & 8 ? "arena overflow" : "overflow", cc);
    ++fallbacks_;
  }
  ENC_OK(hipEventRecord(ev[1], st));
  const u64 total = host_misc_[0];
  if (total > cap) return -2;
  ENC_OK(hipEventRecord(ev[2], st));
  if (total && !cached)  // the cached path wrote the ids in place (k_cache_words)
    k_encode_emit<<<dim3((unsigned)nb), dim3(kThreads), 0, st>>>(pad_, tcnt_, bcnt_ + nb, out);
  ENC_OK(hipGetLastError());
  ENC_OK(hipEventRecord(ev[3], st));
  ENC_OK(hipStreamSynchronize(st));
  if (kernel_ms) {
    float a = 0, b = 0;
    ENC_OK(hipEventElapsedTime(&a, ev[0], ev[1]));
    ENC_OK(hipEventElapsedTime(&b, ev[2], ev[3]));
    *kernel_ms = (double)a + (double)b;
  }
  return (int64_t)total;
}

bool EncodeDevice::reserve_host(size_t n) {
  if (n <= host_cap_) return true;
  if (dtext_) (void)hipFree(dtext_);
  if (dout_) (void)hipFree(dout_);
  dtext_ = nullptr;
  dout_ = nullptr;
  host_cap_ = 0;
  if (hipMalloc(&dtext_, n) != hipSuccess || hipMalloc(&dout_, n * 4) != hipSuccess) return false;
  host_cap_ = n;
  return true;
}

// Host text in pieces of at most kHostPiece bytes, each cut just after a delimiter (words never
// straddle two pieces, so the ids are those of one call): device memory stays at ~14 B per piece
// byte (5 B staging + the scratch reserve() sizes) whatever the text length.
int64_t EncodeDevice::encode_host(const uint8_t* text, size_t n, int32_t* out, size_t cap) {
  if (n == 0) return 0;
  if (!text || !out) return -1;
  DeviceGuard guard;
  ENC_OK(hipSetDevice(device_));
  size_t piece = kHostPiece;
  if (const char* e = std::getenv("SHREDWORD_ENCODE_PIECE"))  // tests: small pieces
    piece = std::max<size_t>((size_t)std::strtoull(e, nullptr, 10), (size_t)kEncMaxWord + 2);
  piece = std::min(n, piece);
  if (!reserve_host(piece)) {
    std::fprintf(stderr, "[ERROR]\t encoder: staging allocation failed (%zu bytes)\n", piece);
    return -1;
  }
  hipStream_t st = (hipStream_t)stream_;
  size_t pos = 0, done = 0;
  while (pos < n) {
    size_t len = std::min(piece, n - pos);
    if (pos + len < n) {  // end the piece after its last delimiter
      size_t k = len;
      const size_t lo = len > (size_t)kEncMaxWord + 1 ? len - (size_t)kEncMaxWord - 1 : 0;
      while (k > lo) {
        const uint8_t c = text[pos + k - 1];
        if (c == 9 || c == 10 || c == 13 || c == 32) break;
        --k;
      }
      if (k == lo) return -3;  // no delimiter in the last kEncMaxWord + 1 bytes: a word past the limit
      len = k;
    }
    ENC_OK(hipMemcpyAsync(dtext_, text + pos, len, hipMemcpyHostToDevice, st));
    const int64_t r = encode(dtext_, len, dout_, cap - done, nullptr, nullptr);
    if (r < 0) return r;
    if (r > 0) {
      ENC_OK(hipMemcpyAsync(out + done, dout_, (size_t)r * 4, hipMemcpyDeviceToHost, st));
      ENC_OK(hipStreamSynchronize(st));
    }
    done += (size_t)r;
    pos += len;
  }
  return (int64_t)done;
}

}  // namespace shred
