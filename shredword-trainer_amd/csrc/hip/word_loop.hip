// MI355X (gfx950) kernels of the indexed merge loop (host/word_loop.h) and its host driver.
//
//   k_word_loop       the merge loop: one persistent workgroup (16 wave64s) that takes merge /
//                     undo commands from a ring in pinned host memory.  Per merge (a, b) -> X:
//                     directory lookup of (a, b) -> its word list; a lane per listed word scans
//                     it greedily left to right (reference bpe.cpp:265-296), emits the four
//                     neighbour deltas per occurrence into an LDS hash keyed (neighbour slot,
//                     category) with Σ weight and min first touch (FreqChangeMap, bpe.cpp:9-50),
//                     and compacts the word in place; the records go to host memory behind one
//                     system release and a flag; then the new pairs (p, X) / (X, n) are grouped
//                     in LDS and appended to the pool under new directory entries.
//   k_wl_emit_pairs   initial index: every adjacent non-unk pair of every word -> (key, word)
//   k_wl_mark / k_wl_scatter / k_wl_dir_init   sorted runs -> pool + directory
//   k_words_to_tiles  the word table back into the tile stream (headers + tokens)
//
// Integer and index work only: no MFMA.  Everything the loop touches per merge is a few KB of
// the word table and the index, so the bound is the chain of dependent memory round trips, not
// bandwidth.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../host/common.h"
#include "../host/word_loop.h"

namespace shred {

#define WL_OK(expr)                                                                         \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "[ERROR]\t HIP %s failed: %s (%s:%d)\n", #expr, hipGetErrorString(e_), \
                   __FILE__, __LINE__);                                                     \
      std::fflush(stderr);                                                                  \
      std::abort();                                                                         \
    }                                                                                       \
  } while (0)

namespace {

typedef unsigned long long u64;

constexpr int kWlThreads = 1024;
constexpr int kWlWaves = kWlThreads / 64;
constexpr int kDh = 2048;               // LDS delta hash slots
constexpr int kBh = 2048;               // LDS new-pair hash slots (build round)
constexpr uint32_t kRing = 64;          // command ring entries
constexpr uint32_t kOpMerge = 1, kOpStop = 2, kOpTimeout = 3, kOpUnmerge = 4;
constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;
constexpr u64 kEmpty64 = ~0ull;
constexpr uint32_t kInvalidSeq = 0xFFFFFFFFu;
// dstate words
constexpr int kStSpill = 0, kStPoolTop = 1, kStKeys = 2, kStError = 3;
// error codes (dstate[kStError], reported by the host)
constexpr uint32_t kErrPool = 1, kErrStage = 2, kErrDir = 3, kErrLookup = 4;

struct WlCmd {
  u64 g[4];  // granules (seq | value << 32): op | slot << 8, a, b, X
};

struct WlSlotDev {
  DeltaRecord* recs;  // host-visible
  uint32_t* hdr;      // host-visible: [0] records, [1] flag, [2] candidates, [3] changed words,
                      //   [4..5] occurrences (u64), [6..7] device ticks command -> flag (u64)
  uint32_t rec_cap;
};

struct WlParams {
  int32_t* wtok;
  const uint32_t* woff;
  uint32_t* wlen;
  uint32_t* wmark;
  const u64* weight;
  uint32_t nwords;
  uint32_t* pool;
  u64 pool_cap;
  u64* dkey;
  u64* dval;
  uint32_t* dseq;
  u64 dir_mask;
  uint32_t* valid_seq;
  uint32_t id_cap;
  u64* sk[2];
  uint32_t* sw[2];
  uint32_t* sslot;
  u64 stage_cap;
  u64* dsum;
  u64* dft;
  uint32_t* dlist;
  uint32_t* dstate;
  uint32_t cap;     // delta slots: ids in [0, cap) have slot id + 1, others (unk) slot 0
  int32_t unk;
  const WlCmd* ring;
  uint32_t* status;  // host-visible: [0] exit op
  uint32_t seq0;
  uint32_t idle_polls;
  WlSlotDev sl[WordLoop::kSlots];
};

__device__ __forceinline__ u64 mix64(u64 k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  k *= 0xC4CEB9FE1A85EC53ull;
  k ^= k >> 33;
  return k;
}
__device__ __forceinline__ u64 pair_key(int32_t a, int32_t b) { return ((u64)(uint32_t)a << 32) | (uint32_t)b; }
__device__ __forceinline__ uint32_t slot_of(int32_t id, uint32_t cap) {
  return (uint32_t)id < cap ? (uint32_t)id + 1u : 0u;
}
__device__ __forceinline__ u64 ld_agent(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct DeltaH {
  uint32_t key[kDh];
  u64 sum[kDh];
  u64 ft[kDh];
};
struct BuildH {
  u64 key[kBh];
  uint32_t cnt[kBh];
  uint32_t fill[kBh];
  uint32_t off[kBh];
};
union LdsU {
  DeltaH d;
  BuildH b;
};

// One neighbour delta (reference freq_change_add, bpe.cpp:274-290): Σ weight and min first touch
// per key = slot * 4 + category, in the LDS hash; keys past it go to the global spill tables.
__device__ __forceinline__ void delta_add(DeltaH& h, const WlParams& p, uint32_t key, u64 w, u64 ft) {
  uint32_t s = (key * 2654435761u) >> (32 - 11);
#pragma unroll 1
  for (int probe = 0; probe < 32; ++probe) {
    const uint32_t prev = atomicCAS(&h.key[s], kEmpty32, key);
    if (prev == kEmpty32 || prev == key) {
      atomicAdd(&h.sum[s], w);
      atomicMin(&h.ft[s], ft);
      return;
    }
    s = (s + 1) & (kDh - 1);
  }
  const u64 old = atomicAdd(&p.dsum[key], w);
  atomicMin(&p.dft[key], ft);
  if (old == 0) p.dlist[atomicAdd(&p.dstate[kStSpill], 1u)] = key;  // weights are >= 1
}

// A new pair of merge X listed for word w (superset entries are harmless: the word is rescanned).
__device__ __forceinline__ void stage_pair(const WlParams& p, uint32_t* n_stage, int32_t c, int32_t d, uint32_t w) {
  if (c == p.unk || d == p.unk) return;  // pairs holding unk are never merged (bpe.cpp:251-258)
  const uint32_t i = atomicAdd(n_stage, 1u);
  if (i < p.stage_cap) {
    p.sk[0][i] = pair_key(c, d);
    p.sw[0][i] = w;
  } else {
    atomicMax(&p.dstate[kStError], kErrStage);
  }
}

// Merge (a, b) -> X in word w, greedy left to right as the reference's chain walk; returns the
// occurrences merged.  First touch = (rank << 32) | (input position << 2) | category.
__device__ __forceinline__ uint32_t merge_word(const WlParams& p, DeltaH& h, uint32_t* n_stage, uint32_t w, int32_t a,
                                               int32_t b, int32_t X, uint32_t seq) {
  const uint32_t old = atomicExch(&p.wmark[w], seq);  // a list may name a word twice
  const uint32_t o = p.woff[w];
  const uint32_t L = p.wlen[w];
  if (old == seq || L < 2) return 0;
  const u64 wc = p.weight[w];
  const u64 rank = (u64)w << 32;
  int32_t* t = p.wtok + o;
  uint32_t j = 0, k = 0, occ = 0;
  int32_t prev = 0;
  int32_t c0 = t[0], c1 = t[1];
#pragma unroll 1
  while (j < L) {
    if (j + 1 < L && c0 == a && c1 == b) {
      const bool has_n = j + 2 < L;
      const int32_t n = has_n ? t[j + 2] : 0;  // the original next token (bpe.cpp:283-289)
      const int32_t n2 = j + 3 < L ? t[j + 3] : 0;
      const u64 ft = rank | ((u64)j << 2);
      if (k > 0) {  // left neighbour: X when it was just produced (bpe.cpp:276-279)
        delta_add(h, p, slot_of(prev, p.cap) * 4u + 0u, wc, ft | 0u);
        delta_add(h, p, slot_of(prev, p.cap) * 4u + 1u, wc, ft | 1u);
        stage_pair(p, n_stage, prev, X, w);
      }
      if (has_n) {
        delta_add(h, p, slot_of(n, p.cap) * 4u + 2u, wc, ft | 2u);
        delta_add(h, p, slot_of(n, p.cap) * 4u + 3u, wc, ft | 3u);
        stage_pair(p, n_stage, X, n, w);
      }
      t[k] = X;
      prev = X;
      ++k;
      ++occ;
      j += 2;
      c0 = n;
      c1 = n2;
    } else {
      if (occ) t[k] = c0;  // positions before the first occurrence are unchanged
      prev = c0;
      ++k;
      ++j;
      c0 = c1;
      c1 = j + 1 < L ? t[j + 1] : 0;
    }
  }
  if (occ) p.wlen[w] = k;
  return occ;
}

// Undo of merge X in word w: every X back into (a, b), right to left in place.
__device__ __forceinline__ void unmerge_word(const WlParams& p, uint32_t w, int32_t a, int32_t b, int32_t X,
                                             uint32_t seq) {
  const uint32_t old = atomicExch(&p.wmark[w], seq);
  const uint32_t o = p.woff[w];
  const uint32_t L = p.wlen[w];
  if (old == seq || L == 0) return;
  int32_t* t = p.wtok + o;
  uint32_t nx = 0;
  for (uint32_t j = 0; j < L; ++j) nx += t[j] == X;
  if (!nx) return;
  uint32_t q = L + nx;
  for (uint32_t j = L; j-- > 0;) {
    const int32_t v = t[j];
    if (v == X) {
      t[--q] = b;
      t[--q] = a;
    } else {
      t[--q] = v;
    }
  }
  p.wlen[w] = L + nx;
}

__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Directory insert of a key of merge `seq` (one thread per key; keys of one round are distinct).
__device__ __forceinline__ void dir_insert(const WlParams& p, u64 key, uint32_t off, uint32_t cnt, uint32_t seq) {
  u64 h = mix64(key) & p.dir_mask;
  for (u64 probe = 0; probe <= p.dir_mask; ++probe) {
    const u64 prev = atomicCAS(&p.dkey[h], kEmpty64, key);
    if (prev == kEmpty64 || prev == key) {
      p.dval[h] = (u64)off | ((u64)cnt << 32);
      p.dseq[h] = seq;
      if (prev == kEmpty64) {
        const uint32_t n = atomicAdd(&p.dstate[kStKeys], 1u);
        if ((u64)n * 4 > (p.dir_mask + 1) * 3) atomicMax(&p.dstate[kStError], kErrDir);
      }
      return;
    }
    h = (h + 1) & p.dir_mask;
  }
  atomicMax(&p.dstate[kStError], kErrDir);
}

}  // namespace

// The merge loop (see the file comment).  One workgroup; command numbers start at p.seq0.
__global__ __launch_bounds__(kWlThreads) void k_word_loop(WlParams p) {
  __shared__ LdsU u;
  __shared__ uint32_t s_cmd[8];
  __shared__ uint32_t s_nout, s_nstage, s_ndefer, s_pool_top, s_base, s_total;
  __shared__ u64 s_lk[2];  // lookup: pool offset, count
  __shared__ u64 s_occ, s_changed;
  __shared__ uint32_t s_wsum[kWlWaves];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t tid = threadIdx.x;
  if (tid == 0) s_pool_top = ld_agent(&p.dstate[kStPoolTop]);
  uint32_t expect = p.seq0;
  uint32_t exit_op = kOpStop;
  __syncthreads();
  for (;;) {
    // ---- wave 0 waits for the next command (one round trip reads all four granules)
    if (wid == 0) {
      uint32_t op = 0, a = 0, b = 0, X = 0, idle = 0;
      const u64* g = p.ring[expect % kRing].g;
      for (;;) {
        const u64 v = lane < 4 ? __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
        const bool tagged = lane >= 4 || (uint32_t)v == expect;
        if (__all(tagged)) {
          const uint32_t val = (uint32_t)(v >> 32);
          op = __shfl(val, 0, 64);
          a = __shfl(val, 1, 64);
          b = __shfl(val, 2, 64);
          X = __shfl(val, 3, 64);
          break;
        }
        if (++idle >= p.idle_polls) {
          op = kOpTimeout;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) {
        s_cmd[0] = op & 0xFFu;
        s_cmd[1] = a;
        s_cmd[2] = b;
        s_cmd[3] = X;
        s_cmd[4] = (op >> 8) & 0xFFu;  // slot
        s_cmd[5] = expect;
      }
    }
    __syncthreads();
    const uint32_t op = s_cmd[0];
    const int32_t a = (int32_t)s_cmd[1], b = (int32_t)s_cmd[2], X = (int32_t)s_cmd[3];
    const uint32_t slot = s_cmd[4], seq = s_cmd[5];
    ++expect;
    if (op != kOpMerge && op != kOpUnmerge) {
      exit_op = op;
      break;
    }
    // ---- the word list of (a, b): wave 0 probes 16 directory slots per round trip
    u64 t_cmd = 0;
    if (wid == 0) {
      if (lane == 0) t_cmd = __builtin_amdgcn_s_memrealtime();
      const u64 key = pair_key(a, b);
      const int32_t M = a > b ? a : b;
      u64 h = mix64(key) & p.dir_mask;
      u64 off = 0, cnt = 0;
      bool err = false;
      for (uint32_t base = 0;; base += 16) {
        const u64 idx = (h + base + (u64)lane) & p.dir_mask;
        u64 k = kEmpty64, v = 0;
        uint32_t sq = 0, vs = 0;
        if (lane < 16) {
          k = ld_agent(p.dkey + idx);
          v = p.dval[idx];
          sq = p.dseq[idx];
        }
        if (lane == 16) vs = M >= kBaseVocab && (uint32_t)M < p.id_cap ? p.valid_seq[M] : 0u;
        vs = __shfl(vs, 16, 64);
        const u64 hit = __ballot(lane < 16 && k == key);
        const u64 emp = __ballot(lane < 16 && k == kEmpty64);
        const u64 any = hit | emp;
        if (any) {
          const int f = __ffsll((long long)any) - 1;
          if ((hit >> f) & 1ull) {
            const u64 vf = __shfl(v, f, 64);
            const uint32_t sf = __shfl(sq, f, 64);
            if (sf == vs) {
              off = (uint32_t)vf;
              cnt = vf >> 32;
            } else {
              err = op == kOpMerge;
            }
          } else {
            err = op == kOpMerge;  // a selected pair always has a list
          }
          break;
        }
        if (base > p.dir_mask) {
          err = op == kOpMerge;
          break;
        }
      }
      if (lane == 0) {
        s_lk[0] = off;
        s_lk[1] = cnt;
        s_nout = 0;
        s_nstage = 0;
        s_occ = 0;
        s_changed = 0;
        if (err) atomicMax(&p.dstate[kStError], kErrLookup);
      }
    }
    if (op == kOpMerge)
      for (int i = tid; i < kDh; i += kWlThreads) {
        u.d.key[i] = kEmpty32;
        u.d.sum[i] = 0;
        u.d.ft[i] = kEmpty64;
      }
    __syncthreads();
    const u64 off = s_lk[0], cnt = s_lk[1];
    if (op == kOpUnmerge) {
      for (u64 i = tid; i < cnt; i += kWlThreads) unmerge_word(p, p.pool[off + i], a, b, X, seq);
      __syncthreads();
      if (tid == 0 && X >= kBaseVocab && (uint32_t)X < p.id_cap) p.valid_seq[X] = kInvalidSeq;
      __syncthreads();
      continue;
    }
    // ---- the merge over the listed words, a lane per word
    uint32_t my_occ = 0, my_changed = 0;
    for (u64 i = tid; i < cnt; i += kWlThreads) {
      const uint32_t m = merge_word(p, u.d, &s_nstage, p.pool[off + i], a, b, X, seq);
      my_occ += m;
      my_changed += m ? 1u : 0u;
    }
    {
      const uint32_t wo = wave_incl_add(my_occ), wc = wave_incl_add(my_changed);
      if (lane == 63 && (wo || wc)) {
        atomicAdd(&s_occ, (u64)wo);
        atomicAdd(&s_changed, (u64)wc);
      }
    }
    __syncthreads();
    // ---- the records to host memory (LDS hash, then the spilled keys), then the flag
    const WlSlotDev& sd = p.sl[slot & (WordLoop::kSlots - 1)];
    for (int i = tid; i < kDh; i += kWlThreads) {
      const uint32_t key = u.d.key[i];
      if (key == kEmpty32) continue;
      const uint32_t r = atomicAdd(&s_nout, 1u);
      u64* dst = reinterpret_cast<u64*>(sd.recs + r);
      dst[0] = (u64)key;
      dst[1] = u.d.sum[i];
      dst[2] = u.d.ft[i];
    }
    __syncthreads();
    {
      const uint32_t nsp = ld_agent(&p.dstate[kStSpill]);
      for (uint32_t i = tid; i < nsp; i += kWlThreads) {
        const uint32_t key = p.dlist[i];
        const u64 sum = atomicExch(&p.dsum[key], 0ull);
        const u64 ft = atomicExch(&p.dft[key], kEmpty64);
        const uint32_t r = atomicAdd(&s_nout, 1u);
        u64* dst = reinterpret_cast<u64*>(sd.recs + r);
        dst[0] = (u64)key;
        dst[1] = sum;
        dst[2] = ft;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      p.dstate[kStSpill] = 0;
      sd.hdr[0] = s_nout;
      sd.hdr[2] = (uint32_t)cnt;
      sd.hdr[3] = (uint32_t)s_changed;
      reinterpret_cast<u64*>(sd.hdr)[2] = s_occ;
      reinterpret_cast<u64*>(sd.hdr)[3] = (u64)__builtin_amdgcn_s_memrealtime() - t_cmd;
      __threadfence_system();
      __hip_atomic_store(sd.hdr + 1, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // ---- the index entries of merge X's new pairs (after the flag: off the host's path)
    uint32_t n = s_nstage < p.stage_cap ? s_nstage : (uint32_t)p.stage_cap;
    int src = 0;
    while (n > 0) {
      for (int i = tid; i < kBh; i += kWlThreads) {
        u.b.key[i] = kEmpty64;
        u.b.cnt[i] = 0;
        u.b.fill[i] = 0;
      }
      if (tid == 0) s_ndefer = 0;
      __syncthreads();
      for (uint32_t e = tid; e < n; e += kWlThreads) {
        const u64 key = p.sk[src][e];
        uint32_t s = (uint32_t)(mix64(key) >> 53) & (kBh - 1);
        uint32_t got = kEmpty32;
        for (int probe = 0; probe < 64; ++probe) {
          const u64 prev = atomicCAS(&u.b.key[s], kEmpty64, key);
          if (prev == kEmpty64 || prev == key) {
            got = s;
            break;
          }
          s = (s + 1) & (kBh - 1);
        }
        if (got != kEmpty32) {
          atomicAdd(&u.b.cnt[got], 1u);
        } else {  // this round's table is full: the entry waits for the next round
          const uint32_t d = atomicAdd(&s_ndefer, 1u);
          p.sk[src ^ 1][d] = key;
          p.sw[src ^ 1][d] = p.sw[src][e];
        }
        p.sslot[e] = got;
      }
      __syncthreads();
      {  // exclusive offsets of the slots (2 per thread), the round's total
        const uint32_t c0 = u.b.cnt[2 * tid], c1 = u.b.cnt[2 * tid + 1];
        const uint32_t incl = wave_incl_add(c0 + c1);
        if (lane == 63) s_wsum[wid] = incl;
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (int q = 0; q < kWlWaves; ++q) {
          before += q < wid ? s_wsum[q] : 0u;
          total += s_wsum[q];
        }
        const uint32_t ex = before + incl - (c0 + c1);
        u.b.off[2 * tid] = ex;
        u.b.off[2 * tid + 1] = ex + c0;
        if (tid == 0) {
          s_base = s_pool_top;
          s_total = total;
          if ((u64)s_pool_top + total > p.pool_cap) atomicMax(&p.dstate[kStError], kErrPool);
          else s_pool_top += total;
        }
      }
      __syncthreads();
      const uint32_t base = s_base;
      const bool fits = (u64)base + s_total <= p.pool_cap;
      if (fits) {
        for (uint32_t e = tid; e < n; e += kWlThreads) {
          const uint32_t s = p.sslot[e];
          if (s == kEmpty32) continue;
          const uint32_t pos = base + u.b.off[s] + atomicAdd(&u.b.fill[s], 1u);
          p.pool[pos] = p.sw[src][e];
        }
        for (int s = tid; s < kBh; s += kWlThreads) {
          const u64 key = u.b.key[s];
          if (key != kEmpty64) dir_insert(p, key, base + u.b.off[s], u.b.cnt[s], seq);
        }
      }
      __syncthreads();
      n = s_ndefer;
      src ^= 1;
      if (n) {  // deferred entries live in the other buffer pair now; keep buffer 0 the source
        for (uint32_t e = tid; e < n; e += kWlThreads) {
          p.sk[0][e] = p.sk[1][e];
          p.sw[0][e] = p.sw[1][e];
        }
        src = 0;
        __syncthreads();
      }
    }
    if (tid == 0 && X >= kBaseVocab && (uint32_t)X < p.id_cap) p.valid_seq[X] = seq;
    __syncthreads();
  }
  if (tid == 0) {
    p.dstate[kStPoolTop] = s_pool_top;
    __threadfence_system();
    __hip_atomic_store(&p.status[0], exit_op, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

namespace {

// Initial index: pair j of word w goes to entry (woff[w] - w) + j (a word of capacity c owns
// c - 1 entries); pairs holding unk and capacity past the live length emit EMPTY.
__global__ void k_wl_emit_pairs(const int32_t* wtok, const uint32_t* woff, const uint32_t* wlen, uint32_t W,
                                int32_t unk, u64* key, uint32_t* val) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < W; w += gridDim.x * blockDim.x) {
    const uint32_t o = woff[w], capw = woff[w + 1] - o, L = wlen[w];
    const uint64_t base = (uint64_t)o - w;
    for (uint32_t j = 0; j + 1 < capw; ++j) {
      u64 k = kEmpty64;
      if (j + 1 < L) {
        const int32_t x = wtok[o + j], y = wtok[o + j + 1];
        if (x != unk && y != unk) k = pair_key(x, y);
      }
      key[base + j] = k;
      val[base + j] = w;
    }
  }
}

// Sorted (key, word) runs: keep the first of equal (key, word) entries; mark the first entry of
// each key.  Word ids are ascending inside a key (stable sort of entries emitted in word order).
__global__ void k_wl_mark(const u64* key, const uint32_t* val, uint64_t n, uint32_t* keep, uint32_t* head) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const u64 k = key[i];
    const bool valid = k != kEmpty64;
    const bool first_key = valid && (i == 0 || key[i - 1] != k);
    keep[i] = valid && (first_key || val[i - 1] != val[i]);
    head[i] = first_key;
  }
}

__global__ void k_wl_scatter(const u64* key, const uint32_t* val, uint64_t n, const uint32_t* keep,
                             const uint32_t* pos, const uint32_t* head, const uint32_t* kidx, uint32_t* pool,
                             u64* ikey, u64* ival) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (keep[i]) pool[pos[i]] = val[i];
    if (head[i]) {
      ikey[kidx[i]] = key[i];
      ival[kidx[i]] = pos[i];  // offset; the count is filled in by k_wl_counts
    }
  }
}

__global__ void k_wl_counts(u64* ival, uint64_t nk, uint64_t total) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nk; i += (uint64_t)gridDim.x * blockDim.x) {
    const u64 o = ival[i] & 0xFFFFFFFFull;
    const u64 e = i + 1 < nk ? (ival[i + 1] & 0xFFFFFFFFull) : total;
    ival[i] = o | ((e - o) << 32);
  }
}

// The initial directory (after a memset of the keys to EMPTY): no key repeats.
__global__ void k_wl_dir_init(const u64* ikey, const u64* ival, uint64_t nk, u64* dkey, u64* dval, uint32_t* dseq,
                              u64 mask) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nk; i += (uint64_t)gridDim.x * blockDim.x) {
    const u64 key = ikey[i];
    u64 h = mix64(key) & mask;
    for (;;) {
      const u64 prev = atomicCAS(&dkey[h], kEmpty64, key);
      if (prev == kEmpty64) {
        dval[h] = ival[i];
        dseq[h] = 0;
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

// Words -> tiles: a wave per tile writes [header][tokens] for its words in rank order and the
// tile's live length; the old tail up to the previous length becomes padding.
__global__ void k_words_to_tiles(const int32_t* wtok, const uint32_t* woff, const uint32_t* wlen,
                                 const uint32_t* tile_first, const uint32_t* tile_nw, uint32_t ntiles, int32_t* tok,
                                 const uint64_t* tile_off, uint32_t* tile_len) {
  const int lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (blockDim.x / 64);
  for (uint32_t t = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); t < ntiles; t += waves) {
    int32_t* dst = tok + tile_off[t];
    const uint32_t f = tile_first[t], nw = tile_nw[t];
    uint32_t base = 0;
    for (uint32_t q = 0; q < nw; q += 64) {
      const uint32_t w = f + q + (uint32_t)lane;
      const bool on = q + (uint32_t)lane < nw;
      const uint32_t len = on ? wlen[w] : 0u;
      const uint32_t need = on ? len + 1u : 0u;
      const uint32_t incl = wave_incl_add(need);
      if (on) {
        int32_t* d = dst + base + incl - need;
        d[0] = (int32_t)((uint32_t)kHeaderBase + w);
        const int32_t* s = wtok + woff[w];
        for (uint32_t j = 0; j < len; ++j) d[1 + j] = s[j];
      }
      base += __shfl(incl, 63, 64);
    }
    const uint32_t old = tile_len[t];
    for (uint32_t i = base + (uint32_t)lane; i < old; i += 64) dst[i] = INT32_MIN;
    if (lane == 0) tile_len[t] = base;
  }
}

template <class T>
T* wl_alloc(size_t n, size_t* acc) {
  void* p = nullptr;
  WL_OK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
  *acc += std::max<size_t>(n, 1) * sizeof(T);
  return static_cast<T*>(p);
}

inline hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

}  // namespace

// ==========================================================================================
WordLoop::WordLoop(int ordinal, void* stream, int32_t unk_id) : ordinal_(ordinal), stream_(stream), unk_(unk_id) {
  WL_OK(hipSetDevice(ordinal_));
  const unsigned pin = hipHostMallocMapped | hipHostMallocCoherent;
  WL_OK(hipHostMalloc(&ring_, sizeof(WlCmd) * kRing, pin));
  std::memset(ring_, 0, sizeof(WlCmd) * kRing);
  WL_OK(hipHostGetDevicePointer(&ring_dev_, ring_, 0));
  WL_OK(hipHostMalloc((void**)&status_, 64, pin));
  std::memset(status_, 0, 64);
  WL_OK(hipHostGetDevicePointer(&status_dev_, status_, 0));
  for (auto& e : ev_) {
    hipEvent_t ev;
    WL_OK(hipEventCreate(&ev));
    e = ev;
  }
}

WordLoop::~WordLoop() {
  (void)hipSetDevice(ordinal_);
  if (running_ && posted_.empty()) stop();
  (void)hipStreamSynchronize(S(stream_));
  free_all();
  for (Slot& s : slot_) {
    if (s.host_recs) (void)hipHostFree(s.host_recs);
    if (s.host_hdr) (void)hipHostFree(s.host_hdr);
  }
  if (ring_) (void)hipHostFree(ring_);
  if (status_) (void)hipHostFree(status_);
  for (auto e : ev_)
    if (e) (void)hipEventDestroy((hipEvent_t)e);
}

void WordLoop::free_all() {
  void* ptrs[] = {wtok_, wtok0_, woff_, wlen_, wlen0_, wmark_, tile_first_, tile_nw_, pool_, dkey_, dval_, dseq_,
                  init_key_, init_val_, valid_seq_, stage_key_[0], stage_key_[1], stage_w_[0], stage_w_[1],
                  stage_slot_, dsum_, dft_, dlist_, dstate_};
  for (void* p : ptrs)
    if (p) WL_OK(hipFree(p));
  wtok_ = wtok0_ = nullptr;
  woff_ = wlen_ = wlen0_ = wmark_ = tile_first_ = tile_nw_ = pool_ = dseq_ = valid_seq_ = stage_slot_ = dlist_ =
      dstate_ = nullptr;
  dkey_ = dval_ = init_key_ = init_val_ = dsum_ = dft_ = nullptr;
  stage_key_[0] = stage_key_[1] = nullptr;
  stage_w_[0] = stage_w_[1] = nullptr;
  cap_ = id_cap_ = 0;
  bytes_ = 0;
  ready_ = false;
}

bool WordLoop::upload(const TiledStream& ts, const uint64_t* d_weight) {
  WL_OK(hipSetDevice(ordinal_));
  if (running_) stop();
  free_all();
  // the words of the tile stream in rank order (types layout: one entry per distinct word)
  std::vector<uint32_t> woff, tfirst, tnw;
  std::vector<int32_t> wtok;
  woff.reserve(ts.entries + 1);
  wtok.reserve(ts.live);
  tfirst.reserve(ts.num_tiles());
  tnw.reserve(ts.num_tiles());
  uint32_t expect_rank = 0;
  for (size_t t = 0; t < ts.num_tiles(); ++t) {
    const int32_t* p = ts.tok.data() + ts.off[t];
    tfirst.push_back((uint32_t)woff.size());
    uint32_t nw = 0;
    for (uint32_t i = 0; i < ts.len[t]; ++i) {
      if (p[i] < kHeaderLimit) {
        const uint32_t r = (uint32_t)(p[i] - kHeaderBase);
        if (r != expect_rank) return false;  // not the whole table in rank order: not for this loop
        ++expect_rank;
        if (wtok.size() >= 0xFFFFFFF0ull) return false;
        woff.push_back((uint32_t)wtok.size());
        ++nw;
      } else {
        if (woff.empty()) return false;
        wtok.push_back(p[i]);
      }
    }
    tnw.push_back(nw);
  }
  woff.push_back((uint32_t)wtok.size());
  nwords_ = (uint32_t)(woff.size() - 1);
  nsym_ = wtok.size();
  ntiles_ = (uint32_t)ts.num_tiles();
  if (nwords_ == 0 || nsym_ - nwords_ >= (1ull << 31)) return false;  // hipcub sizes are int
  std::vector<uint32_t> wlen(nwords_);
  for (uint32_t w = 0; w < nwords_; ++w) {
    wlen[w] = woff[w + 1] - woff[w];
    if (wlen[w] == 0) return false;  // words are never empty (strtok)
  }
  weight_ = reinterpret_cast<const unsigned long long*>(d_weight);
  woff_h_ = woff;
  wtok_ = wl_alloc<int32_t>(nsym_ + 4, &bytes_);
  wtok0_ = wl_alloc<int32_t>(nsym_ + 4, &bytes_);
  woff_ = wl_alloc<uint32_t>(nwords_ + 1, &bytes_);
  wlen_ = wl_alloc<uint32_t>(nwords_, &bytes_);
  wlen0_ = wl_alloc<uint32_t>(nwords_, &bytes_);
  wmark_ = wl_alloc<uint32_t>(nwords_, &bytes_);
  tile_first_ = wl_alloc<uint32_t>(ntiles_, &bytes_);
  tile_nw_ = wl_alloc<uint32_t>(ntiles_, &bytes_);
  hipStream_t s = S(stream_);
  WL_OK(hipMemcpyAsync(wtok0_, wtok.data(), nsym_ * sizeof(int32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(woff_, woff.data(), woff.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(wlen0_, wlen.data(), nwords_ * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(tile_first_, tfirst.data(), ntiles_ * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(tile_nw_, tnw.data(), ntiles_ * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(wtok_, wtok0_, nsym_ * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  WL_OK(hipMemcpyAsync(wlen_, wlen0_, nwords_ * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  WL_OK(hipMemsetAsync(wmark_, 0, nwords_ * sizeof(uint32_t), s));
  // index capacity: the initial entries (< S), plus <= 2 per occurrence merged (Σ <= S) for
  // the run and its undone guesses; directory at most 3/4 full
  const uint64_t npairs = nsym_ - nwords_;
  pool_cap_ = npairs + 4 * nsym_ + 4096;
  pool_ = wl_alloc<uint32_t>(pool_cap_, &bytes_);
  uint64_t want = 2 * (std::min<uint64_t>(npairs, 1ull << 24) + 2 * nsym_) + 4096;
  dir_cap_ = 1ull << 16;
  while (dir_cap_ < want && dir_cap_ < (1ull << 28)) dir_cap_ <<= 1;
  dkey_ = wl_alloc<u64>(dir_cap_, &bytes_);
  dval_ = wl_alloc<u64>(dir_cap_, &bytes_);
  dseq_ = wl_alloc<uint32_t>(dir_cap_, &bytes_);
  stage_cap_ = nsym_ + 4096;  // a merge stages <= 2 pairs per occurrence, <= 1 per token of a word
  for (int k = 0; k < 2; ++k) {
    stage_key_[k] = wl_alloc<u64>(stage_cap_, &bytes_);
    stage_w_[k] = wl_alloc<uint32_t>(stage_cap_, &bytes_);
  }
  stage_slot_ = wl_alloc<uint32_t>(stage_cap_, &bytes_);
  dstate_ = wl_alloc<uint32_t>(8, &bytes_);
  WL_OK(hipMemsetAsync(dstate_, 0, 8 * sizeof(uint32_t), s));
  reserve(kBaseVocab + 1);
  build_index();
  ready_ = true;
  dirty_ = false;
  return true;
}

// The index of the current words: every (pair, word) once, grouped by pair.
void WordLoop::build_index() {
  hipStream_t s = S(stream_);
  const uint64_t n = nsym_ - nwords_;
  size_t acc = 0;
  u64* kin = wl_alloc<u64>(n, &acc);
  u64* kout = wl_alloc<u64>(n, &acc);
  uint32_t* vin = wl_alloc<uint32_t>(n, &acc);
  uint32_t* vout = wl_alloc<uint32_t>(n, &acc);
  uint32_t* keep = wl_alloc<uint32_t>(n + 1, &acc);
  uint32_t* head = wl_alloc<uint32_t>(n + 1, &acc);
  uint32_t* pos = wl_alloc<uint32_t>(n + 1, &acc);
  uint32_t* kidx = wl_alloc<uint32_t>(n + 1, &acc);
  const int grid = 2048;
  k_wl_emit_pairs<<<grid, 256, 0, s>>>(wtok_, woff_, wlen_, nwords_, unk_, kin, vin);
  WL_OK(hipGetLastError());
  size_t tmp_bytes = 0, tb2 = 0;
  WL_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kin, kout, vin, vout, (int)n, 0, 64, s));
  WL_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, keep, pos, (int)n + 1, s));
  tmp_bytes = std::max(tmp_bytes, tb2);
  void* tmp = wl_alloc<uint8_t>(tmp_bytes, &acc);
  WL_OK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, vout, (int)n, 0, 64, s));
  WL_OK(hipMemsetAsync(keep + n, 0, sizeof(uint32_t), s));
  WL_OK(hipMemsetAsync(head + n, 0, sizeof(uint32_t), s));
  k_wl_mark<<<grid, 256, 0, s>>>(kout, vout, n, keep, head);
  WL_OK(hipGetLastError());
  WL_OK(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, keep, pos, (int)n + 1, s));
  WL_OK(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, head, kidx, (int)n + 1, s));
  uint32_t tot[2] = {0, 0};
  WL_OK(hipMemcpyAsync(&tot[0], pos + n, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  WL_OK(hipMemcpyAsync(&tot[1], kidx + n, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  WL_OK(hipStreamSynchronize(s));
  init_pool_n_ = tot[0];
  init_keys_n_ = tot[1];
  if (init_key_) WL_OK(hipFree(init_key_));
  if (init_val_) WL_OK(hipFree(init_val_));
  init_key_ = wl_alloc<u64>(init_keys_n_, &bytes_);
  init_val_ = wl_alloc<u64>(init_keys_n_, &bytes_);
  k_wl_scatter<<<grid, 256, 0, s>>>(kout, vout, n, keep, pos, head, kidx, pool_, init_key_, init_val_);
  WL_OK(hipGetLastError());
  k_wl_counts<<<256, 256, 0, s>>>(init_val_, init_keys_n_, init_pool_n_);
  WL_OK(hipGetLastError());
  WL_OK(hipStreamSynchronize(s));
  for (void* p : {(void*)kin, (void*)kout, (void*)vin, (void*)vout, (void*)keep, (void*)head, (void*)pos, (void*)kidx,
                  tmp})
    WL_OK(hipFree(p));
  restore_index();
}

// The directory and counters as right after build_index().
void WordLoop::restore_index() {
  hipStream_t s = S(stream_);
  WL_OK(hipMemsetAsync(dkey_, 0xFF, dir_cap_ * sizeof(u64), s));
  if (init_keys_n_) {
    k_wl_dir_init<<<1024, 256, 0, s>>>(init_key_, init_val_, init_keys_n_, dkey_, dval_, dseq_, dir_cap_ - 1);
    WL_OK(hipGetLastError());
  }
  if (valid_seq_) WL_OK(hipMemsetAsync(valid_seq_, 0, id_cap_ * sizeof(uint32_t), s));
  const uint32_t st[4] = {0, (uint32_t)init_pool_n_, (uint32_t)init_keys_n_, 0};
  WL_OK(hipMemcpyAsync(dstate_, st, sizeof(st), hipMemcpyHostToDevice, s));
  WL_OK(hipStreamSynchronize(s));
}

bool WordLoop::load_current(const TiledStream& ts) {
  WL_OK(hipSetDevice(ordinal_));
  if (!ready_ || !posted_.empty()) return false;
  stop();
  std::vector<int32_t> wtok(nsym_, 0);
  std::vector<uint32_t> wlen(nwords_, 0);
  uint32_t w = 0;
  bool open = false;
  for (size_t t = 0; t < ts.num_tiles(); ++t) {
    const int32_t* p = ts.tok.data() + ts.off[t];
    for (uint32_t i = 0; i < ts.len[t]; ++i) {
      if (p[i] < kHeaderLimit) {
        if (open) ++w;
        if ((uint32_t)(p[i] - kHeaderBase) != w || w >= nwords_) return false;
        open = true;
      } else {
        if (!open || wlen[w] >= woff_h_[w + 1] - woff_h_[w]) return false;
        wtok[woff_h_[w] + wlen[w]++] = p[i];
      }
    }
  }
  if (!open || w + 1 != nwords_) return false;
  hipStream_t s = S(stream_);
  WL_OK(hipMemcpyAsync(wtok_, wtok.data(), nsym_ * sizeof(int32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(wlen_, wlen.data(), nwords_ * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipStreamSynchronize(s));
  build_index();
  dirty_ = false;
  return true;
}

void WordLoop::reset() {
  WL_OK(hipSetDevice(ordinal_));
  if (!ready_) return;
  if (!posted_.empty()) fatal("WordLoop::reset with a merge in flight");
  stop();
  hipStream_t s = S(stream_);
  WL_OK(hipMemcpyAsync(wtok_, wtok0_, nsym_ * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  WL_OK(hipMemcpyAsync(wlen_, wlen0_, nwords_ * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  restore_index();
  dirty_ = false;
}

void WordLoop::ensure_slots(uint32_t cap) {
  const uint32_t rec_cap = 4 * (cap + 1) + 64;
  const unsigned pin = hipHostMallocMapped | hipHostMallocCoherent;
  for (Slot& sl : slot_) {
    if (sl.host_recs) WL_OK(hipHostFree(sl.host_recs));
    WL_OK(hipHostMalloc((void**)&sl.host_recs, (size_t)rec_cap * sizeof(DeltaRecord), pin));
    WL_OK(hipHostGetDevicePointer(&sl.dev_recs, sl.host_recs, 0));
    if (!sl.host_hdr) {
      WL_OK(hipHostMalloc((void**)&sl.host_hdr, 64, pin));
      std::memset(sl.host_hdr, 0, 64);
      WL_OK(hipHostGetDevicePointer(&sl.dev_hdr, sl.host_hdr, 0));
    }
    sl.rec_cap = rec_cap;
  }
}

void WordLoop::reserve(int32_t max_id) {
  // + kSlots: the guesses posted past the last merge of a batch (rolled back at its end) use ids
  // up to max_id + kSlots - 1, and the tables can grow only while nothing is in flight
  const uint32_t need = (uint32_t)std::max<int32_t>(max_id, 0) + 2 + kSlots;
  if (need <= cap_ && dsum_) return;
  if (!posted_.empty()) fatal("WordLoop::reserve with a merge in flight");
  stop();
  uint32_t cap = std::max<uint32_t>(cap_ ? cap_ : 4096, 4096);
  while (cap < need) cap *= 2;
  hipStream_t s = S(stream_);
  for (void* p : {(void*)dsum_, (void*)dft_, (void*)dlist_})
    if (p) WL_OK(hipFree(p));
  const size_t keys = 4 * ((size_t)cap + 1);
  dsum_ = wl_alloc<u64>(keys, &bytes_);
  dft_ = wl_alloc<u64>(keys, &bytes_);
  dlist_ = wl_alloc<uint32_t>(keys, &bytes_);
  WL_OK(hipMemsetAsync(dsum_, 0, keys * sizeof(u64), s));
  WL_OK(hipMemsetAsync(dft_, 0xFF, keys * sizeof(u64), s));
  uint32_t* vs = wl_alloc<uint32_t>(cap, &bytes_);
  WL_OK(hipMemsetAsync(vs, 0, (size_t)cap * sizeof(uint32_t), s));
  if (valid_seq_) {
    WL_OK(hipMemcpyAsync(vs, valid_seq_, (size_t)id_cap_ * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    WL_OK(hipStreamSynchronize(s));
    WL_OK(hipFree(valid_seq_));
  }
  valid_seq_ = vs;
  id_cap_ = cap;
  cap_ = cap;
  ensure_slots(cap);
  WL_OK(hipStreamSynchronize(s));
}

void WordLoop::launch() {
  WlParams p{};
  p.wtok = wtok_;
  p.woff = woff_;
  p.wlen = wlen_;
  p.wmark = wmark_;
  p.weight = weight_;
  p.nwords = nwords_;
  p.pool = pool_;
  p.pool_cap = pool_cap_;
  p.dkey = dkey_;
  p.dval = dval_;
  p.dseq = dseq_;
  p.dir_mask = dir_cap_ - 1;
  p.valid_seq = valid_seq_;
  p.id_cap = id_cap_;
  p.sk[0] = stage_key_[0];
  p.sk[1] = stage_key_[1];
  p.sw[0] = stage_w_[0];
  p.sw[1] = stage_w_[1];
  p.sslot = stage_slot_;
  p.stage_cap = stage_cap_;
  p.dsum = dsum_;
  p.dft = dft_;
  p.dlist = dlist_;
  p.dstate = dstate_;
  p.cap = cap_;
  p.unk = unk_;
  p.ring = static_cast<const WlCmd*>(ring_dev_);
  p.status = static_cast<uint32_t*>(status_dev_);
  p.seq0 = seq_ + 1;
  p.idle_polls = 1u << 22;  // ~10 s without a command: the launch ends itself (the host relaunches)
  for (int k = 0; k < kSlots; ++k) {
    p.sl[k].recs = static_cast<DeltaRecord*>(slot_[k].dev_recs);
    p.sl[k].hdr = static_cast<uint32_t*>(slot_[k].dev_hdr);
    p.sl[k].rec_cap = slot_[k].rec_cap;
  }
  status_[0] = 0;
  WL_OK(hipEventRecord((hipEvent_t)ev_[0], S(stream_)));
  k_word_loop<<<1, kWlThreads, 0, S(stream_)>>>(p);
  WL_OK(hipGetLastError());
  WL_OK(hipEventRecord((hipEvent_t)ev_[1], S(stream_)));
  running_ = true;
  ++st_.launches;
}

uint32_t WordLoop::post(uint32_t op, int32_t a, int32_t b, int32_t X) {
  if (running_ && __atomic_load_n(&status_[0], __ATOMIC_ACQUIRE) == kOpTimeout) {
    if (!posted_.empty()) fatal("k_word_loop ended on its time-out with merges in flight");
    WL_OK(hipStreamSynchronize(S(stream_)));
    running_ = false;
  }
  if (!running_) {
    if (op == kOpStop) return 0;
    launch();
  }
  const uint32_t seq = ++seq_;
  const uint32_t slot = (uint32_t)X & (kSlots - 1);
  u64* g = static_cast<WlCmd*>(ring_)[seq % kRing].g;
  const uint32_t vals[4] = {op | (slot << 8), (uint32_t)a, (uint32_t)b, (uint32_t)X};
  for (int k = 0; k < 4; ++k) __atomic_store_n(&g[k], (u64)seq | ((u64)vals[k] << 32), __ATOMIC_RELAXED);
  std::atomic_thread_fence(std::memory_order_release);
  return seq;
}

void WordLoop::post_merge(int32_t a, int32_t b, int32_t X) {
  if (!ready_) fatal("WordLoop::post_merge before upload");
  if (posted_.size() >= (size_t)kSlots) fatal("WordLoop: every merge slot is in flight");
  if (X < 0 || (uint32_t)X + 2 > cap_) fatal("WordLoop: merge id beyond the reserved ids");
  Slot& sl = slot_[(uint32_t)X & (kSlots - 1)];
  (void)sl;
  const uint32_t seq = post(kOpMerge, a, b, X);
  posted_.push_back({X, a, b, seq, now_seconds()});
  dirty_ = true;
}

void WordLoop::wait_flag(const Slot& sl, uint32_t seq) {
  volatile uint32_t* flag = sl.host_hdr + 1;
  const double t0 = now_seconds();
  unsigned spins = 0;
  while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
    __builtin_ia32_pause();
    if (++spins % 4096 != 0) continue;
    if (__atomic_load_n(&status_[0], __ATOMIC_ACQUIRE) != 0) fatal("k_word_loop ended with a merge in flight");
    if (now_seconds() - t0 > 60.0) {
      const hipError_t e = hipStreamQuery(S(stream_));
      if (e != hipSuccess && e != hipErrorNotReady) WL_OK(e);
      if (now_seconds() - t0 > 300.0) fatal("k_word_loop did not signal completion within 300 s");
    }
  }
}

size_t WordLoop::collect(int32_t X, const DeltaRecord** recs) {
  if (posted_.empty() || posted_.front().X != X) fatal("WordLoop::collect: X is not the oldest posted merge");
  const Post pp = posted_.front();
  posted_.erase(posted_.begin());
  const Slot& sl = slot_[(uint32_t)X & (kSlots - 1)];
  wait_flag(sl, pp.seq);
  st_.wait_us += 1e6 * (now_seconds() - pp.t_post);
  const uint32_t* h = sl.host_hdr;
  const size_t n = h[0];
  st_.merges += 1;
  st_.candidates += h[2];
  st_.changed += h[3];
  st_.occurrences += reinterpret_cast<const uint64_t*>(h)[2];
  st_.dev_us += 1e-2 * (double)reinterpret_cast<const uint64_t*>(h)[3];  // s_memrealtime: 100 MHz
  if (n > sl.rec_cap) fatal("k_word_loop: record overflow");
  *recs = sl.host_recs;
  return n;
}

void WordLoop::rollback(int32_t X) {
  while (!posted_.empty() && posted_.back().X >= X) {
    const Post pp = posted_.back();
    posted_.pop_back();
    // no wait: the loop takes commands in order, so the undo follows the guess
    post(kOpUnmerge, pp.a, pp.b, pp.X);
    ++st_.undos;
  }
}

void WordLoop::stop() {
  if (!running_) return;
  WL_OK(hipSetDevice(ordinal_));
  if (!posted_.empty()) fatal("WordLoop::stop with a merge in flight");
  post(kOpStop, 0, 0, 0);
  WL_OK(hipStreamSynchronize(S(stream_)));
  running_ = false;
  float ms = 0;
  WL_OK(hipEventElapsedTime(&ms, (hipEvent_t)ev_[0], (hipEvent_t)ev_[1]));
  st_.kernel_ms += ms;
  uint32_t ds[4];
  WL_OK(hipMemcpy(ds, dstate_, sizeof(ds), hipMemcpyDeviceToHost));
  if (ds[kStError]) {
    static const char* what[] = {"", "index pool exhausted", "new-pair staging overflow", "index directory full",
                                 "a merged pair had no word list"};
    std::fprintf(stderr, "[ERROR]\t k_word_loop: %s (code %u)\n", ds[kStError] < 5 ? what[ds[kStError]] : "?",
                 ds[kStError]);
    fatal("k_word_loop failed");
  }
}

uint64_t WordLoop::pool_used() const {
  uint32_t v = 0;
  if (dstate_) WL_OK(hipMemcpy(&v, dstate_ + kStPoolTop, sizeof(v), hipMemcpyDeviceToHost));
  return v;
}

void WordLoop::sync_tiles(int32_t* tok, const uint64_t* tile_off, uint32_t* tile_len) {
  if (!dirty_ || !ready_) return;
  if (running_) stop();
  const int grid = (int)std::min<uint32_t>((ntiles_ + 3) / 4, 4096);
  k_words_to_tiles<<<std::max(grid, 1), 256, 0, S(stream_)>>>(wtok_, woff_, wlen_, tile_first_, tile_nw_, ntiles_, tok,
                                                           tile_off, tile_len);
  WL_OK(hipGetLastError());
  dirty_ = false;
}

}  // namespace shred
