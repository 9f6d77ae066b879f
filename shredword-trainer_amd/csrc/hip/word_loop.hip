// MI355X (gfx950) kernels of the indexed merge loop (host/word_loop.h) and its host driver.
//
//   k_word_loop       the merge loop: one persistent workgroup (16 wave64s) that takes merge /
//                     undo commands from a ring in pinned host memory.  Per merge (a, b) -> X:
//                     the word list of (a, b) (the words-of list of a or b, or the initial pair
//                     directory); a lane per listed word loads the word's run with seven 16-B
//                     loads into an LDS strip, scans it greedily left to right (reference
//                     bpe.cpp:265-296), emits the four neighbour deltas per occurrence into an LDS
//                     hash keyed (neighbour slot, category) with Σ weight and min first touch
//                     (FreqChangeMap, bpe.cpp:9-50), compacts the word in place and appends it to
//                     the words of X when it changed; the records go to host memory behind one
//                     system release and a flag.
//   k_wl_emit_pairs   initial index: every adjacent non-unk pair of every word -> (key, word)
//   k_wl_mark / k_wl_scatter / k_wl_counts / k_wl_dir_init   sorted runs -> pool + directory
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
#include <functional>
#include <thread>
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

constexpr int kWlThreads = 512;
constexpr int kDh = 2048;               // LDS delta hash slots
constexpr int kStripV = 7;              // 16-B loads per word run: [length][weight lo, hi][25 tokens]
constexpr int kStrip = 4 * kStripV;     // ints per lane in the LDS strip
// A run's header: its live length, then the word's weight (u64, the count of the word) inline, so
// that the run's loads bring it and a scanned word costs no separate weight line (round 6: a third
// of the loop's HBM read requests were those lines)
constexpr uint32_t kRunHdr = 3;
constexpr uint32_t kStripTok = kStrip - kRunHdr;
// Runs are 16-B aligned with a capacity of whole 16-B groups.  (Round 6 measured 128-B aligned
// runs: one L2 line per run load, HBM reads of the loop -30%, but the table grew 2.5x, past what
// the MALL keeps, and the loop got slower; the groups a word needs ride in its pool entries
// instead, see WEnt.)
constexpr uint32_t kRunAlign = 4;  // ints
__host__ __device__ constexpr uint32_t run_cap(uint32_t len) {
  return (kRunHdr + len + kRunAlign - 1u) & ~(kRunAlign - 1u);
}
constexpr int kB = 8;                   // pool entries per lane per scan round (one load batch)
#ifdef SHRED_WL_NO_PREFETCH
constexpr bool kWlPrefetch = false;     // (A/B builds) each word's run loaded in its own iteration
#else
constexpr bool kWlPrefetch = true;      // the next word's run loads while this one merges
#endif
constexpr int kQ = kWlThreads * kB + kWlThreads;
// tiebreak=device (k_word_loop<true>) holds its LDS frontier beside the loop's arrays: it queues
// 6 entries a lane per round so that everything fits the 160 KB of LDS
constexpr int kBSelf = 6;
template <bool kSelf>
struct QueueShape {
  static constexpr int kBatch = kSelf ? kBSelf : kB;
  static constexpr int kCap = kWlThreads * kBatch + kWlThreads;
};
// Diagnostic builds (-DSHRED_WL_STAMPS, tools/build_variant.sh): per-merge phase stamps of the
// indexed loop in header words [32, 44) (WordLoop::collect puts them in the trace)
#ifdef SHRED_WL_STAMPS
#define WL_ST(...) __VA_ARGS__
#else
#define WL_ST(...)
#endif
constexpr int kXs = 16;
// A/B builds (-DSHRED_WL_NT_WORDS): the word-run write-backs and pool appends as nontemporal stores
typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16(void* dst, int4 v) {
#ifdef SHRED_WL_NT_WORDS
  v4i_t x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<v4i_t*>(dst));
#else
  *reinterpret_cast<int4*>(dst) = v;
#endif
}
// stamps build: wave 0's clock (ticks after t0) into xs[i], written by its first active lane (a
// scalar clock read and one LDS store: no per-lane atomics, which would cost more than the stamped work)
__device__ __forceinline__ void wl_stamp(uint32_t* xs, int i, unsigned long long t0) {
#ifdef SHRED_WL_STAMPS
  const unsigned long long now = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x >> 6) == 0 && (threadIdx.x & 63) == (uint32_t)(__ffsll((long long)__ballot(1)) - 1))
    xs[i] = (uint32_t)(now - t0);
#endif
}  // LDS queue of filtered entries (a round + a remainder)
constexpr uint32_t kDeltaBucketsDev = 1024;  // the reference's FREQ_CHANGE_BUCKETS (bpe.cpp:16)
constexpr uint32_t kRing = 64;          // command ring entries
constexpr uint32_t kOpMerge = 1, kOpStop = 2, kOpTimeout = 3, kOpUnmerge = 4;
constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;
constexpr u64 kEmpty64 = ~0ull;
constexpr uint32_t kNoList = 0xFFFFFFFFu;
// dstate words: [1] pool top, [3] error
constexpr int kStPoolTop = 1, kStError = 3;
// error codes (dstate[kStError], reported by the host)
constexpr uint32_t kErrPool = 1, kErrList = 2, kErrLookup = 4;

struct WlCmd {
  // granules (seq | value << 32): op | slot << 8, a, b, X, then the words-of list of max(a, b)
  // when the host knows it (offset, count + 1; 0: look it up), one 64-B line
  u64 g[8];
};
constexpr int kCmdGranules = 6;

struct WlSlotDev {
  DeltaRecord* recs;  // host-visible
  uint32_t* hdr;      // host-visible: [0] records, [1] flag, [2] listed words, [3] changed words,
                      //   [4..5] occurrences (u64), [6..7] device ticks command -> flag (u64),
                      //   [8..9] ticks command -> list known, [10..11] ticks command -> words merged,
                      //   [12] words whose runs were read, [13] 1: a filtered words-of list,
                      //   [14] run ints read (length + tokens), [15] run ints written back,
                      //   [16..18] stamps (10 ns ticks after the command, thread 0): pool entries
                      //   loaded, first run loaded, first word merged
  uint32_t rec_cap;
};

// A pool entry: the word and a 64-bit filter.  In the words-of list of id M (the words merge M
// changed) the filter holds a bit per (neighbour, side) of M in the word right after merge M:
// nbit(p, 0) for each left neighbour p (X when just produced), nbit(n, 1) for each original
// token n after the pair.  A merge never makes two older ids adjacent, so every adjacency
// (c, M) / (M, d) the word holds later it held right after merge M: a word holding the pair
// now has its bit.  Initial-index entries (exact lists) hold all ones.
struct WEnt {
  u64 e;    // run offset << 32 | groups << 28 | word id (groups: the 16-B groups of the word's run
            // capacity, at most kStripV: a word's run load issues only those, round 6)
  u64 sig;
};
// The small-merge path hands its records over without ordering them before the flag (round 6):
// the records, the header and two tagged checksum granules go out back to back behind one release
// fence, and the host accepts them once both granules carry the command's tag and the checksum of
// header words 0..31 and the records matches (so a record still in flight is never read).  The
// checksum weighs word i by an odd constant of its position, so records swapped between positions
// or a stale block do not cancel out.
__host__ __device__ __forceinline__ u64 hand_weight(uint32_t i) { return 0x9E3779B97F4A7C15ull + 2ull * i; }
constexpr int kCksWord = 30;  // header u64 words 30, 31: seq << 32 | checksum low / high half
constexpr int kGroupShift = 28;
constexpr u64 kWordMask = (1ull << kGroupShift) - 1;
__host__ __device__ __forceinline__ uint32_t ent_groups(u64 e) { return (uint32_t)(e >> kGroupShift) & 0xFu; }

// tiebreak=device (K5 as the selector, WordLoop::run_select): the loop picks its own merges from
// a pair table on the device.  Table: open addressing on the pair key, 16 B a slot -- the key,
// then a word holding the count (low 48 bits) and the slot's frontier position + 1 (high 16
// bits, 0: not in the frontier), so one atomicAdd on the word both counts and tells where the
// LDS copy is (pairs holding unk are never in it).  Frontier: the slots of every pair ranked at or above a threshold
// (count desc, key asc) plus stale ones; each merge takes the best live frontier entry, and pairs
// a merge creates above the threshold join it (only new pairs ever gain: every other count only
// falls).  An empty frontier sends the launch back to the host, which rebuilds it whole-chip.
struct SelParams {
  u64* tab;           // slot h: tab[2h] pair key (kEmpty64 = empty), tab[2h + 1] count | pos + 1 << 48
  u64 pmask;
  uint32_t* fr[2];    // frontier buffers (slots); st[kSelBuf] says which is current
  uint32_t fcap;
  uint32_t* st;       // see kSel* below
  const u64* thr;     // threshold (count, key): every pair ranked at or above it is in the frontier
  u64* out;           // per merge: key, count
  u64* log;           // the launch's pair-count changes (key, signed delta), applied to the table between launches
  u64 log_cap;        //   entries
  int32_t X0;         // id of merge 0 of this training
  uint32_t n_max;     // merges wanted
  u64 min_freq;
  uint32_t fill_max;  // inserts allowed before the table counts as full
  uint32_t probe;     // diagnostic (SHREDWORD_SEL_PROBE): 1 skips the table's HBM updates (timing only: wrong counts)
};
// st words
constexpr int kSelM = 0, kSelNF = 1, kSelBuf = 2, kSelStatus = 3, kSelIns = 4, kSelErr = 5, kSelStats = 6;
constexpr int kSelWords = kSelStats + 2 * 12 + 2;  // st: 6 words, then 12 u64 statistics, then the log's length (u64)
constexpr int kSelLogW = kSelStats + 2 * 12;
// exit status: merges done (target reached / below min_pair_freq), frontier to rebuild, table full
// (the in-kernel fill bound: one more merge's new pairs might not fit; the host grows the table)
constexpr uint32_t kSelDone = 1, kSelRebuild = 2, kSelFull = 3;
// The frontier lives in LDS for the whole launch: each entry's count follows the table's (the
// merge's records add to both; inf[slot] = LDS position + 1), so a select is an LDS scan.  A
// rebuild picks kSelK entries; merges append, and past kSelF - kSelSlack entries the dead ones
// (below the threshold, or merged) are compacted away in LDS.  When more than kSelF - kSelRoom
// stay live the launch ends for a rebuild (a compaction per merge would cost more).
constexpr uint32_t kSelF = 1536, kSelK = 768, kSelRoom = 384, kSelSlack = 96;
constexpr u64 kCntMask = (1ull << 48) - 1;  // the count in a slot's count word; pos + 1 above it
constexpr int kPosShift = 48;
template <bool kOn>
struct SelLds {  // k_word_loop<false>: none
  u64 key[1], cnt[1];
  uint32_t idx[1], n;
};
// The frontier's LDS index (round 5): pair key -> position + 1 (16 bits, two to a word), so a
// record finds its pair's LDS copy without a table round trip, and the table's count words carry
// no positions (the table's atomics need no return value).
constexpr uint32_t kSelIdx = 4096;
template <>
struct SelLds<true> {
  u64 key[kSelF], cnt[kSelF];
  uint32_t idx[kSelIdx / 2], n;
};
struct WlParams {
  int32_t* wtok;
  const u64* weight;
  WEnt* pool;
  u64 pool_cap;
  const u64* dkey;
  const u64* dval;
  u64 dir_mask;
  u64* lst;          // per id: words-of list, pool offset | count << 32
  uint32_t* lseq;    // per id: the command that made it (~0: none)
  uint32_t id_cap;
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
  uint32_t fin_max;  // K4 on the device: merges with at most this many records leave as ordered changes (0: off)
  uint32_t fin_min;  //   and at least this many (> 0: the small-merge path stays on; its merges leave raw)
  uint32_t prefetch;  // 1: the poller wave reads the next command while the records go out (exact mode)
  // 1: the merge's barriers drain every wave's stores (0: only with spills or K4).  With 0 the
  // word-run (wtok), pool and lst stores of a merge may still be in flight when its flag is raised;
  // that is sound only because nothing reads them before the next command's __syncthreads, which
  // drains them, and the host never reads them while the loop runs.  Any new reader of wtok, pool
  // or lst inside a merge's records phase, or on the host after a flag, needs drain = 1 (K4 sets
  // it: finalize reads the merged words).  tests/test_gpu_parity.py runs both modes.
  uint32_t drain;
  uint32_t fast;      // 1: merges listing <= kWlThreads words take the small-merge path (exact mode)
  WlSlotDev sl[WordLoop::kSlots];
  SelParams sel;  // k_word_loop<true> only
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
__device__ __forceinline__ uint32_t sel_idx_home(u64 k) { return (uint32_t)(mix64(k) >> 40) & (kSelIdx - 1); }
// position of key in the frontier, or -1 (also for a dead entry never compacted: those are found
// and their counts kept, harmlessly)
__device__ __forceinline__ int sel_idx_find(const SelLds<true>& F, u64 k) {
  uint32_t h = sel_idx_home(k);
#pragma unroll 1
  for (uint32_t probe = 0; probe < kSelIdx; ++probe) {
    const uint32_t v = (F.idx[h >> 1] >> ((h & 1u) * 16u)) & 0xFFFFu;
    if (v == 0) return -1;
    if (F.key[v - 1u] == k) return (int)(v - 1u);
    h = (h + 1u) & (kSelIdx - 1u);
  }
  return -1;
}
__device__ __forceinline__ bool sel_idx_insert(SelLds<true>& F, u64 k, uint32_t pos) {
  uint32_t h = sel_idx_home(k);
#pragma unroll 1
  for (uint32_t probe = 0; probe < kSelIdx;) {
    const uint32_t sh = (h & 1u) * 16u;
    const uint32_t old = F.idx[h >> 1];
    if (((old >> sh) & 0xFFFFu) == 0u) {
      if (atomicCAS(&F.idx[h >> 1], old, old | ((pos + 1u) << sh)) == old) return true;
      continue;  // the word changed under us: look again
    }
    h = (h + 1u) & (kSelIdx - 1u);
    ++probe;
  }
  return false;
}

__device__ __forceinline__ uint32_t slot_of(int32_t id, uint32_t cap) {
  return (uint32_t)id < cap ? (uint32_t)id + 1u : 0u;
}
// filter bit of neighbour id on side s (0: left of M, 1: right of M)
__device__ __forceinline__ u64 nbit(int32_t id, uint32_t s) {
  const uint32_t v = (uint32_t)id * 2u + s;
  return 1ull << ((v ^ (v >> 6) ^ (v >> 12) ^ (v >> 18)) & 63u);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld_agent64(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// tiebreak=device order: larger count first, then the smaller key
__device__ __forceinline__ bool sel_better(u64 c, u64 k, u64 c2, u64 k2) { return c > c2 || (c == c2 && k < k2); }
__device__ __forceinline__ bool sel_at_least(u64 c, u64 k, u64 tc, u64 tk) { return c > tc || (c == tc && k <= tk); }
// The table slot of pair key pk, inserted when absent (~0 when the table is past its probe bound).
// ins / err: counters of inserts and probe overflows (LDS in the loop, global in k_sel_insert).
__device__ __forceinline__ u64 sel_slot(const SelParams& q, u64 pk, uint32_t* ins, uint32_t* err) {
  u64 h = mix64(pk) & q.pmask;
#pragma unroll 1
  for (uint32_t probe = 0; probe < 4096u; ++probe) {
    const u64 cur = ld_agent64(q.tab + 2 * h);
    if (cur == pk) return h;
    if (cur == kEmpty64) {
      const u64 prev = atomicCAS(q.tab + 2 * h, kEmpty64, pk);
      if (prev == kEmpty64) {
        atomicAdd(ins, 1u);
        return h;
      }
      if (prev == pk) return h;
    }
    h = (h + 1) & q.pmask;
  }
  atomicMax(err, 1u);
  return ~0ull;
}
// One combined record of merge (a, b) -> X as a change of a pair's count (the reference's
// FreqChangeMap entry, bpe.cpp:297-313, minus the pair merged and pairs holding unk).  The table
// is only read between launches (the frontier's rebuild), so its change is logged (a coalesced
// store, no round trip) and applied in bulk by k_sel_apply_log; a pair already in the frontier gets
// it in LDS through the frontier's index.  Pairs holding X are new (their count was 0): their count
// is the sum of their records' deltas, listed in LDS (nkey / ncnt) for the frontier -- (X, a) has
// two records, NewRight(a) listed and OldLeft(X) summed into *dxa, added when it is appended.
struct SelNew {
  u64* key;
  u64* cnt;
  uint32_t* n;
  uint32_t cap;
  u64* dxa;
  uint32_t* over;
  u64* log;         // this merge's table changes go to log[0, *nlog)
  uint32_t* nlog;
};
__device__ __forceinline__ void sel_record(const SelParams& q, SelLds<true>& F, const SelNew& nw, int32_t unk,
                                           uint32_t key, u64 sum, int32_t a, int32_t b, int32_t X) {
  const uint32_t sl = key >> 2, cat = key & 3u;
  const int32_t id = sl == 0 ? unk : (int32_t)(sl - 1u);
  if (id == unk || sum == 0) return;
  const int32_t f = cat < 2u ? id : (cat == 2u ? b : X);
  const int32_t g = cat == 0u ? a : (cat == 1u ? X : id);
  if (f == a && g == b) return;
  const u64 pk = pair_key(f, g);
  const u64 d = (cat & 1u) ? sum : (u64)(-(int64_t)sum);
  if (!(q.probe & 1u)) {  // the table's change, applied between launches (k_sel_apply_log)
    const uint32_t j = atomicAdd(nw.nlog, 1u);
    nw.log[2 * (u64)j] = pk;
    nw.log[2 * (u64)j + 1] = d;
  }
  if (f != X && g != X) {
    const int pos = sel_idx_find(F, pk);
    if (pos >= 0) atomicAdd(reinterpret_cast<unsigned long long*>(&F.cnt[pos]), (unsigned long long)d);
  } else if (cat == 0u) {  // OldLeft(X): (X, a)
    atomicAdd(reinterpret_cast<unsigned long long*>(nw.dxa), (unsigned long long)d);
  } else {
    const uint32_t i = atomicAdd(nw.n, 1u);
    if (i < nw.cap) {
      nw.key[i] = pk;
      nw.cnt[i] = d;
    } else {
      *nw.over = 1u;  // the frontier may miss a pair: rebuild
    }
  }
}

struct DeltaH {
  uint32_t key[kDh];
  u64 sum[kDh];  // Σ weight
  u64 ft[kDh];   // min first touch
};

// The merge's shared state in LDS.
struct MergeCtx {
  uint32_t* nspill;  // delta keys spilled past the LDS hash
  uint32_t* nkeys;   // delta keys in the LDS hash
  uint32_t* kbits;   // their slots as a bitmap (kDh bits: the small-merge path's records and clear)
};

// Neighbour deltas (reference freq_change_add, bpe.cpp:274-290): Σ weight and min first touch
// per key = slot * 4 + category, in the LDS hash; keys past it go to the global spill tables.
// The four deltas of one occurrence (prev: the left neighbour after merging, X when just
// produced, has_l false at the word's start; n: the original token after the pair, has_n false
// at the word's end); returns its filter bits.  The four keys are probed together, so their CAS
// round trips overlap (one LDS latency a probe step instead of four), as delta_add would do
// them one by one; a key still unplaced after kProbes steps goes to the global spill tables.
// kProbes is a template argument so that the tests can force the spill path (kProbes 0: every key
// spills, 1: most of a busy merge's) with no cost to the default kernel (32; C3 spills one or two
// keys in 29,000 indexed merges).
constexpr int kProbesDefault = 32;

// Sum of a u32 over the wave by DPP row shifts and row broadcasts (lane 63 holds it), read back
// as a scalar.  Call it with every lane active (0 from lanes that add nothing).  A per-lane
// atomicAdd on one LDS word instead compiles to a loop over the active lanes (the compiler's
// iterative atomic combine: ~7 scalar instructions a lane), microseconds a merge at 64 lanes.
// Inclusive prefix sum of a u32 over the wave (same DPP steps; every lane active).
__device__ __forceinline__ uint32_t wave_scan32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

template <int kProbes>
__device__ __forceinline__ u64 occurrence(const WlParams& p, DeltaH& h, const MergeCtx& c, bool has_l, int32_t prev,
                                          bool has_n, int32_t n, u64 wc, u64 ft) {
  u64 f = 0;
  const uint32_t sl = slot_of(prev, p.cap) * 4u, sn = slot_of(n, p.cap) * 4u;
  const uint32_t key[4] = {sl + 0u, sl + 1u, sn + 2u, sn + 3u};
  bool pend[4] = {has_l, has_l, has_n, has_n};
  uint32_t slot[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) slot[k] = (key[k] * 2654435761u) >> (32 - 11);
#pragma unroll 1
  for (int probe = 0; probe < kProbes && (pend[0] | pend[1] | pend[2] | pend[3]); ++probe) {
    uint32_t prv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) prv[k] = pend[k] ? atomicCAS(&h.key[slot[k]], kEmpty32, key[k]) : 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (pend[k] && prv[k] == kEmpty32) {  // a key new to the hash: its slot's bit (no return values)
        atomicOr(&c.kbits[slot[k] >> 5], 1u << (slot[k] & 31u));
        atomicAdd(c.nkeys, 1u);
      }
      if (!pend[k]) continue;
      if (prv[k] == kEmpty32 || prv[k] == key[k]) {
        atomicAdd(&h.sum[slot[k]], wc);
        atomicMin(&h.ft[slot[k]], ft | (u64)k);
        pend[k] = false;
      } else {
        slot[k] = (slot[k] + 1) & (kDh - 1);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (pend[k]) {  // the LDS hash is full around this key: the global tables take it
      const u64 old = atomicAdd(&p.dsum[key[k]], wc);
      atomicMin(&p.dft[key[k]], ft | (u64)k);
      if (old == 0) p.dlist[atomicAdd(c.nspill, 1u)] = key[k];  // weights are >= 1
    }
  if (has_l) f |= nbit(prev, 0);
  if (has_n) f |= nbit(n, 1);
  return f;
}

// Merge (a, b) -> X in one word of L tokens read from HBM (t: its tokens), greedy left to right
// as the reference's chain walk (the path of words longer than the strip); returns the
// occurrences merged, the new length in *len and the filter bits in *sig.  First touch =
// (rank << 32) | (input position << 2) | category.
template <int kProbes>
__device__ __forceinline__ uint32_t merge_run(const WlParams& p, DeltaH& h, const MergeCtx& c, int32_t* t, uint32_t L,
                                              u64 e, u64 wc, int32_t a, int32_t b, int32_t X, uint32_t* len,
                                              u64* sig) {
  const u64 rank = (e & kWordMask) << 32;
  uint32_t j = 0, k = 0, occ = 0;
  u64 f = 0;
  int32_t prev = 0;
  int32_t c0 = t[0], c1 = L > 1 ? t[1] : 0;
#pragma unroll 1
  while (j < L) {
    if (j + 1 < L && c0 == a && c1 == b) {
      const bool has_n = j + 2 < L;
      const int32_t n = has_n ? t[j + 2] : 0;  // the original next token (bpe.cpp:283-289)
      const int32_t n2 = j + 3 < L ? t[j + 3] : 0;
      f |= occurrence<kProbes>(p, h, c, k > 0, prev, has_n, n, wc, rank | ((u64)j << 2));
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
  *len = k;
  *sig = f;
  return occ;
}

// A word's run: kStripV 16-B loads (one round trip), the length and up to kStripTok tokens.
struct Run {
  int4 v[kStripV];
};
__device__ __forceinline__ Run load_run(const int32_t* r, uint32_t groups = kStripV) {
  Run x;
  const int4* r4 = reinterpret_cast<const int4*>(r);
#pragma unroll
  for (int q = 0; q < kStripV; ++q) x.v[q] = (uint32_t)q < groups ? r4[q] : make_int4(0, 0, 0, 0);
  return x;
}
__device__ __forceinline__ u64 run_weight(const Run& x) {
  return (u64)(uint32_t)x.v[0].y | ((u64)(uint32_t)x.v[0].z << 32);
}
__device__ __forceinline__ int32_t run_at(const Run& x, int i) {
  const int4 q = x.v[i >> 2];
  return (i & 3) == 0 ? q.x : (i & 3) == 1 ? q.y : (i & 3) == 2 ? q.z : q.w;
}

// Merge (a, b) -> X in a word of L <= kStripTok tokens held in registers, in two passes so that
// a wave's lanes emit their deltas in lock step: (1) the greedy left-to-right walk, unrolled and
// branch-free over the registers (position j is taken by the pair (j, j + 1) unless the
// previous position was), writes the output to this lane's LDS strip (skipped positions write
// the length slot, rewritten last) and marks the output positions holding X; (2) per
// occurrence, lowest output position first, the four neighbour deltas — left neighbour
// out[k - 1] (X when just produced), right neighbour the original token after the pair
// (out[k + 1], or a where that is the next occurrence's X); input position of occurrence o at
// output k: k + o.  The changed run is written back with 16-B stores.  Same results as merge_run.
template <int kProbes>
__device__ __forceinline__ uint32_t merge_regs(const WlParams& p, DeltaH& h, const MergeCtx& c, int32_t* s,
                                               int32_t* r, const Run& x, uint32_t L, u64 e, u64 wc, int32_t a,
                                               int32_t b, int32_t X, uint32_t* len, u64* sig, uint32_t* xs = nullptr,
                                               u64 t0 = 0) {
  uint32_t k = 0, xm = 0;
  bool skip = false;
#pragma unroll
  for (int j = 0; j < (int)kStripTok; ++j) {
    if ((j & 3) == 0 && !__any((uint32_t)j < L)) break;  // every lane's word has ended
    const int32_t t0 = run_at(x, (int)kRunHdr + j);
    const int32_t t1 = j + 1 < (int)kStripTok ? run_at(x, (int)kRunHdr + 1 + j) : 0;
    const bool emit = (uint32_t)j < L && !skip;
    const bool m = emit && (uint32_t)(j + 1) < L && t0 == a && t1 == b;
    s[(emit ? kRunHdr + k : 0u) * kWlThreads] = m ? X : t0;
    xm |= (m ? 1u : 0u) << k;
    k += emit ? 1u : 0u;
    skip = m;
  }
  if (xs) wl_stamp(xs, 4, t0);  // (stamps build) the walk done
  *len = k;
  *sig = 0;
  if (!xm) return 0;
  const uint32_t occ = (uint32_t)__popc(xm);
  const u64 rank = (e & kWordMask) << 32;
  uint32_t m = xm, o = 0;
  u64 f = 0;
  while (__ballot(m != 0u)) {
    if (m) {
      const uint32_t ko = (uint32_t)__ffs(m) - 1u;
      m &= m - 1u;
      const uint32_t jo = ko + o;
      ++o;
      const int32_t prev = ko > 0 ? s[(kRunHdr - 1u + ko) * kWlThreads] : 0;  // out[ko - 1]
      const bool has_n = jo + 2 < L;
      const int32_t nx = has_n ? s[(kRunHdr + 1u + ko) * kWlThreads] : 0;  // out[ko + 1]
      f |= occurrence<kProbes>(p, h, c, ko > 0, prev, has_n, nx == X ? a : nx, wc, rank | ((u64)jo << 2));
    }
  }
  if (xs) wl_stamp(xs, 5, t0);  // the occurrences' deltas issued
  *sig = f;
  // the run [length][weight][k tokens] from the first 16-B group that changed
  s[0] = (int32_t)k;
  int4* r4 = reinterpret_cast<int4*>(r);
  const uint32_t q0 = ((uint32_t)__ffs(xm) + kRunHdr - 1u) >> 2;  // (kRunHdr + first X position) / 4
  int4 v[kStripV];  // every group read at once (one LDS wait), the changed ones stored
#pragma unroll
  for (int q = 0; q < kStripV; ++q) {
    v[q].x = s[(4 * q + 0) * kWlThreads];
    v[q].y = s[(4 * q + 1) * kWlThreads];
    v[q].z = s[(4 * q + 2) * kWlThreads];
    v[q].w = s[(4 * q + 3) * kWlThreads];
  }
  v[0].y = x.v[0].y;  // the weight, as it was
  v[0].z = x.v[0].z;
#pragma unroll
  for (int q = 0; q < kStripV; ++q)
    if ((uint32_t)q <= ((k + kRunHdr - 1u) >> 2) && (q == 0 || (uint32_t)q >= q0)) st16(&r4[q], v[q]);
  if (xs) wl_stamp(xs, 6, t0);  // the write-back issued
  return occ;
}

// Undo of merge X in one word (tokens t, L of them): every X back into (a, b), right to left in
// place; returns the new length.
__device__ __forceinline__ uint32_t unmerge_run(int32_t* t, uint32_t L, int32_t a, int32_t b, int32_t X) {
  uint32_t nx = 0;
  for (uint32_t j = 0; j < L; ++j) nx += t[j] == X;
  if (!nx) return L;
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
  return L + nx;
}

// Inclusive wave max of a u64 on DPP row shifts and row broadcasts (identity 0; lane 63 holds
// the wave's max): a few cycles a step instead of an LDS round trip per __shfl.
template <int kCtrl, int kRowMask = 0xf, bool kBound = true>
__device__ __forceinline__ u64 wl_dpp64(u64 x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, kCtrl, kRowMask, 0xf, kBound);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), kCtrl, kRowMask, 0xf, kBound);
  return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 wl_max64(u64 a, u64 b) { return a > b ? a : b; }
__device__ __forceinline__ u64 wave_max64(u64 x) {
  x = wl_max64(x, wl_dpp64<0x111>(x));
  x = wl_max64(x, wl_dpp64<0x112>(x));
  x = wl_max64(x, wl_dpp64<0x114>(x));
  x = wl_max64(x, wl_dpp64<0x118>(x));
  x = wl_max64(x, wl_dpp64<0x142, 0xa, false>(x));
  x = wl_max64(x, wl_dpp64<0x143, 0xc, false>(x));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63);
  return ((u64)hi << 32) | lo;
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

// The loop's state in LDS.
struct LoopS {
  alignas(16) uint32_t hs[32];  // the small-merge path's header, staged for 16-B stores (word 1 = 0: not the flag)
  uint32_t cmd[8];
  uint32_t nout, nchg, pool_top, err, scan, filter, nspill, qn, nkeys, nfin;
  uint32_t rd, wr;  // run ints read (length + tokens of every scanned word) / written back (changed words)
  u64 lst_x;        // the words-of list written for X (offset | (count + 1) << 32), for the host
  u64 last_lst;     // the last merge's X and its words-of list (offset | count << 32), kept in LDS so
  int32_t last_x;   //   that a merge of the pair the loop just made skips the list lookup (-1: none)
  uint32_t st[4];
  u64 lk[2];  // word list: pool offset, count
  u64 need;   // filter bits the listed words must hold
  u64 occ, t[2];
  u64 t_wait, t_idle, t_undo;  // s_memrealtime: this command's wait began; idle / undo since the last flag
  u64 t_seen;                   // (stamps build) the poller saw the command's granules tagged
  uint32_t t_rel;               // ticks of the last flag's system release (diagnostic)
  uint32_t xs[kXs];             // SHRED_WL_STAMPS: phase stamps (ticks after the command) and counts
  // tiebreak=device
  uint32_t sm, snk, snew, status, sel_pos, sover, scompact, sins, serr;
  u64 sel_cnt, dxa, t_rec, t_app, logn;
  uint32_t lognew, newtot;
  u64 bc[kWlThreads / 64], bk[kWlThreads / 64];
  uint32_t bs[kWlThreads / 64];
};


// K4 on the device (reference FreqChangeMap, bpe.cpp:9-50, applied at :297-313):
// the merge's n records (LDS hash + spilled keys) leave as the reference's changes, in the order
// the reference applies them, so the host only walks them.  Per record the pair (first, second)
// and its signed delta; records of one pair key combined (Σ delta, min first touch); the merged
// pair (a, b) dropped (the host skips it); order: bucket key % 1024 ascending, then first touch
// descending (the bucket chains' head insertion).  The key is the reference's
// ((u64)(i64)first << 32) | (u64)(i64)second, sign extension included (a negative second id
// makes every such key equal, as in the reference).  First touches are unique per record, so the
// min-first-touch record of a key leads it and a bucket's order is a rank by first touch.
// LDS (the merge's arrays are free by now): records in q (hk, delta, ft, then a bucket-sorted ft
// copy; kFinMax each), the combine table in the strip (hk, min ft, Σ delta; 2 kFinMax slots), the
// 1024 bucket counters in h.key.  Returns the changes written (host records, in order).
constexpr uint32_t kFinMax = 1024;
constexpr uint32_t kFinTab = 2 * kFinMax;
// the combine table's empty key: (INT32_MAX, INT32_MAX) is no pair's key (ids are < 2^30), while
// ~0 is one: (f, s) with a negative second id (unk = -1) sign-extends to all ones
constexpr u64 kFinEmpty = 0x7FFFFFFF7FFFFFFFull;
static_assert(4 * kFinMax <= (uint32_t)kQ, "record arrays in the queue");
static_assert(3 * kFinTab * 8 <= (uint32_t)(kStrip * kWlThreads * 4), "combine table in the strip");
static_assert(kDeltaBucketsDev * 4 <= kDh * 4, "bucket counters in the hash keys");

__device__ __forceinline__ void fin_record(u64* q, uint32_t r, uint32_t key, u64 sum, u64 ft, int32_t unk, int32_t a,
                                           int32_t b, int32_t X) {
  const uint32_t sl = key >> 2, cat = key & 3u;
  const int32_t id = sl == 0 ? unk : (int32_t)(sl - 1u);
  const int32_t f = cat < 2u ? id : (cat == 2u ? b : X);
  const int32_t g = cat == 0u ? a : (cat == 1u ? X : id);
  q[r] = ((u64)(int64_t)f << 32) | (u64)(int64_t)g;
  q[kFinMax + r] = (cat & 1u) ? sum : (u64)(-(int64_t)sum);
  q[2 * kFinMax + r] = ft;
}

// The merge's records (LDS hash slots, then the spilled keys) as (hk, delta, ft) in q[0, n).
__device__ __forceinline__ void fin_gather(const WlParams& p, DeltaH& h, LoopS& S, u64* q, int32_t a, int32_t b,
                                           int32_t X) {
  const uint32_t tid = threadIdx.x;
  for (int i = tid; i < kDh; i += kWlThreads) {
    const uint32_t key = h.key[i];
    if (key != kEmpty32) fin_record(q, atomicAdd(&S.nout, 1u), key, h.sum[i], h.ft[i], p.unk, a, b, X);
  }
  const uint32_t nsp = S.nspill;
  for (uint32_t i = tid; i < nsp; i += kWlThreads) {
    const uint32_t key = p.dlist[i];
    const u64 sum = atomicExch(&p.dsum[key], 0ull);
    const u64 ft = atomicExch(&p.dft[key], kEmpty64);
    fin_record(q, atomicAdd(&S.nout, 1u), key, sum, ft, p.unk, a, b, X);
  }
}

__device__ __forceinline__ u64 rl64(u64 x, uint32_t j) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)j);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), (int)j);
  return ((u64)hi << 32) | lo;
}

// finalize_changes for n <= 64 records, by one wave alone (no barrier, no LDS atomics): lane i
// holds record i; the combine and the ranks are scalar loops over the records (readlane
// broadcasts).  Same output as finalize_changes.  Returns the changes written.
__device__ uint32_t finalize_wave(const u64* q, const WlSlotDev& sd, int32_t a, int32_t b, uint32_t n) {
  const int lane = threadIdx.x & 63;
  const bool mine = (uint32_t)lane < n;
  const u64 hk = mine ? q[lane] : kFinEmpty;
  const u64 d = mine ? q[kFinMax + lane] : 0ull;
  const u64 ft = mine ? q[2 * kFinMax + lane] : kEmpty64;
  const u64 kab = ((u64)(int64_t)a << 32) | (u64)(int64_t)b;
  // records of one key: Σ delta, the min first touch leads
  u64 sum = 0;
  bool lead = mine && hk != kab;
#pragma unroll 1
  for (uint32_t j = 0; j < n; ++j) {
    const u64 hj = rl64(hk, j), fj = rl64(ft, j), dj = rl64(d, j);
    const bool same = hj == hk;
    sum += same ? dj : 0ull;
    lead = lead && !(same && fj < ft);
  }
  // place = leaders before this one: bucket ascending, then first touch descending
  const u64 lm = __ballot(lead);
  const uint32_t bk = (uint32_t)hk & (kDeltaBucketsDev - 1);
  uint32_t r = 0;
#pragma unroll 1
  for (u64 rest = lm; rest; rest &= rest - 1) {
    const uint32_t j = (uint32_t)__builtin_ctzll(rest);
    const uint32_t bj = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hk, (int)j) & (kDeltaBucketsDev - 1);
    const u64 fj = rl64(ft, j);
    r += (bj < bk || (bj == bk && fj > ft)) ? 1u : 0u;
  }
  if (lead) {
    u64* dst = reinterpret_cast<u64*>(sd.recs + r);
    dst[0] = hk;
    dst[1] = sum;
    dst[2] = ft;
  }
  return (uint32_t)__popcll(lm);
}

__device__ uint32_t finalize_changes(const WlParams& p, DeltaH& h, LoopS& S, u64* q, u64* tab, const WlSlotDev& sd,
                                     int32_t a, int32_t b, int32_t X, uint32_t n) {
  const uint32_t tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  u64* const fhk = q;
  u64* const fd = q + kFinMax;
  u64* const fft = q + 2 * kFinMax;
  u64* const mft = q + 3 * kFinMax;
  u64* const thk = tab;
  u64* const tft = tab + kFinTab;
  u64* const td = tab + 2 * kFinTab;
  uint32_t* const cnt = h.key;
  // 1. records -> (hk, delta, ft) in LDS; combine table cleared
  fin_gather(p, h, S, q, a, b, X);
  for (uint32_t i = tid; i < kFinTab; i += kWlThreads) {
    thk[i] = kFinEmpty;
    tft[i] = kEmpty64;
    td[i] = 0;
  }
  __syncthreads();
  // 2. combine per key: Σ delta and min first touch in the table
  constexpr int kPer = (int)(kFinMax / kWlThreads);
  uint32_t slot[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint32_t i = tid + (uint32_t)j * kWlThreads;
    slot[j] = 0;
    if (i < n) {
      const u64 hk = fhk[i];
      uint32_t t = (uint32_t)mix64(hk) & (kFinTab - 1);
#pragma unroll 1
      for (;;) {
        const u64 prev = atomicCAS(reinterpret_cast<unsigned long long*>(&thk[t]), kFinEmpty, hk);
        if (prev == kFinEmpty || prev == hk) break;
        t = (t + 1) & (kFinTab - 1);
      }
      slot[j] = t;
      atomicMin(reinterpret_cast<unsigned long long*>(&tft[t]), fft[i]);
      atomicAdd(reinterpret_cast<unsigned long long*>(&td[t]), fd[i]);
    }
  }
  for (uint32_t i = tid; i < kDeltaBucketsDev; i += kWlThreads) cnt[i] = 0;
  __syncthreads();
  // 3. a key's leader (its min first touch) takes a place in its bucket
  const u64 kab = ((u64)(int64_t)a << 32) | (u64)(int64_t)b;
  uint32_t li[kPer];
  bool lead[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint32_t i = tid + (uint32_t)j * kWlThreads;
    lead[j] = i < n && tft[slot[j]] == fft[i] && fhk[i] != kab;
    li[j] = lead[j] ? atomicAdd(&cnt[fhk[i] & (kDeltaBucketsDev - 1)], 1u) : 0u;
  }
  __syncthreads();
  // 4. bucket bases: exclusive scan of the 1024 counters, two a thread
  static_assert(kDeltaBucketsDev == 2 * kWlThreads, "two counters a thread");
  {
    const uint32_t c0 = cnt[2 * tid], c1 = cnt[2 * tid + 1];
    const uint32_t incl = wave_incl_add(c0 + c1);
    if (lane == 63) S.bs[wid] = incl;
    __syncthreads();
    uint32_t base = incl - c0 - c1, tot = 0;
    for (int w = 0; w < kWlThreads / 64; ++w) {
      if (w < wid) base += S.bs[w];
      tot += S.bs[w];
    }
    cnt[2 * tid] = base;
    cnt[2 * tid + 1] = base + c0;
    if (tid == 0) S.nfin = tot;
  }
  __syncthreads();
  // 5. each bucket's first touches side by side
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint32_t i = tid + (uint32_t)j * kWlThreads;
    if (lead[j]) mft[cnt[fhk[i] & (kDeltaBucketsDev - 1)] + li[j]] = fft[i];
  }
  __syncthreads();
  // 6. place = bucket base + the bucket's members with a later first touch
  const uint32_t m = S.nfin;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (!lead[j]) continue;
    const uint32_t i = tid + (uint32_t)j * kWlThreads;
    const uint32_t bk = (uint32_t)(fhk[i] & (kDeltaBucketsDev - 1));
    const uint32_t beg = cnt[bk], end = bk + 1 < kDeltaBucketsDev ? cnt[bk + 1] : m;
    const u64 ft = fft[i];
    uint32_t r = 0;
    for (uint32_t k = beg; k < end; ++k) r += mft[k] > ft ? 1u : 0u;
    u64* dst = reinterpret_cast<u64*>(sd.recs + beg + r);
    dst[0] = fhk[i];
    dst[1] = td[slot[j]];
    dst[2] = ft;
  }
  return m;
}

}  // namespace

// The merge loop (see the file comment).  One workgroup; command numbers start at p.seq0.
// kSelf (tiebreak=device): no host commands; the loop selects each merge from the device pair
// table's frontier (p.sel) and folds the merge's records back into the table.
// kProbes: the LDS delta hash's probe bound (kProbesDefault; 0 and 1 force the HBM spill path).
template <bool kSelf, int kProbes>
__global__ __launch_bounds__(kWlThreads) void k_word_loop(WlParams p) {
  __shared__ int32_t s_strip[kStrip * kWlThreads];  // [position][lane]: conflict-free per wave
  __shared__ DeltaH s_h;
  __shared__ LoopS S;
  constexpr int kBq = QueueShape<kSelf>::kBatch;
  constexpr int kQs = QueueShape<kSelf>::kCap;
  __shared__ u64 s_q[kQs];  // the listed entries that pass the filter, merged densely
  __shared__ SelLds<kSelf> s_f;
  __shared__ uint32_t s_kbits[kDh / 32];  // the merge's delta keys: a bit per hash slot in use
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t tid = threadIdx.x;
  int32_t* const mys = s_strip + tid;
  if (tid == 0) {
    S.pool_top = ld_agent(&p.dstate[kStPoolTop]);
    S.t_idle = 0;
    S.t_undo = 0;
    S.t_rel = 0;
    S.last_x = -1;
    S.last_lst = 0;
  }
  // The delta hash is clean between merges: cleared once here, then every merge clears what it
  // used once its records are out (the small-merge path only its own slots, by the key list)
  for (int i = tid; i < kDh; i += kWlThreads) {
    s_h.key[i] = kEmpty32;
    s_h.sum[i] = 0;
    s_h.ft[i] = kEmpty64;
  }
  if (tid < kDh / 32) s_kbits[tid] = 0;
  uint32_t expect = p.seq0;
  uint32_t exit_op = kOpStop;
  const MergeCtx mc{&S.nspill, &S.nkeys, s_kbits};
  // the small-merge path (p.fast, exact mode): the last wave writes the records and raises the flag;
  // it merges words only when a merge lists more than kWlThreads - 64 of them
  const bool fast = !kSelf && p.fast != 0 && (p.fin_max == 0 || p.fin_min != 0);
  constexpr int kFlagWave = kWlThreads / 64 - 1;
  // command prefetch (p.prefetch, exact mode): the poller wave (wave 1) reads the next command's
  // granules while the other waves write the current merge's records and its flag, so a command
  // the host already posted is in registers when the loop comes round (a poll is a PCIe round
  // trip, ≈ 1.6 µs, that late merges otherwise pay after every flag)
  const bool pfon = !kSelf && p.prefetch != 0;
  const int poll_wave = pfon ? 1 : 0;
  u64 pre_v = 0;
  bool pre_ok = false;
  // the merge's word-run and pool stores need not land before the records go out: nothing reads
  // them until the next command's barrier, which drains them; spilled deltas (read back by the
  // records phase) and K4 (which reads the merged words) still drain at the merge's end
  const bool drain = p.drain != 0 || p.fin_max != 0;
  if constexpr (kSelf) {  // the rebuilt frontier into LDS, indexed by pair key
    const SelParams& q = p.sel;
    const uint32_t nf = min(ld_agent(q.st + kSelNF), kSelK);
    for (uint32_t i = tid; i < kSelIdx / 2; i += kWlThreads) s_f.idx[i] = 0;
    for (uint32_t i = tid; i < nf; i += kWlThreads) {
      const uint32_t sl = ld_agent(q.fr[0] + i);
      s_f.key[i] = ld_agent64(q.tab + 2 * (u64)sl);
      s_f.cnt[i] = ld_agent64(q.tab + 2 * (u64)sl + 1) & kCntMask;
    }
    if (tid == 0) {
      s_f.n = nf;
      S.sm = ld_agent(q.st + kSelM);  // merges so far (kept in LDS from here on)
      S.scompact = 0;
      S.sins = ld_agent(q.st + kSelIns);  // the table's inserts so far (the host's and earlier launches')
      S.serr = 0;
      S.sover = 0;
      S.logn = 0;  // the host applied the previous launch's log
      S.lognew = 0;
      S.newtot = 0;
    }
    __syncthreads();
    for (uint32_t i = tid; i < nf; i += kWlThreads)
      if (!sel_idx_insert(s_f, s_f.key[i], i)) S.sover = 1;
  }
  __syncthreads();
  for (;;) {
    if constexpr (kSelf) {
      // ---- tiebreak=device: the best live frontier entry (count desc, key asc; at or above the
      // threshold) is the merge, by a scan of the LDS frontier
      const SelParams& q = p.sel;
      if (tid == 0) {
        S.snk = 0;
        S.status = 0;
        S.t_wait = __builtin_amdgcn_s_memrealtime();
      }
      __syncthreads();
      const uint32_t nf = min(s_f.n, kSelF);
      const u64 tc = q.thr[0], tk = q.thr[1];
      u64 bc = 0, bk = kEmpty64;
      uint32_t bs = kEmpty32, live = 0;
      {  // this thread's entries tid, tid + 256, ...: every load issued before the first compare
        constexpr int kPerF = (int)((kSelF + kWlThreads - 1) / kWlThreads);
        u64 fc[kPerF], fk[kPerF];
#pragma unroll
        for (int j = 0; j < kPerF; ++j) {
          const uint32_t i = (uint32_t)j * kWlThreads + (uint32_t)tid;
          fc[j] = i < nf ? s_f.cnt[i] : 0ull;
          fk[j] = i < nf ? s_f.key[i] : kEmpty64;
        }
#pragma unroll
        for (int j = 0; j < kPerF; ++j) {
          if (fk[j] != kEmpty64 && sel_at_least(fc[j], fk[j], tc, tk)) {
            ++live;
            if (sel_better(fc[j], fk[j], bc, bk)) {
              bc = fc[j];
              bk = fk[j];
              bs = (uint32_t)j * kWlThreads + (uint32_t)tid;
            }
          }
        }
      }
      if (__ballot(live != 0) && lane == 0) atomicAdd(&S.snk, 1u);
      {  // the wave's best (count desc, key asc): the max count, then the least key holding it
        const u64 wc = wave_max64(bc);
        const u64 wk = ~wave_max64(bc == wc ? ~bk : 0ull);
        const u64 who = __ballot(bc == wc && bk == wk);
        const int src = who ? (int)__builtin_ctzll(who) : 0;
        bs = (uint32_t)__builtin_amdgcn_readlane((int)bs, src);
        bc = wc;
        bk = wk;
      }
      if (lane == 0) {
        S.bc[wid] = bc;
        S.bk[wid] = bk;
        S.bs[wid] = bs;
      }
      __syncthreads();
      if (tid == 0) {
        for (int w = 1; w < kWlThreads / 64; ++w)
          if (sel_better(S.bc[w], S.bk[w], bc, bk)) {
            bc = S.bc[w];
            bk = S.bk[w];
            bs = S.bs[w];
          }
        const uint32_t m = S.sm;
        uint32_t status = 0;
        if (m >= q.n_max) status = kSelDone;
        else if (S.logn + 4ull * ((u64)p.cap + 2u) > q.log_cap) status = kSelRebuild;  // the log must be applied first
        // only pairs holding a new id are ever inserted: the table's fill is known without it
        // (a merge inserts at most 2 (cap + 1) pairs: (p, X) and (X, n) for every neighbour id)
        else if ((u64)S.sins + S.newtot + 2ull * ((u64)p.cap + 2u) > q.fill_max) status = kSelFull;
        else if (S.snk == 0) status = kSelRebuild;  // nothing at or above the threshold is left
        else if (bc < q.min_freq) status = kSelDone;
        S.cmd[0] = status ? kOpStop : kOpMerge;
        S.status = status;
        if (!status) {
          const int32_t a = (int32_t)(uint32_t)(bk >> 32), b = (int32_t)(uint32_t)bk;
          S.cmd[1] = (uint32_t)a;
          S.cmd[2] = (uint32_t)b;
          S.cmd[3] = (uint32_t)(q.X0 + (int32_t)m);
          S.cmd[4] = 0;
          S.cmd[5] = expect;
          S.cmd[6] = 0;  // no list given: the loop looks it up
          S.cmd[7] = 0;
          S.sel_pos = bs;
          S.sel_cnt = bc;
          q.out[2 * (u64)m] = bk;
          q.out[2 * (u64)m + 1] = bc;
        }
      }
    } else if (wid == poll_wave) {
      // ---- the poller wave waits for the next command (one round trip reads all four granules;
      // none when the prefetched granules already carry it)
      const u64* g = p.ring[expect % kRing].g;
      const u64 t_wait = __builtin_amdgcn_s_memrealtime();
      uint32_t op = 0, a = 0, b = 0, X = 0, idle = 0;
      u64 v = pre_ok ? pre_v
                     : (lane < kCmdGranules ? __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull);
      pre_ok = false;
      uint32_t loff = 0, lcnt1 = 0;
      for (;;) {
        const bool tagged = lane >= kCmdGranules || (uint32_t)v == expect;
        if (__all(tagged)) {
          WL_ST(if (lane == 0) S.t_seen = __builtin_amdgcn_s_memrealtime();)
          const uint32_t val = (uint32_t)(v >> 32);
          op = __shfl(val, 0, 64);
          a = __shfl(val, 1, 64);
          b = __shfl(val, 2, 64);
          X = __shfl(val, 3, 64);
          loff = __shfl(val, 4, 64);
          lcnt1 = __shfl(val, 5, 64);
          break;
        }
        if (++idle >= p.idle_polls) {
          op = kOpTimeout;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = lane < kCmdGranules ? __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
      }
      if (lane == 0) {
        S.cmd[0] = op & 0xFFu;
        S.cmd[1] = a;
        S.cmd[2] = b;
        S.cmd[3] = X;
        S.cmd[4] = (op >> 8) & 0xFFu;  // slot
        S.cmd[5] = expect;
        S.cmd[6] = lcnt1;
        S.cmd[7] = loff;
        S.t_wait = t_wait;
      }
    }
    __syncthreads();
    const uint32_t op = S.cmd[0];
    const int32_t a = (int32_t)S.cmd[1], b = (int32_t)S.cmd[2], X = (int32_t)S.cmd[3];
    const uint32_t slot = S.cmd[4], seq = S.cmd[5];
    ++expect;
    if (op != kOpMerge && op != kOpUnmerge) {
      exit_op = kSelf ? S.status : op;
      break;
    }
    // ---- the word list.  Merge (a, b), M = max(a, b): when the loop created M, M's words-of
    // list with the filter bit of the pair's other id on its side ((c, M): c on the left, (M, d):
    // d on the right, (M, M): M on the left); else the initial directory entry of (a, b) (every
    // word that held the pair when the index was built, exact).  Undo: the words of X, exactly.
    // Wave 0 reads the id tables and 16 directory slots in one round trip.
    const u64 t_cmd = __builtin_amdgcn_s_memrealtime();
    WL_ST(const u64 c_cmd = __builtin_amdgcn_s_memtime();)
    if (wid == 0) {
      const bool undo = op == kOpUnmerge;
      const int32_t M = undo ? X : (a > b ? a : b);
      // the host sent M's words-of list, or M is the loop's last merge (its list in LDS): no lookup
      const bool recent = !undo && M == S.last_x;
      const uint32_t given = undo ? 0u : (S.cmd[6] ? S.cmd[6] : recent ? (uint32_t)(S.last_lst >> 32) + 1u : 0u);
      const uint32_t goff = S.cmd[6] ? S.cmd[7] : (uint32_t)S.last_lst;
      u64 lv64 = 0;
      bool lv = false;
      if (!given && (lane == 16 || lane == 17) && M >= 0 && (uint32_t)M < p.id_cap) {
        if (lane == 16) lv = p.lseq[M] != kNoList;
        if (lane == 17) lv64 = p.lst[M];
      }
      const u64 key = pair_key(a, b);
      const u64 h = mix64(key) & p.dir_mask;
      u64 dk = kEmpty64, dv = 0;
      if (!given && !undo && lane < 16) {
        dk = p.dkey[(h + (u64)lane) & p.dir_mask];
        dv = p.dval[(h + (u64)lane) & p.dir_mask];
      }
      const bool has_list = given || ((__ballot(lv) >> 16) & 1ull);
      const u64 wl = given ? ((u64)goff | ((u64)(given - 1u) << 32)) : __shfl(lv64, 17, 64);
      u64 off = 0, cnt = 0, need = 0;
      bool err = false;
      if (has_list) {
        off = (uint32_t)wl;
        cnt = wl >> 32;
        if (!undo) need = a == b ? nbit(M, 0) : b == M ? nbit(a, 0) : nbit(b, 1);
      } else if (undo) {
        err = true;  // every merged id has its words-of list
      } else {
        for (u64 base = 0;; base += 16) {
          if (base) {
            dk = kEmpty64;
            if (lane < 16) {
              dk = p.dkey[(h + base + (u64)lane) & p.dir_mask];
              dv = p.dval[(h + base + (u64)lane) & p.dir_mask];
            }
          }
          const u64 hit = __ballot(lane < 16 && dk == key);
          const u64 emp = __ballot(lane < 16 && dk == kEmpty64);
          const u64 any = hit | emp;
          if (any) {
            const int f = __ffsll((long long)any) - 1;
            const u64 vf = __shfl(dv, f, 64);
            if ((hit >> f) & 1ull) {
              off = (uint32_t)vf;
              cnt = vf >> 32;
            } else {
              err = true;  // a selected pair always has a list
            }
            break;
          }
          if (base > p.dir_mask) {
            err = true;
            break;
          }
        }
      }
      if (lane == 0) {
        S.lk[0] = off;
        S.lk[1] = err ? 0 : cnt;
        S.need = need;
        S.nout = 0;
        S.nchg = 0;
        S.scan = 0;
        S.rd = 0;
        S.wr = 0;
        S.nspill = 0;
        S.nkeys = 0;
        S.filter = need != 0;
        S.occ = 0;
        S.err = 0;
        S.st[0] = S.st[1] = S.st[2] = S.st[3] = 0;
        WL_ST(for (int i = 0; i < kXs; ++i) S.xs[i] = 0; S.xs[8] = given ? 1u : 0u;)
        if (err) atomicMax(&p.dstate[kStError], undo ? kErrList : kErrLookup);
        if (!undo && (u64)S.pool_top + cnt > p.pool_cap) {
          S.err = 1;
          atomicMax(&p.dstate[kStError], kErrPool);
        }
        S.t[0] = __builtin_amdgcn_s_memrealtime() - t_cmd;
      }
    }
    __syncthreads();
    WL_ST(if (tid == 0) S.xs[0] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd);)
    const u64 off = S.lk[0], cnt = S.lk[1];
    const uint32_t top = S.pool_top;
    if (op == kOpUnmerge) {
      for (u64 i = tid; i < cnt; i += kWlThreads) {
        const u64 e = p.pool[off + i].e;
        int32_t* r = p.wtok + (uint32_t)(e >> 32);
        const uint32_t L = (uint32_t)r[0];
        const uint32_t nl = unmerge_run(r + kRunHdr, L, a, b, X);
        if (nl != L) r[0] = (int32_t)nl;
      }
      __syncthreads();
      if (tid == 0 && X >= 0 && (uint32_t)X < p.id_cap) {
        if (off + cnt == (u64)S.pool_top) S.pool_top = (uint32_t)off;  // the guess's list was the last one
        p.lseq[X] = kNoList;
        if (S.last_x == X) S.last_x = -1;
      }
      if (tid == 0) {
        S.t_idle += t_cmd - S.t_wait;
        S.t_undo += __builtin_amdgcn_s_memrealtime() - t_cmd;
      }
      __syncthreads();
      continue;
    }
    const bool append = S.err == 0;
    const u64 need = S.need;
    if ((fast || (kSelf && p.fast != 0)) && op == kOpMerge && cnt <= (u64)kWlThreads) {
      // ---- the small-merge path (every late merge: a few hundred listed words, tens changed).  A
      // lane per listed entry, no queue and no barrier before the merge: entry tid's filter decides
      // and a passing lane loads its word's run and weight right away (the only hop after the
      // entry), merges it in registers (merge_regs) and stores it back.  The delta keys are listed
      // as they enter the LDS hash, so the records phase reads (and clears) only those.  The last
      // wave writes the records and raises the flag: it issued no word stores (unless more than
      // kWlThreads - 64 words are listed), so its drain and release wait for the records alone --
      // the other waves' word-run and pool stores drain at the next command's barrier (the rule
      // at WlParams::drain; with drain = 1 they drain here).  tiebreak=device (kSelf) merges the
      // same way and then takes the common tail below (pair table + frontier, no host records).
      u64 e = kEmpty64;
      bool pass = false;
      if (tid < cnt) {
        const WEnt v = p.pool[off + tid];
        e = v.e;
        pass = (v.sig & need) == need;
      }
      WL_ST(if (pass) wl_stamp(S.xs, 2, t_cmd);)
      uint32_t occ = 0, L = 0, nl = 0;
      u64 nsig = 0;
      if (pass) {
        int32_t* r = p.wtok + (uint32_t)(e >> 32);
        const Run x = load_run(r, ent_groups(e));
        const u64 wc = run_weight(x);
        L = (uint32_t)x.v[0].x;
        nl = L;
        WL_ST(wl_stamp(S.xs, 3, t_cmd);)
        if (L >= 2) {
          if (L <= kStripTok) {
            occ = merge_regs<kProbes>(p, s_h, mc, mys, r, x, L, e, wc, a, b, X, &nl, &nsig
                                      WL_ST(, S.xs, t_cmd));
          } else {
            occ = merge_run<kProbes>(p, s_h, mc, r + kRunHdr, L, e, wc, a, b, X, &nl, &nsig);
            if (occ) r[0] = (int32_t)nl;
          }
        }
      }
      const u64 chg = __ballot(occ != 0);
      if (chg) {  // the changed words become the words of X
        const int lead = __ffsll((long long)chg) - 1;
        uint32_t nb = 0;
        if (lane == lead) nb = atomicAdd(&S.nchg, (uint32_t)__popcll(chg));
        nb = __shfl(nb, lead, 64);
        if (occ && append) {
          WEnt ne;
          ne.e = e;
          ne.sig = nsig;
          st16(&p.pool[(u64)top + nb + (uint32_t)__popcll(chg & ((1ull << lane) - 1ull))],
               make_int4((int)(uint32_t)ne.e, (int)(uint32_t)(ne.e >> 32), (int)(uint32_t)ne.sig, (int)(uint32_t)(ne.sig >> 32)));
        }
      }
      if (const u64 sm = __ballot(pass)) {  // statistics: wave sums, one LDS add each per wave
        const uint32_t w_occ = wave_sum32(occ), w_rd = wave_sum32(pass ? 1u + L : 0u);
        const uint32_t w_wr = wave_sum32(occ ? 1u + nl : 0u);
        if (lane == 0) {
          atomicAdd(&S.occ, (u64)w_occ);
          atomicAdd(&S.scan, (uint32_t)__popcll(sm));
          atomicAdd(&S.rd, w_rd);
          atomicAdd(&S.wr, w_wr);
        }
      }
      WL_ST(wl_stamp(S.xs, 7, t_cmd);)
      // read before the barrier: past it the poller wave may already be waiting for the next command
      // (it writes S.t_wait there); the flag wave has not written the header yet
      const u64 t_wait = S.t_wait;
      WL_ST(const u64 t_seen_m = S.t_seen;)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every delta is in the hash
      // spilled deltas' HBM atomics complete (S.nspill is final); K4 never runs here, so only the
      // drain option itself drains
      if (p.drain != 0 || S.nspill) __syncthreads();
      WL_ST(wl_stamp(S.xs, 9, t_cmd);)
      if constexpr (!kSelf) {
        const uint32_t nchg = append ? S.nchg : 0u;
        if (wid == 0 && lane == 0 && X >= 0 && (uint32_t)X < p.id_cap) {
          p.lst[X] = (u64)top | ((u64)nchg << 32);
          p.lseq[X] = seq;
        }
        if (wid == kFlagWave) {
          const WlSlotDev& sd = p.sl[slot & (WordLoop::kSlots - 1)];
          const u64 t_out = __builtin_amdgcn_s_memrealtime();
          WL_ST(if (lane == 0) S.xs[12] = (uint32_t)(t_out - t_cmd);)
          // the records: lane l takes the slots of bitmap word l (32 slots), placed by a wave scan
          // of the words' popcounts; the slots are cleared as they are read
          const uint32_t nsp = S.nspill;
          uint32_t bw = s_kbits[lane];
          s_kbits[lane] = 0;
          const uint32_t nb = (uint32_t)__popc(bw);
          const uint32_t incl = wave_scan32(nb);
          const uint32_t nk = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
          uint32_t ri = incl - nb;
          WL_ST(if (lane == 0) S.xs[13] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd);)
          u64 cks = 0;  // this lane's share of the hand-off checksum
          for (; bw; bw &= bw - 1u, ++ri) {
            const uint32_t h = (uint32_t)lane * 32u + (uint32_t)__builtin_ctz(bw);
            u64* dst = reinterpret_cast<u64*>(sd.recs + ri);
            const u64 w0 = (u64)s_h.key[h], w1 = s_h.sum[h], w2 = s_h.ft[h];
            dst[0] = w0;
            dst[1] = w1;
            dst[2] = w2;
            cks += w0 * hand_weight(16u + 3u * ri) + w1 * hand_weight(17u + 3u * ri) + w2 * hand_weight(18u + 3u * ri);
            s_h.key[h] = kEmpty32;
            s_h.sum[h] = 0;
            s_h.ft[h] = kEmpty64;
          }
          WL_ST(if (lane == 0) S.xs[14] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd);)
          for (uint32_t i = (uint32_t)lane; i < nsp; i += 64u) {  // then the keys spilled to HBM
            const uint32_t key = p.dlist[i];
            const u64 sum = atomicExch(&p.dsum[key], 0ull);
            const u64 ft = atomicExch(&p.dft[key], kEmpty64);
            u64* dst = reinterpret_cast<u64*>(sd.recs + nk + i);
            dst[0] = (u64)key;
            dst[1] = sum;
            dst[2] = ft;
            const uint32_t r = nk + i;
            cks += (u64)key * hand_weight(16u + 3u * r) + sum * hand_weight(17u + 3u * r) + ft * hand_weight(18u + 3u * r);
          }
          WL_ST(if (lane == 0) S.xs[10] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd);)
          if (lane == 0) {
            S.lst_x = 0;
            S.last_x = -1;
            if (X >= 0 && (uint32_t)X < p.id_cap) {
              S.pool_top = top + nchg;
              S.lst_x = (u64)top | ((u64)(nchg + 1u) << 32);  // for the host: offset, count + 1
              S.last_x = X;
              S.last_lst = (u64)top | ((u64)nchg << 32);
            }
            // the header, staged in LDS and written by 8 lanes with one 16-B store each
            uint32_t* hs = S.hs;
            u64* hs64 = reinterpret_cast<u64*>(hs);
            const u64 now = __builtin_amdgcn_s_memrealtime();
            hs[0] = nk + nsp;
            hs[1] = 0u;  // (the flag word: the ordered paths' flag; this path's are the checksum granules)
            hs[2] = (uint32_t)cnt;
            hs[3] = S.nchg;
            hs64[2] = S.occ;
            hs64[3] = now - t_cmd;
            hs64[4] = S.t[0];
            hs64[5] = t_out - t_cmd;
            hs[12] = S.scan;
            hs[13] = S.filter;
            hs[14] = S.rd;
            hs[15] = S.wr;
            hs[16] = hs[17] = hs[18] = 0u;  // (the queued path's stamps)
            hs[19] = nsp;
            hs[20] = (uint32_t)(S.t_idle + (t_cmd - t_wait));
            hs[21] = (uint32_t)S.t_undo;
            hs[22] = 0u;
            hs[23] = nk + nsp;
            hs64[12] = S.lst_x;
            hs64[13] = t_cmd;
            hs64[14] = t_wait;
            hs[30] = (uint32_t)(now - t_out);
            hs[31] = S.t_rel;
            S.t_idle = 0;
            S.t_undo = 0;
          }
          if (lane < 8) {
            const int4 hv = reinterpret_cast<const int4*>(S.hs)[lane];
            reinterpret_cast<int4*>(sd.hdr)[lane] = hv;
            const u64 lo = (u64)(uint32_t)hv.x | ((u64)(uint32_t)hv.y << 32), hi = (u64)(uint32_t)hv.z | ((u64)(uint32_t)hv.w << 32);
            cks += lo * hand_weight(2u * lane) + hi * hand_weight(2u * lane + 1u);
          }
          {  // the wave's sum (DPP row shifts and broadcasts, lane 63), then the tagged granules
            cks += wl_dpp64<0x111>(cks);
            cks += wl_dpp64<0x112>(cks);
            cks += wl_dpp64<0x114>(cks);
            cks += wl_dpp64<0x118>(cks);
            cks += wl_dpp64<0x142, 0xa, false>(cks);
            cks += wl_dpp64<0x143, 0xc, false>(cks);
            cks = rl64(cks, 63);
          }
          if (lane == 0) {
            const u64 t_r0 = __builtin_amdgcn_s_memrealtime();
            // stamps build: [1] the shader clock (MHz) over the merge, [9] cycles of one s_memrealtime
            WL_ST(sd.hdr[48] = (uint32_t)t_seen_m;
                const u64 c_now = __builtin_amdgcn_s_memtime(); const u64 t_now = __builtin_amdgcn_s_memrealtime();
                  S.xs[1] = (uint32_t)((c_now - c_cmd) * 100ull / (t_now - t_cmd + 1ull));
                  S.xs[11] = (uint32_t)(t_r0 - t_cmd); for (int i = 0; i < kXs; ++i) sd.hdr[32 + i] = S.xs[i];)
            // the checksum granules right behind the records and the header (no drain between), then
            // one system-scope release fence: the L2 write-back that sends them all out promptly
            u64* h64w = reinterpret_cast<u64*>(sd.hdr);
            h64w[kCksWord] = ((u64)seq << 32) | (cks & 0xFFFFFFFFull);
            h64w[kCksWord + 1] = ((u64)seq << 32) | (cks >> 32);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            S.t_rel = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_r0);
          }
        } else if (pfon && wid == poll_wave) {  // the next command's granules, in flight meanwhile
          pre_v = lane < kCmdGranules
                      ? __hip_atomic_load(p.ring[expect % kRing].g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                      : 0ull;
          pre_ok = true;
        }
        continue;  // (the next command's barrier orders the flag wave's LDS writes before any use)
      }
    } else {
    // ---- the merge over the listed words; changed words become the words of X.  Each round a
    // lane loads kB pool entries (coalesced) and queues in LDS those whose filter holds the
    // pair's bit; once a workgroup's worth is queued (and at the end) the queue is merged
    // densely, a lane per word: the run in one round trip, the walk in registers.
    uint32_t my_occ = 0, my_scan = 0, my_rd = 0, my_wr = 0;
    if (tid == 0) S.qn = 0;
    for (u64 base = 0; base < cnt; base += (u64)kWlThreads * kBq) {
      u64 ex[kBq], sx[kBq];
#pragma unroll
      for (int q = 0; q < kBq; ++q) {
        const u64 i = base + (u64)q * kWlThreads + tid;
        ex[q] = kEmpty64;
        sx[q] = 0;
        if (i < cnt) {
          const WEnt v = p.pool[off + i];
          ex[q] = v.e;
          sx[q] = v.sig;
        }
      }
      if (base == 0 && tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        S.st[0] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd);
      }
#pragma unroll
      for (int q = 0; q < kBq; ++q) {
        const bool pass = ex[q] != kEmpty64 && (sx[q] & need) == need;
        const u64 bl = __ballot(pass);
        if (bl) {
          const int lead = __ffsll((long long)bl) - 1;
          uint32_t qb = 0;
          if (lane == lead) qb = atomicAdd(&S.qn, (uint32_t)__popcll(bl));
          qb = __shfl(qb, lead, 64);
          if (pass) s_q[qb + (uint32_t)__popcll(bl & ((1ull << lane) - 1ull))] = ex[q];
        }
      }
      __syncthreads();
      const uint32_t qn = S.qn;
      __syncthreads();  // every thread has read qn before the next round queues more
      const bool last = base + (u64)kWlThreads * kBq >= cnt;
      if (qn < (uint32_t)kWlThreads && !last) continue;
      WL_ST(if (tid == 0) { if (!S.xs[1]) S.xs[1] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd); ++S.xs[9]; })
      // A lane's words one after another, the next word's run and weight loading while this one
      // merges (the compiler's waits count the loads; big merges queue up to 9 words a lane)
      const uint32_t qend = ((qn + kWlThreads - 1) / kWlThreads) * kWlThreads;
      u64 e_n = kEmpty64;
      Run x_n{};
      if (kWlPrefetch && tid < qn) {
        e_n = s_q[tid];
        x_n = load_run(p.wtok + (uint32_t)(e_n >> 32), ent_groups(e_n));
      }
      for (uint32_t qi = tid; qi < qend; qi += kWlThreads) {
        if (!kWlPrefetch && qi < qn) {
          e_n = s_q[qi];
          x_n = load_run(p.wtok + (uint32_t)(e_n >> 32), ent_groups(e_n));
        }
        const u64 e = e_n;
        const Run x = x_n;
        const u64 wc = run_weight(x);
        if (kWlPrefetch && qi + kWlThreads < qn) {
          e_n = s_q[qi + kWlThreads];
          x_n = load_run(p.wtok + (uint32_t)(e_n >> 32), ent_groups(e_n));
        }
        uint32_t occ = 0;
        u64 nsig = 0;
        if (qi < qn) {
          int32_t* r = p.wtok + (uint32_t)(e >> 32);
          const uint32_t L = (uint32_t)x.v[0].x;
          uint32_t nl = L;
          WL_ST(atomicMax(&S.xs[2], (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd)); atomicMax(&S.xs[6], L);
                if (L > kStripTok) atomicAdd(&S.xs[5], 1u);)
          if (qi == 0 && base == 0) S.st[1] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd);
          ++my_scan;
          if (L >= 2) {
            if (L <= kStripTok) {
              occ = merge_regs<kProbes>(p, s_h, mc, mys, r, x, L, e, wc, a, b, X, &nl, &nsig);
            } else {
              occ = merge_run<kProbes>(p, s_h, mc, r + kRunHdr, L, e, wc, a, b, X, &nl, &nsig);
              if (occ) r[0] = (int32_t)nl;
            }
          }
          WL_ST(atomicMax(&S.xs[3], (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd)); atomicMax(&S.xs[7], occ);)
          my_occ += occ;
          my_rd += 1u + L;
          my_wr += occ ? 1u + nl : 0u;
          if (qi == 0 && base == 0) S.st[2] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd);
        }
        const u64 chg = __ballot(occ != 0);
        if (chg) {
          const int lead = __ffsll((long long)chg) - 1;
          uint32_t nb = 0;
          if (lane == lead) nb = atomicAdd(&S.nchg, (uint32_t)__popcll(chg));
          nb = __shfl(nb, lead, 64);
          if (occ && append) {
            const uint32_t rk = (uint32_t)__popcll(chg & ((1ull << lane) - 1ull));
            WEnt ne;
            ne.e = e;
            ne.sig = nsig;
            p.pool[(u64)top + nb + rk] = ne;
          }
        }
      }
      if (drain) __syncthreads();
      else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (tid == 0) S.qn = 0;
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    {  // statistics: wave sums, one LDS add each per wave
      const uint32_t w_occ = wave_sum32(my_occ), w_scan = wave_sum32(my_scan);
      const uint32_t w_rd = wave_sum32(my_rd), w_wr = wave_sum32(my_wr);
      if (lane == 0 && w_scan) {
        atomicAdd(&S.occ, (u64)w_occ);
        atomicAdd(&S.scan, w_scan);
        atomicAdd(&S.rd, w_rd);
        atomicAdd(&S.wr, w_wr);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (drain || S.nspill) __syncthreads();  // (uniform: S.nspill is final after the barrier above)
    WL_ST(if (tid == 0) S.xs[4] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd);)
    }
    const uint32_t nchg = append ? S.nchg : 0u;
    if (tid < kDh / 32) s_kbits[tid] = 0;  // (this path reads the whole hash; the next barrier orders it)
    if constexpr (kSelf) {
      // ---- tiebreak=device: the records change the pair table (atomics nobody waits for) and,
      // through the frontier's LDS index, the frontier's counts; the pairs this merge created that
      // rank at or above the threshold join the frontier -- their counts come from the records
      // (they were 0 before), so nothing is read back from the table
      const SelParams& q = p.sel;
      const u64 t_tab = __builtin_amdgcn_s_memrealtime();
      if (tid == 0) {
        S.last_x = -1;
        if (X >= 0 && (uint32_t)X < p.id_cap) {
          p.lst[X] = (u64)top | ((u64)nchg << 32);
          p.lseq[X] = seq;
          S.pool_top = top + nchg;
          S.last_x = X;
          S.last_lst = (u64)top | ((u64)nchg << 32);
        }
        S.snew = 0;
        S.dxa = 0;
      }
      __syncthreads();
      constexpr uint32_t kNewCap = (uint32_t)kQs / 2;  // the new pairs' list in the merge queue's LDS (free now)
      const SelNew nw{s_q, s_q + kNewCap, &S.snew, kNewCap, &S.dxa, &S.sover, q.log + 2 * S.logn, &S.lognew};
      for (int i = tid; i < kDh; i += kWlThreads) {
        const uint32_t key = s_h.key[i];
        if (key != kEmpty32) {
          sel_record(q, s_f, nw, p.unk, key, s_h.sum[i], a, b, X);
          s_h.key[i] = kEmpty32;  // the hash is clean between merges
          s_h.sum[i] = 0;
          s_h.ft[i] = kEmpty64;
        }
      }
      const uint32_t nsp = S.nspill;
      for (uint32_t i = tid; i < nsp; i += kWlThreads) {
        const uint32_t key = p.dlist[i];
        const u64 sum = atomicExch(&p.dsum[key], 0ull);
        atomicExch(&p.dft[key], kEmpty64);
        sel_record(q, s_f, nw, p.unk, key, sum, a, b, X);
      }
      // LDS results only: the table's atomics stay in flight (a plain __syncthreads would drain them)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (tid == 0) S.t_rec = __builtin_amdgcn_s_memrealtime();
      if (tid == 0) {  // the merged pair: count 0 (it never occurs again); in the table by its LDS
        s_f.cnt[S.sel_pos] = 0;  // count's opposite, so the log's adds need no order
        u64* lg = q.log + 2 * (S.logn + S.lognew);
        lg[0] = pair_key(a, b);
        lg[1] = (u64)(-(int64_t)S.sel_cnt);
        S.logn += S.lognew + 1u;
        S.lognew = 0;
        S.newtot += S.snew;
      }
      const u64 tc = q.thr[0], tk = q.thr[1];
      const uint32_t nnew = min(S.snew, kNewCap);
      const u64 kxa = pair_key(X, a), dxa = S.dxa;
      for (uint32_t i = tid; i < nnew; i += kWlThreads) {
        const u64 k = nw.key[i];
        const u64 c = nw.cnt[i] + (k == kxa ? dxa : 0ull);
        if (sel_at_least(c, k, tc, tk)) {
          const uint32_t pos = atomicAdd(&s_f.n, 1u);
          if (pos < kSelF) {
            s_f.key[pos] = k;
            s_f.cnt[pos] = c;
            if (!sel_idx_insert(s_f, k, pos)) S.sover = 1;
          } else {
            S.sover = 1;  // the frontier lost an entry: rebuild
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (tid == 0) S.t_app = __builtin_amdgcn_s_memrealtime();
      // past kSelF - kSelRoom entries: the dead ones go (in place, order kept) and the index is
      // rebuilt for the new positions
      if (!S.sover && s_f.n > kSelF - kSelSlack) {
        constexpr int kPer = (int)((kSelF + kWlThreads - 1) / kWlThreads);
        const uint32_t n0 = s_f.n;
        u64 ck[kPer], kk[kPer];
        uint32_t mine = 0, keepm = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {  // thread t holds entries kPer*t .. kPer*t + kPer-1
          const uint32_t i = (uint32_t)kPer * tid + (uint32_t)j;
          ck[j] = 0;
          kk[j] = kEmpty64;
          if (i < n0) {
            ck[j] = s_f.cnt[i];
            kk[j] = s_f.key[i];
            if (kk[j] != kEmpty64 && sel_at_least(ck[j], kk[j], tc, tk)) {
              keepm |= 1u << j;
              ++mine;
            }
          }
        }
        const uint32_t incl = wave_incl_add(mine);
        if (lane == 63) S.bs[wid] = incl;  // wave totals
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint32_t base = incl - mine;
        for (int w = 0; w < wid; ++w) base += S.bs[w];
        uint32_t tot = 0;
        for (int w = 0; w < kWlThreads / 64; ++w) tot += S.bs[w];
        for (uint32_t i = tid; i < kSelIdx / 2; i += kWlThreads) s_f.idx[i] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every entry is in registers before any is moved
        const uint32_t b0 = base;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const uint32_t i = (uint32_t)kPer * tid + (uint32_t)j;
          if (i >= n0 || !((keepm >> j) & 1u)) continue;
          s_f.cnt[base] = ck[j];
          s_f.key[base] = kk[j];
          ++base;
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        for (uint32_t i = b0; i < base; ++i)
          if (!sel_idx_insert(s_f, s_f.key[i], i)) S.sover = 1;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (tid == 0) {
          s_f.n = tot;
          ++S.scompact;
          if (tot > kSelF - kSelRoom) S.sover = 1;  // mostly live: a rebuild, not a compaction per merge
        }
      }
      if (tid == 0) {
        q.st[kSelNF] = min(s_f.n, kSelF);
        q.st[kSelM] = S.sm + 1u;
        ++S.sm;  // the merge count stays in LDS for the launch (this loop is its only writer)
        // statistics (st words 6..): select ticks, merge ticks (u64 each), listed / changed words,
        // occurrences (u64), new pairs
        u64* t64 = reinterpret_cast<u64*>(q.st + kSelStats);
        const u64 now = __builtin_amdgcn_s_memrealtime();
        t64[0] += t_cmd - S.t_wait;
        t64[1] += now - t_cmd;
        t64[2] += cnt;
        t64[3] += nchg;
        t64[4] += S.occ;
        t64[5] += nnew;
        t64[6] += now - t_tab;  // of t64[1]: the table and frontier update
        t64[7] += S.scompact ? 1u : 0u;
        t64[8] += S.t_rec - t_tab;    // records -> table + frontier counts + new-pair list
        t64[9] += S.t_app - S.t_rec;  // merged pair, new pairs appended
        t64[10] += now - S.t_app;     // compaction (when due), bookkeeping
        q.st[kSelBuf] = S.scompact;  // (statistic: LDS compactions of this launch)
        // after a complete merge: a frontier that lost an entry needs a rebuild, a table past its
        // fill bound must grow (the host stops)
        S.status = S.sover ? kSelRebuild : 0u;  // (the table's fill is checked when its log is applied)
      }
      __syncthreads();
      if (S.status) {
        exit_op = S.status;
        break;
      }
      continue;
    }
    // ---- the records to host memory (LDS hash, then the spilled keys), then the flag
    const WlSlotDev& sd = p.sl[slot & (WordLoop::kSlots - 1)];
    if (tid == 0) {
      S.t[1] = __builtin_amdgcn_s_memrealtime() - t_cmd;
      S.lst_x = 0;
      if (X >= 0 && (uint32_t)X < p.id_cap) {
        p.lst[X] = (u64)top | ((u64)nchg << 32);
        p.lseq[X] = seq;
        S.pool_top = top + nchg;
        S.lst_x = (u64)top | ((u64)(nchg + 1u) << 32);  // for the host: offset, count + 1
      }
      S.last_x = S.lst_x ? X : -1;
      S.last_lst = (u64)top | ((u64)nchg << 32);
    }
    const uint32_t nrec = S.nkeys + S.nspill;
    const bool fin = p.fin_max != 0 && nrec <= p.fin_max && nrec <= kFinMax && nrec >= p.fin_min;
    const u64 t_fin = __builtin_amdgcn_s_memrealtime();
    if (fin && nrec <= 64u) {  // one wave combines and orders them
      fin_gather(p, s_h, S, s_q, a, b, X);
      __syncthreads();
      if (wid == 0) {
        const uint32_t m = finalize_wave(s_q, sd, a, b, nrec);
        if (lane == 0) S.nfin = m;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (fin) {
      finalize_changes(p, s_h, S, s_q, reinterpret_cast<u64*>(s_strip), sd, a, b, X, nrec);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (pfon && wid == 1) {
      // the poller wave: the next command's granules, in flight while the others write records
      pre_v = lane < kCmdGranules
                  ? __hip_atomic_load(p.ring[expect % kRing].g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                  : 0ull;
      pre_ok = true;
    } else {
      // every wave but the poller (with the prefetch on) writes the records
      const uint32_t rt = pfon ? (tid < 64u ? tid : tid - 64u) : tid;
      const uint32_t rs = pfon ? (uint32_t)kWlThreads - 64u : (uint32_t)kWlThreads;
      for (uint32_t i = rt; i < (uint32_t)kDh; i += rs) {
        const uint32_t key = s_h.key[i];
        if (key == kEmpty32) continue;
        const uint32_t r = atomicAdd(&S.nout, 1u);
        u64* dst = reinterpret_cast<u64*>(sd.recs + r);
        dst[0] = (u64)key;
        dst[1] = s_h.sum[i];
        dst[2] = s_h.ft[i];
        s_h.key[i] = kEmpty32;  // the hash is clean between merges
        s_h.sum[i] = 0;
        s_h.ft[i] = kEmpty64;
      }
      const uint32_t nsp = S.nspill;  // complete: every delta was added before the barrier above
      for (uint32_t i = rt; i < nsp; i += rs) {
        const uint32_t key = p.dlist[i];
        const u64 sum = atomicExch(&p.dsum[key], 0ull);
        const u64 ft = atomicExch(&p.dft[key], kEmpty64);
        const uint32_t r = atomicAdd(&S.nout, 1u);
        u64* dst = reinterpret_cast<u64*>(sd.recs + r);
        dst[0] = (u64)key;
        dst[1] = sum;
        dst[2] = ft;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // LDS only: the poller's prefetch stays in flight (every other wave drained its stores above)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    WL_ST(if (tid == 0) S.xs[10] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cmd);)
    if (fin)  // K4 used the hash keys as bucket counters: clean it whole (ordered by the next barrier)
      for (int i = tid; i < kDh; i += kWlThreads) {
        s_h.key[i] = kEmpty32;
        s_h.sum[i] = 0;
        s_h.ft[i] = kEmpty64;
      }
    if (tid == 0) {
      sd.hdr[0] = fin ? S.nfin : S.nout;
      sd.hdr[22] = fin ? 1u : 0u;  // 1: ordered changes (finalize_changes), else raw records
      sd.hdr[23] = nrec;
      sd.hdr[30] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_fin);  // records out: gather (+ finalize)
      sd.hdr[2] = (uint32_t)cnt;
      sd.hdr[3] = S.nchg;
      u64* h64 = reinterpret_cast<u64*>(sd.hdr);
      h64[2] = S.occ;
      h64[3] = (u64)__builtin_amdgcn_s_memrealtime() - t_cmd;
      h64[4] = S.t[0];
      h64[5] = S.t[1];
      sd.hdr[12] = S.scan;
      sd.hdr[13] = S.filter;
      sd.hdr[14] = S.rd;
      sd.hdr[15] = S.wr;
      sd.hdr[16] = S.st[0];
      sd.hdr[17] = S.st[1];
      sd.hdr[18] = S.st[2];
      sd.hdr[19] = S.nspill;  // delta keys that spilled past the LDS hash to HBM
      // device time outside merges since the previous flag: waiting for commands, undoing guesses
      sd.hdr[20] = (uint32_t)(S.t_idle + (t_cmd - S.t_wait));
      sd.hdr[21] = (uint32_t)S.t_undo;
      sd.hdr[31] = S.t_rel;  // the previous flag's system release (L2 write-back + flag store), ticks
      h64[12] = S.lst_x;  // X's words-of list (0: none)
      h64[13] = t_cmd;    // diagnostic: absolute device clock at the command and at the wait's start
      h64[14] = S.t_wait;
      S.t_idle = 0;
      S.t_undo = 0;
      // one system-scope release (L2 write-back of the records and header, then the flag)
      const u64 t_r0 = __builtin_amdgcn_s_memrealtime();
      WL_ST(S.xs[11] = (uint32_t)(t_r0 - t_cmd); for (int i = 0; i < kXs; ++i) sd.hdr[32 + i] = S.xs[i];)
      __hip_atomic_store(sd.hdr + 1, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      S.t_rel = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_r0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // (the prefetch still in flight)
  }
  if (tid == 0) {
    p.dstate[kStPoolTop] = S.pool_top;
    if constexpr (kSelf) {
      p.sel.st[kSelIns] = S.sins;
      *reinterpret_cast<u64*>(p.sel.st + kSelLogW) = S.logn;
      p.sel.st[kSelErr] = S.serr;
      p.sel.st[kSelStatus] = exit_op;
      __threadfence_system();
      return;
    }
    p.status[1] = expect - 1u;  // the command this launch did not take (a time-out's resume point)
    __threadfence_system();
    __hip_atomic_store(&p.status[0], exit_op, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

namespace {

// Initial index, compact (round 6: the sort no longer spans the runs' padding): word w's
// adjacent pairs go to entries base[w] .. base[w] + L - 2 (base: exclusive sum of the words' pair
// counts, k_wl_pair_counts); pairs holding unk emit EMPTY.
__global__ void k_wl_pair_counts(const int32_t* wtok, const uint32_t* woff, uint32_t W, uint32_t* cnt) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w <= W; w += gridDim.x * blockDim.x) {
    const uint32_t L = w < W ? (uint32_t)wtok[woff[w]] : 0u;
    cnt[w] = L >= 2 ? L - 1 : 0u;
  }
}
__global__ void k_wl_emit_pairs(const int32_t* wtok, const uint32_t* woff, const uint32_t* base, uint32_t W,
                                int32_t unk, u64* key, uint32_t* val) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < W; w += gridDim.x * blockDim.x) {
    const uint32_t o = woff[w], b = base[w], np = base[w + 1] - b;
    const int32_t* t = wtok + o + kRunHdr;
    for (uint32_t j = 0; j < np; ++j) {
      const int32_t x = t[j], y = t[j + 1];
      key[b + j] = (x != unk && y != unk) ? pair_key(x, y) : kEmpty64;
      val[b + j] = w;
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
                             const uint32_t* pos, const uint32_t* head, const uint32_t* kidx, const uint32_t* woff,
                             WEnt* pool, u64* ikey, u64* ival) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (keep[i]) {
      WEnt ent;
      const uint32_t w = val[i], cap4 = (woff[w + 1] - woff[w]) >> 2;  // the run's 16-B groups
      ent.e = ((u64)woff[w] << 32) | ((u64)min(cap4, (uint32_t)kStripV) << kGroupShift) | w;
      ent.sig = ~0ull;  // an exact list: no filter
      pool[pos[i]] = ent;
    }
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
__global__ void k_wl_dir_init(const u64* ikey, const u64* ival, uint64_t nk, u64* dkey, u64* dval, u64 mask) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nk; i += (uint64_t)gridDim.x * blockDim.x) {
    const u64 key = ikey[i];
    u64 h = mix64(key) & mask;
    for (;;) {
      const u64 prev = atomicCAS(&dkey[h], kEmpty64, key);
      if (prev == kEmpty64) {
        dval[h] = ival[i];
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

// Each run's header gets its word's weight (ints 1-2), after a host upload of the runs.
__global__ void k_wl_set_weights(int32_t* wtok, const uint32_t* woff, uint32_t W, const u64* weight) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < W; w += gridDim.x * blockDim.x) {
    const u64 c = weight[w];
    wtok[woff[w] + 1] = (int32_t)(uint32_t)c;
    wtok[woff[w] + 2] = (int32_t)(uint32_t)(c >> 32);
  }
}

// Words -> tiles: a wave per tile writes [header][tokens] for its words in rank order and the
// tile's live length; the old tail up to the previous length becomes padding.
__global__ void k_words_to_tiles(const int32_t* wtok, const uint32_t* woff, const uint32_t* tile_first,
                                 const uint32_t* tile_nw, uint32_t ntiles, int32_t* tok, const uint64_t* tile_off,
                                 uint32_t* tile_len) {
  const int lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (blockDim.x / 64);
  for (uint32_t t = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); t < ntiles; t += waves) {
    int32_t* dst = tok + tile_off[t];
    const uint32_t f = tile_first[t], nw = tile_nw[t];
    uint32_t base = 0;
    for (uint32_t q = 0; q < nw; q += 64) {
      const uint32_t w = f + q + (uint32_t)lane;
      const bool on = q + (uint32_t)lane < nw;
      const int32_t* s = on ? wtok + woff[w] : wtok;
      const uint32_t len = on ? (uint32_t)s[0] : 0u;
      const uint32_t need = on ? len + 1u : 0u;
      const uint32_t incl = wave_incl_add(need);
      if (on) {
        int32_t* d = dst + base + incl - need;
        d[0] = (int32_t)((uint32_t)kHeaderBase + w);
        for (uint32_t j = 0; j < len; ++j) d[1 + j] = s[kRunHdr + j];
      }
      base += __shfl(incl, 63, 64);
    }
    const uint32_t old = tile_len[t];
    for (uint32_t i = base + (uint32_t)lane; i < old; i += 64) dst[i] = INT32_MIN;
    if (lane == 0) tile_len[t] = base;
  }
}

// Tiles -> words (inverse of k_words_to_tiles): a thread per tile walks its entries; each word's
// tokens go to its run after the live length.
__global__ void k_tiles_to_words(const int32_t* tok, const uint64_t* tile_off, const uint32_t* tile_len,
                                 uint32_t ntiles, const uint32_t* woff, int32_t* wtok) {
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += gridDim.x * blockDim.x) {
    const int32_t* src = tok + tile_off[t];
    const uint32_t n = tile_len[t];
    int32_t* run = nullptr;
    uint32_t len = 0;
    for (uint32_t i = 0; i < n; ++i) {
      const int32_t v = src[i];
      if (v < kHeaderLimit) {
        if (run) run[0] = (int32_t)len;
        const uint32_t w = (uint32_t)(v - kHeaderBase);
        run = wtok + woff[w];
        len = 0;
      } else if (run) {
        run[kRunHdr + len++] = v;
      }
    }
    if (run) run[0] = (int32_t)len;
  }
}

// ---- tiebreak=device: the frontier's rebuild (whole chip) and the table's initial pairs
constexpr uint32_t kSelBuckets = 65536u + 48u * 256u;  // exact counts below 2^16, 256 per octave above
constexpr uint32_t kSelLds = 16384;                    // buckets counted in LDS per workgroup
__host__ __device__ __forceinline__ uint32_t sel_bucket(u64 c) {
  if (c < 65536) return (uint32_t)c;
  int lg = 63;
  while (!((c >> lg) & 1ull)) --lg;
  return 65536u + (uint32_t)(lg - 16) * 256u + (uint32_t)((c >> (lg - 8)) & 255u);
}
// the smallest count in bucket b
inline u64 sel_bucket_lo(uint32_t b) {
  if (b < 65536u) return b;
  const uint32_t lg = 16u + (b - 65536u) / 256u, mant = (b - 65536u) % 256u;
  return (u64)(256u + mant) << (lg - 8u);
}

__global__ void k_sel_hist(u64* tab, u64 n, u64 minf, uint32_t* hist) {
  __shared__ uint32_t h[kSelLds];
  for (uint32_t i = threadIdx.x; i < kSelLds; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    const u64 cv = tab[2 * i + 1], c = cv & kCntMask;
    if (cv >> kPosShift) tab[2 * i + 1] = c;  // the last launch's frontier positions are void now
    if (tab[2 * i] == kEmpty64 || c < minf) continue;
    const uint32_t b = sel_bucket(c);
    if (b < kSelLds) atomicAdd(&h[b], 1u);
    else atomicAdd(&hist[b], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < kSelLds; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

__global__ void k_sel_collect(const u64* tab, u64 n, u64 minf, uint32_t bstar, uint32_t* out, uint32_t* nout,
                              u64 cap) {
  const int lane = threadIdx.x & 63;
  for (u64 i0 = blockIdx.x * (u64)blockDim.x; i0 < n; i0 += (u64)gridDim.x * blockDim.x) {
    const u64 i = i0 + threadIdx.x;
    bool take = false;
    if (i < n) {
      const u64 c = tab[2 * i + 1] & kCntMask;
      take = tab[2 * i] != kEmpty64 && c >= minf && sel_bucket(c) >= bstar;
    }
    const u64 bl = __ballot(take);
    if (!bl) continue;
    const int lead = __ffsll((long long)bl) - 1;
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(nout, (uint32_t)__popcll(bl));
    base = __shfl(base, lead, 64);
    const uint32_t pos = base + (uint32_t)__popcll(bl & ((1ull << lane) - 1ull));
    if (take && pos < cap) out[pos] = (uint32_t)i;
  }
}

__global__ void k_sel_gather(const uint32_t* slots, uint32_t n, const u64* tab, u64* key, u64* negc, uint32_t* idx) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    key[i] = tab[2 * (u64)slots[i]];
    negc[i] = ~(tab[2 * (u64)slots[i] + 1] & kCntMask);
    idx[i] = i;
  }
}

// idx: the sorted order; the first n of the collected slots in that order -> the frontier
__global__ void k_sel_pick(const uint32_t* slots, const uint32_t* idx, uint32_t n, uint32_t* fr) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    fr[i] = slots[idx ? idx[i] : i];
}

__global__ void k_sel_insert(const PairCount* pc, uint64_t n, SelParams q) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const u64 h = sel_slot(q, pair_key(pc[i].a, pc[i].b), q.st + kSelIns, q.st + kSelErr);
    if (h != ~0ull) q.tab[2 * h + 1] = pc[i].count & kCntMask;
  }
}

// The launch's logged changes into the table (whole chip, between launches): each a slot
// (inserted when new) and an add; the adds commute, so their order is free.
__global__ void k_sel_apply_log(const u64* log, u64 n, SelParams q) {
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    const u64 h = sel_slot(q, log[2 * i], q.st + kSelIns, q.st + kSelErr);
    if (h != ~0ull) atomicAdd(q.tab + 2 * h + 1, log[2 * i + 1]);
  }
}

// An empty table: every key kEmpty64, every count word 0.
__global__ void k_sel_clear(u64* tab, u64 n) {
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    tab[2 * i] = kEmpty64;
    tab[2 * i + 1] = 0;
  }
}

// The live pairs of a table (count > 0), for a bigger one.
__global__ void k_sel_export(const u64* tab, u64 cap, PairCount* out, uint32_t* n) {
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < cap; i += (u64)gridDim.x * blockDim.x) {
    const u64 k = tab[2 * i], c = tab[2 * i + 1] & kCntMask;
    if (k == kEmpty64 || c == 0) continue;
    const uint32_t j = atomicAdd(n, 1u);
    out[j] = PairCount{(int32_t)(uint32_t)(k >> 32), (int32_t)(uint32_t)k, c, 0};
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

constexpr uint32_t kRunPad = 4 * kStripV + 4;  // ints past the last run (its 16-B loads may overrun)

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
  // the idle bound (polls without a command before the launch ends itself); tests shrink it to
  // race the time-out against the posts
  if (const char* e = std::getenv("SHREDWORD_WL_IDLE_POLLS")) idle_polls_ = (uint32_t)std::strtoul(e, nullptr, 10);
  if (const char* e = std::getenv("SHREDWORD_WL_FINALIZE")) fin_max_ = (uint32_t)std::strtoul(e, nullptr, 10);
  if (const char* e = std::getenv("SHREDWORD_WL_FIN_MIN")) fin_min_ = (uint32_t)std::strtoul(e, nullptr, 10);
  if (const char* e = std::getenv("SHREDWORD_WL_PREFETCH")) prefetch_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("SHREDWORD_WL_DRAIN")) drain_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("SHREDWORD_WL_PROBES")) probes_ = std::atoi(e);
  if (const char* e = std::getenv("SHREDWORD_WL_FAST")) fast_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("SHREDWORD_SELECT_REPORT")) sel_report_ = std::atoi(e) != 0;
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
  sel_free();
  void* ptrs[] = {wtok_, wtok0_, woff_, tile_first_, tile_nw_, pool_, dkey_, dval_, init_key_, init_val_,
                  lst_, lseq_, dsum_, dft_, dlist_, dstate_};
  for (void* p : ptrs)
    if (p) WL_OK(hipFree(p));
  wtok_ = wtok0_ = nullptr;
  woff_ = tile_first_ = tile_nw_ = lseq_ = dlist_ = dstate_ = nullptr;
  pool_ = dkey_ = dval_ = init_key_ = init_val_ = lst_ = dsum_ = dft_ = nullptr;
  cap_ = id_cap_ = 0;
  dir_cap_ = 0;
  bytes_ = 0;
  ready_ = false;
}

bool WordLoop::upload(const TiledStream& ts, const uint64_t* d_weight) {
  WL_OK(hipSetDevice(ordinal_));
  if (running_) stop();
  free_all();
  // the words of the tile stream in rank order (types layout: one entry per distinct word), each
  // as a 16-B aligned run [length][tokens] of round_up(1 + length, 4) ints.  Threads over tile
  // ranges: a sizing pass (words and ints per tile, every header's rank checked against its
  // position), a prefix over the tiles, then each range fills its part of the runs.
  const size_t T = ts.num_tiles();
  const int P = (int)std::max<size_t>(1, std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()),
                                                          T / 64 + 1}));
  auto par = [&](const std::function<void(int)>& f) {
    if (P == 1) return f(0);
    std::vector<std::thread> pool;
    for (int k = 0; k < P; ++k) pool.emplace_back(f, k);
    for (auto& th : pool) th.join();
  };
  auto range = [&](int k, size_t* t0, size_t* t1) {
    *t0 = T * (size_t)k / (size_t)P;
    *t1 = T * (size_t)(k + 1) / (size_t)P;
  };
  std::vector<uint32_t> tnw(T, 0), tfirst(T, 0);
  std::vector<uint64_t> tints(T + 1, 0), ttok(T, 0);
  std::vector<int32_t> tr0(T, -1);  // the rank of the tile's first word (-1: none)
  std::vector<char> bad((size_t)P, 0);
  par([&](int k) {
    size_t t0, t1;
    range(k, &t0, &t1);
    for (size_t t = t0; t < t1 && !bad[(size_t)k]; ++t) {
      const int32_t* p = ts.tok.data() + ts.off[t];
      uint32_t nw = 0, wl = 0;
      uint64_t ints = 0, ntk = 0;
      for (uint32_t i = 0; i < ts.len[t]; ++i) {
        if (p[i] < kHeaderLimit) {
          const int32_t r = (int32_t)(uint32_t)(p[i] - kHeaderBase);
          if (nw == 0) tr0[t] = r;
          else if (r != tr0[t] + (int32_t)nw) bad[(size_t)k] = 1;  // ranks not consecutive
          if (nw) ints += run_cap(wl);
          ++nw;
          wl = 0;
        } else {
          if (nw == 0) bad[(size_t)k] = 1;  // tokens before any header
          ++wl;
          ++ntk;
        }
      }
      if (nw) ints += run_cap(wl);
      tnw[t] = nw;
      tints[t] = ints;
      ttok[t] = ntk;
    }
  });
  for (char b : bad)
    if (b) return false;  // not the whole table in rank order: not for this loop
  uint64_t words = 0, ints = 0, ntok = 0;
  for (size_t t = 0; t < T; ++t) {
    if (tnw[t] && tr0[t] != (int32_t)words) return false;
    tfirst[t] = (uint32_t)words;
    const uint64_t n = tints[t];
    tints[t] = ints;
    words += tnw[t];
    ints += n;
    ntok += ttok[t];
  }
  tints[T] = ints;
  if (ints >= 0xFFFFFF00ull) return false;  // offsets are 32-bit
  std::vector<uint32_t> woff(words + 1);
  std::vector<int32_t> wtok(ints + kRunPad, 0);
  par([&](int k) {
    size_t t0, t1;
    range(k, &t0, &t1);
    for (size_t t = t0; t < t1; ++t) {
      const int32_t* p = ts.tok.data() + ts.off[t];
      uint64_t o = tints[t], w = tfirst[t];
      int32_t* len = nullptr;
      for (uint32_t i = 0; i < ts.len[t]; ++i) {
        if (p[i] < kHeaderLimit) {
          if (len) o = (o + kRunAlign - 1u) & ~(uint64_t)(kRunAlign - 1u);
          woff[w++] = (uint32_t)o;
          len = &wtok[o];
          o += kRunHdr;  // (the weight ints are filled on the device: k_wl_set_weights)
        } else {
          wtok[o++] = p[i];
          ++*len;
        }
      }
    }
  });
  woff[words] = (uint32_t)ints;
  nwords_ = (uint32_t)(woff.size() - 1);
  nint_ = ints;
  ntok_ = ntok;
  ntiles_ = (uint32_t)ts.num_tiles();
  if (nwords_ == 0 || nint_ >= (1ull << 31)) return false;  // hipcub sizes are int
  if (nwords_ > kWordMask) return false;  // word ids share the pool entry with the run's groups
  // the pool (below) is addressed with 32-bit offsets (pool top, lst_, directory values)
  if (3 * ntok_ + 4096 >= (1ull << 32)) return false;
  for (uint32_t w = 0; w < nwords_; ++w)
    if (wtok[woff[w]] == 0) return false;  // words are never empty (strtok)
  weight_ = reinterpret_cast<const unsigned long long*>(d_weight);
  woff_h_ = woff;
  wtok_ = wl_alloc<int32_t>(nint_ + kRunPad, &bytes_);
  wtok0_ = wl_alloc<int32_t>(nint_ + kRunPad, &bytes_);
  woff_ = wl_alloc<uint32_t>(nwords_ + 1, &bytes_);
  tile_first_ = wl_alloc<uint32_t>(ntiles_, &bytes_);
  tile_nw_ = wl_alloc<uint32_t>(ntiles_, &bytes_);
  hipStream_t s = S(stream_);
  WL_OK(hipMemcpyAsync(wtok0_, wtok.data(), (nint_ + kRunPad) * sizeof(int32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(woff_, woff.data(), woff.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  k_wl_set_weights<<<(int)std::min<uint32_t>((nwords_ + 255) / 256, 4096), 256, 0, s>>>(wtok0_, woff_, nwords_, weight_);
  WL_OK(hipGetLastError());
  WL_OK(hipMemcpyAsync(tile_first_, tfirst.data(), ntiles_ * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(tile_nw_, tnw.data(), ntiles_ * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(wtok_, wtok0_, (nint_ + kRunPad) * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  // pool: the initial index (<= one entry per adjacent pair), the words-of lists (a merge lists
  // the words it shortened: Σ over a run <= Σ (length - 1)) and the pair groups (<= 2 entries
  // per occurrence merged: Σ <= 2 Σ (length - 1)); undone guesses release theirs (each is the
  // last when its undo runs)
  pool_cap_ = 3 * ntok_ + 4096;
  pool_ = wl_alloc<u64>(2 * pool_cap_, &bytes_);  // WEnt: entry + signature
  dstate_ = wl_alloc<uint32_t>(8, &bytes_);
  WL_OK(hipMemsetAsync(dstate_, 0, 8 * sizeof(uint32_t), s));
  WL_OK(hipStreamSynchronize(s));
  reserve(kBaseVocab + 1);
  build_index();
  ready_ = true;
  dirty_ = false;
  return true;
}

// The index of the current words: every (pair, word) once, grouped by pair.
void WordLoop::build_index() {
  hipStream_t s = S(stream_);
  size_t acc = 0;
  // the pairs of the current words, compactly: per-word counts, their exclusive sum
  uint32_t* pbase = wl_alloc<uint32_t>((size_t)nwords_ + 2, &acc);
  uint32_t* pcnt = wl_alloc<uint32_t>((size_t)nwords_ + 2, &acc);
  k_wl_pair_counts<<<(int)std::min<uint32_t>((nwords_ + 256) / 256, 4096), 256, 0, s>>>(wtok_, woff_, nwords_, pcnt);
  WL_OK(hipGetLastError());
  {
    size_t tb = 0;
    WL_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, pcnt, pbase, (int)nwords_ + 1, s));
    void* t0 = wl_alloc<uint8_t>(tb, &acc);
    WL_OK(hipcub::DeviceScan::ExclusiveSum(t0, tb, pcnt, pbase, (int)nwords_ + 1, s));
    WL_OK(hipStreamSynchronize(s));
    WL_OK(hipFree(t0));
  }
  uint32_t npairs = 0;
  WL_OK(hipMemcpy(&npairs, pbase + nwords_, sizeof(uint32_t), hipMemcpyDeviceToHost));
  const uint64_t n = std::max<uint64_t>(npairs, 1);
  u64* kin = wl_alloc<u64>(n, &acc);
  u64* kout = wl_alloc<u64>(n, &acc);
  uint32_t* vin = wl_alloc<uint32_t>(n, &acc);
  uint32_t* vout = wl_alloc<uint32_t>(n, &acc);
  uint32_t* keep = wl_alloc<uint32_t>(n + 1, &acc);
  uint32_t* head = wl_alloc<uint32_t>(n + 1, &acc);
  uint32_t* pos = wl_alloc<uint32_t>(n + 1, &acc);
  uint32_t* kidx = wl_alloc<uint32_t>(n + 1, &acc);
  const int grid = 2048;
  if (npairs == 0) {
    WL_OK(hipMemsetAsync(kin, 0xFF, sizeof(u64), s));
    WL_OK(hipMemsetAsync(vin, 0, sizeof(uint32_t), s));
  }
  k_wl_emit_pairs<<<grid, 256, 0, s>>>(wtok_, woff_, pbase, nwords_, unk_, kin, vin);
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
  if (init_pool_n_ > pool_cap_) fatal("WordLoop: the initial index exceeds the pool");
  if (init_key_) WL_OK(hipFree(init_key_));
  if (init_val_) WL_OK(hipFree(init_val_));
  init_key_ = wl_alloc<u64>(init_keys_n_, &bytes_);
  init_val_ = wl_alloc<u64>(init_keys_n_, &bytes_);
  k_wl_scatter<<<grid, 256, 0, s>>>(kout, vout, n, keep, pos, head, kidx, woff_, reinterpret_cast<WEnt*>(pool_),
                                    init_key_, init_val_);
  WL_OK(hipGetLastError());
  k_wl_counts<<<256, 256, 0, s>>>(init_val_, init_keys_n_, init_pool_n_);
  WL_OK(hipGetLastError());
  WL_OK(hipStreamSynchronize(s));
  for (void* p : {(void*)kin, (void*)kout, (void*)vin, (void*)vout, (void*)keep, (void*)head, (void*)pos, (void*)kidx,
                  tmp, (void*)pbase, (void*)pcnt})
    WL_OK(hipFree(p));
  // the directory: at most half full
  uint64_t want = 1024;
  while (want < 2 * init_keys_n_) want <<= 1;
  if (want != dir_cap_) {
    if (dkey_) WL_OK(hipFree(dkey_));
    if (dval_) WL_OK(hipFree(dval_));
    dir_cap_ = want;
    dkey_ = wl_alloc<u64>(dir_cap_, &bytes_);
    dval_ = wl_alloc<u64>(dir_cap_, &bytes_);
  }
  restore_index();
}

// The directory, the words-of lists and the counters as right after build_index().
void WordLoop::restore_index() {
  hipStream_t s = S(stream_);
  std::fill(lists_.begin(), lists_.end(), 0ull);  // no words-of lists: every merge looks its pair up
  WL_OK(hipMemsetAsync(dkey_, 0xFF, dir_cap_ * sizeof(u64), s));
  if (init_keys_n_) {
    k_wl_dir_init<<<1024, 256, 0, s>>>(init_key_, init_val_, init_keys_n_, dkey_, dval_, dir_cap_ - 1);
    WL_OK(hipGetLastError());
  }
  if (lseq_) WL_OK(hipMemsetAsync(lseq_, 0xFF, id_cap_ * sizeof(uint32_t), s));
  const uint32_t st[8] = {0, (uint32_t)init_pool_n_, 0, 0, 0, 0, 0, 0};
  WL_OK(hipMemcpyAsync(dstate_, st, sizeof(st), hipMemcpyHostToDevice, s));
  WL_OK(hipStreamSynchronize(s));
}

bool WordLoop::load_current(const TiledStream& ts) {
  WL_OK(hipSetDevice(ordinal_));
  if (!ready_ || !posted_.empty()) return false;
  stop();
  std::vector<int32_t> wtok(nint_ + kRunPad, 0);
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
        if (!open) return false;
        int32_t& len = wtok[woff_h_[w]];
        if (kRunHdr + (uint32_t)len >= woff_h_[w + 1] - woff_h_[w]) return false;  // past the run
        wtok[woff_h_[w] + kRunHdr + (uint32_t)len] = p[i];
        ++len;
      }
    }
  }
  if (!open || w + 1 != nwords_) return false;
  hipStream_t s = S(stream_);
  WL_OK(hipMemcpyAsync(wtok_, wtok.data(), wtok.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
  k_wl_set_weights<<<(int)std::min<uint32_t>((nwords_ + 255) / 256, 4096), 256, 0, s>>>(wtok_, woff_, nwords_, weight_);
  WL_OK(hipGetLastError());
  WL_OK(hipStreamSynchronize(s));
  build_index();
  dirty_ = false;
  return true;
}

void WordLoop::load_tiles(const int32_t* tok, const uint64_t* tile_off, const uint32_t* tile_len) {
  WL_OK(hipSetDevice(ordinal_));
  if (!ready_) return;
  if (!posted_.empty()) fatal("WordLoop::load_tiles with a merge in flight");
  stop();
  const int grid = (int)std::min<uint32_t>((ntiles_ + 255) / 256, 4096);
  k_tiles_to_words<<<std::max(grid, 1), 256, 0, S(stream_)>>>(tok, tile_off, tile_len, ntiles_, woff_, wtok_);
  WL_OK(hipGetLastError());
  build_index();
  dirty_ = false;
}

void WordLoop::reset_words() {
  WL_OK(hipSetDevice(ordinal_));
  if (!ready_) return;
  if (!posted_.empty()) fatal("WordLoop::reset_words with a merge in flight");
  stop();
  WL_OK(hipMemcpyAsync(wtok_, wtok0_, (nint_ + kRunPad) * sizeof(int32_t), hipMemcpyDeviceToDevice, S(stream_)));
  dirty_ = false;
}

void WordLoop::reset() {
  WL_OK(hipSetDevice(ordinal_));
  if (!ready_) return;
  if (!posted_.empty()) fatal("WordLoop::reset with a merge in flight");
  stop();
  hipStream_t s = S(stream_);
  WL_OK(hipMemcpyAsync(wtok_, wtok0_, (nint_ + kRunPad) * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  restore_index();
  dirty_ = false;
}

void WordLoop::ensure_slots(uint32_t cap) {
  const uint32_t rec_cap = 4 * (cap + 1) + 64;
  // records and headers: non-coherent pinned memory (the device's L2 holds the stores until the
  // release fence writes them back in one go; tools/rec_probe.hip: post -> every record seen
  // 3.1 us coherent + ordered flag, 2.3 us non-coherent + checksummed, round 6)
  const unsigned pin = hipHostMallocMapped | hipHostMallocNonCoherent;
  for (Slot& sl : slot_) {
    if (sl.host_recs) WL_OK(hipHostFree(sl.host_recs));
    WL_OK(hipHostMalloc((void**)&sl.host_recs, (size_t)rec_cap * sizeof(DeltaRecord), pin));
    WL_OK(hipHostGetDevicePointer(&sl.dev_recs, sl.host_recs, 0));
    if (!sl.host_hdr) {
      WL_OK(hipHostMalloc((void**)&sl.host_hdr, 256, pin));
      std::memset(sl.host_hdr, 0, 256);
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
  // the words-of lists (ids past the old capacity have none)
  u64* nl = wl_alloc<u64>(cap, &bytes_);
  uint32_t* ns = wl_alloc<uint32_t>(cap, &bytes_);

  WL_OK(hipMemsetAsync(ns, 0xFF, (size_t)cap * sizeof(uint32_t), s));

  if (lseq_) {
    WL_OK(hipMemcpyAsync(nl, lst_, (size_t)id_cap_ * sizeof(u64), hipMemcpyDeviceToDevice, s));
    WL_OK(hipMemcpyAsync(ns, lseq_, (size_t)id_cap_ * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));

    WL_OK(hipStreamSynchronize(s));
    for (void* q : {(void*)lst_, (void*)lseq_}) WL_OK(hipFree(q));
  }
  lst_ = nl;
  lseq_ = ns;

  id_cap_ = cap;
  cap_ = cap;
  lists_.resize(cap, 0ull);
  ensure_slots(cap);
  WL_OK(hipStreamSynchronize(s));
}

void WordLoop::launch(uint32_t seq0) {
  WlParams p{};
  p.wtok = wtok_;
  p.weight = weight_;
  p.pool = reinterpret_cast<WEnt*>(pool_);
  p.pool_cap = pool_cap_;
  p.dkey = dkey_;
  p.dval = dval_;
  p.dir_mask = dir_cap_ - 1;
  p.lst = lst_;
  p.lseq = lseq_;

  p.id_cap = id_cap_;
  p.dsum = dsum_;
  p.dft = dft_;
  p.dlist = dlist_;
  p.dstate = dstate_;
  p.cap = cap_;
  p.unk = unk_;
  p.ring = static_cast<const WlCmd*>(ring_dev_);
  p.status = static_cast<uint32_t*>(status_dev_);
  p.seq0 = seq0;
  p.idle_polls = idle_polls_;
  p.fin_max = fin_max_;
  p.fin_min = fin_min_;
  p.prefetch = prefetch_ ? 1u : 0u;
  p.drain = drain_ ? 1u : 0u;
  p.fast = fast_ ? 1u : 0u;
  for (int k = 0; k < kSlots; ++k) {
    p.sl[k].recs = static_cast<DeltaRecord*>(slot_[k].dev_recs);
    p.sl[k].hdr = static_cast<uint32_t*>(slot_[k].dev_hdr);
    p.sl[k].rec_cap = slot_[k].rec_cap;
  }
  status_[0] = 0;
  WL_OK(hipEventRecord((hipEvent_t)ev_[0], S(stream_)));
  switch (probes_) {  // SHREDWORD_WL_PROBES (tests): 0 / 1 force the delta hash's HBM spill path
    case 0: k_word_loop<false, 0><<<1, kWlThreads, 0, S(stream_)>>>(p); break;
    case 1: k_word_loop<false, 1><<<1, kWlThreads, 0, S(stream_)>>>(p); break;
    default: k_word_loop<false, kProbesDefault><<<1, kWlThreads, 0, S(stream_)>>>(p); break;
  }
  WL_OK(hipGetLastError());
  WL_OK(hipEventRecord((hipEvent_t)ev_[1], S(stream_)));
  running_ = true;
  ++st_.launches;
}

// The launch ended itself after ~10 s without a command.  It may have done so between a post's
// check and its ring store, so commands can be waiting: the loop published the first command it
// did not take (status_[1]), and a new launch resumes there (the ring still holds them).
void WordLoop::recover_timeout() {
  WL_OK(hipStreamSynchronize(S(stream_)));
  running_ = false;
  const uint32_t next = __atomic_load_n(&status_[1], __ATOMIC_ACQUIRE);
  if (next != seq_ + 1) {  // posted commands were not taken
    if (seq_ + 1 - next > kRing) fatal("k_word_loop: more commands behind its time-out than the ring holds");
    launch(next);
  }
}

uint32_t WordLoop::post(uint32_t op, int32_t a, int32_t b, int32_t X, uint32_t loff, uint32_t lcnt1) {
  if (running_ && __atomic_load_n(&status_[0], __ATOMIC_ACQUIRE) == kOpTimeout) recover_timeout();
  if (!running_) {
    if (op == kOpStop) return 0;
    launch(seq_ + 1);
  }
  const uint32_t seq = ++seq_;
  const uint32_t slot = (uint32_t)X & (kSlots - 1);
  u64* g = static_cast<WlCmd*>(ring_)[seq % kRing].g;
  const uint32_t vals[kCmdGranules] = {op | (slot << 8), (uint32_t)a, (uint32_t)b, (uint32_t)X, loff, lcnt1};
  for (int k = 0; k < kCmdGranules; ++k) __atomic_store_n(&g[k], (u64)seq | ((u64)vals[k] << 32), __ATOMIC_RELAXED);
  std::atomic_thread_fence(std::memory_order_release);
  return seq;
}

void WordLoop::post_merge(int32_t a, int32_t b, int32_t X) {
  if (!ready_) fatal("WordLoop::post_merge before upload");
  if (posted_.size() >= (size_t)kSlots) fatal("WordLoop: every merge slot is in flight");
  if (X < 0 || (uint32_t)X + 2 > cap_) fatal("WordLoop: merge id beyond the reserved ids");
  // the words-of list of max(a, b), when a collected merge made it: the loop skips its lookup
  const int32_t M = a > b ? a : b;
  const uint64_t l = M >= 0 && (size_t)M < lists_.size() ? lists_[M] : 0;
  const uint32_t seq = post(kOpMerge, a, b, X, (uint32_t)l, (uint32_t)(l >> 32));
  posted_.push_back({X, a, b, seq, now_seconds()});
  dirty_ = true;
}

// The small-merge path's hand-off (see hand_weight): both granules tagged with seq, then the
// checksum of header words 0..31 and the header's record count of records.
bool WordLoop::handed_over(const Slot& sl, uint32_t seq) const {
  const uint64_t* h64 = reinterpret_cast<const uint64_t*>(sl.host_hdr);
  const uint64_t g0 = __atomic_load_n(&h64[kCksWord], __ATOMIC_ACQUIRE), g1 = __atomic_load_n(&h64[kCksWord + 1], __ATOMIC_ACQUIRE);
  if ((uint32_t)(g0 >> 32) != seq || (uint32_t)(g1 >> 32) != seq) return false;
  const uint64_t want = (g0 & 0xFFFFFFFFull) | (g1 << 32);
  const uint32_t n = __atomic_load_n(&sl.host_hdr[0], __ATOMIC_ACQUIRE);
  if (n > sl.rec_cap) return false;
  uint64_t c = 0;
  for (uint32_t i = 0; i < 16; ++i) c += __atomic_load_n(&h64[i], __ATOMIC_RELAXED) * hand_weight(i);
  const uint64_t* r = reinterpret_cast<const uint64_t*>(sl.host_recs);
  for (uint32_t i = 0; i < 3 * n; ++i) c += __atomic_load_n(&r[i], __ATOMIC_RELAXED) * hand_weight(16u + i);
  return c == want;
}

void WordLoop::wait_flag(const Slot& sl, uint32_t seq) {
  volatile uint32_t* flag = sl.host_hdr + 1;
  const uint64_t* h64 = reinterpret_cast<const uint64_t*>(sl.host_hdr);
  const double t0 = now_seconds();
  unsigned spins = 0;
  for (;;) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) break;  // the ordered paths' flag
    if ((uint32_t)(__atomic_load_n(&h64[kCksWord + 1], __ATOMIC_ACQUIRE) >> 32) == seq && handed_over(sl, seq)) break;
    __builtin_ia32_pause();
    if (++spins % 4096 != 0) continue;
    const uint32_t st = __atomic_load_n(&status_[0], __ATOMIC_ACQUIRE);
    if (st == kOpTimeout) {
      recover_timeout();  // resumes at the first command it did not take (this one or earlier)
    } else if (st != 0) {
      fatal("k_word_loop ended with a merge in flight");
    }
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
  const double t_seen = now_seconds();
  st_.wait_us += 1e6 * (t_seen - pp.t_post);
  const uint32_t* h = sl.host_hdr;
  const uint64_t* h64 = reinterpret_cast<const uint64_t*>(h);
  const size_t n = h[0];
  st_.merges += 1;
  st_.candidates += h[2];
  st_.scanned += h[12];
  st_.run_ints_read += h[14];
  st_.run_ints_written += h[15];
  st_.records += h[0];
  st_.raw_records += h[22] ? h[23] : h[0];
  st_.finalized += h[22] ? 1u : 0u;
  st_.dev_out_us += 1e-2 * (double)h[30];
  st_.dev_rel_us += 1e-2 * (double)h[31];
  st_.spill_merges += h[19] ? 1u : 0u;
  st_.spill_keys += h[19];
  if (h[22]) {
    st_.dev_fin_us += 1e-2 * (double)h[30];
    st_.fin_records += h[23];
  }
  last_changes_ = h[22] != 0;
  st_.changed += h[3];
  st_.occurrences += h64[2];
  st_.dev_us += 1e-2 * (double)h64[3];  // s_memrealtime: 100 MHz
  st_.dev_lookup_us += 1e-2 * (double)h64[4];
  st_.dev_scan_us += 1e-2 * (double)(h64[5] - h64[4]);
  if (timing_) {
    const uint32_t rec[kTraceFields] = {(uint32_t)X, h[2], h[12], h[3], (uint32_t)h64[2], (uint32_t)(10 * h64[3]),
                                        (uint32_t)(10 * h64[4]), (uint32_t)(10 * (h64[5] - h64[4])),
                                        10 * h[16], 10 * h[17], 10 * h[18], h[19], 10 * h[20],
                                        10 * h[21], (uint32_t)(1e9 * (t_seen - pp.t_post)),
                                        // absolute clocks for a timeline: host 10 ns units since the
                                        // loop was made, device ticks (100 MHz), low 32 bits
                                        (uint32_t)(1e8 * (pp.t_post - t_epoch_)), (uint32_t)(1e8 * (t_seen - t_epoch_)),
                                        (uint32_t)h64[13], (uint32_t)h64[14],
                                        // SHRED_WL_STAMPS builds: phase stamps and counts (0 otherwise)
                                        h[32], h[33], h[34], h[35], h[36], h[37], h[38], h[39], h[40], h[41],
                                        h[42], h[43], h[44], h[45], h[46], h[47],
                                        // the previous flag's release ticks; (stamps) the poller saw the command
                                        h[31], h[48]};
    trace_.insert(trace_.end(), rec, rec + kTraceFields);
  }
  if (n > sl.rec_cap) fatal("k_word_loop: record overflow");
  if (h64[12] && (size_t)X < lists_.size()) lists_[X] = h64[12];
  *recs = sl.host_recs;
  return n;
}

bool WordLoop::peek(int32_t X, const DeltaRecord** recs, size_t* n) const {
  if (posted_.empty() || posted_.front().X != X) return false;
  const Slot& sl = slot_[(uint32_t)X & (kSlots - 1)];
  if (__atomic_load_n(sl.host_hdr + 1, __ATOMIC_ACQUIRE) != posted_.front().seq &&
      !handed_over(sl, posted_.front().seq))
    return false;
  if (sl.host_hdr[22]) return false;  // ordered changes already: nothing for the apply helper to prepare
  const size_t k = sl.host_hdr[0];
  if (k > sl.rec_cap) return false;  // collect() reports it
  *recs = sl.host_recs;
  *n = k;
  return true;
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
  uint32_t ds[8];
  WL_OK(hipMemcpy(ds, dstate_, sizeof(ds), hipMemcpyDeviceToHost));

  if (std::getenv("SHREDWORD_WL_REPORT") && st_.merges)
    std::fprintf(stderr, "[WL] %llu merges: device %.2f us a merge, of it the flag's system release %.2f us, "
                 "records out %.2f us; %llu merges spilled %llu delta keys to HBM\n", (unsigned long long)st_.merges,
                 st_.dev_us / (double)st_.merges, st_.dev_rel_us / (double)st_.merges,
                 st_.dev_out_us / (double)st_.merges, (unsigned long long)st_.spill_merges,
                 (unsigned long long)st_.spill_keys);
  if (ds[kStError]) {
    static const char* what[] = {"", "index pool exhausted", "an undone merge had no word list", "",
                                 "a merged pair had no word list"};
    std::fprintf(stderr, "[ERROR]\t k_word_loop: %s (code %u)\n", ds[kStError] < 5 ? what[ds[kStError]] : "?",
                 ds[kStError]);
    fatal("k_word_loop failed");
  }
}

// ==========================================================================================
// tiebreak=device

void WordLoop::sel_free() {
  void* ptrs[] = {ptab_, fr_[0], fr_[1], sst_dev_, thr_, sout_, upd_, shist_, scol_};
  for (void* q : ptrs)
    if (q) WL_OK(hipFree(q));
  ptab_ = thr_ = sout_ = nullptr;
  fr_[0] = fr_[1] = sst_dev_ = upd_ = shist_ = scol_ = nullptr;
  pcap_ = sout_cap_ = upd_cap_ = scol_cap_ = 0;
  fcap_ = 0;
}

// The frontier from the whole table: the kSelK best pairs by (count desc, key asc) among those
// >= min_freq (all of them when few), their slots flagged; the threshold = the last one taken
// (or, when every pair of the counts' top buckets was taken, the lowest count of those buckets).
bool WordLoop::sel_rebuild(uint64_t min_freq) {
  const double t0 = now_seconds();
  hipStream_t s = S(stream_);
  WL_OK(hipMemsetAsync(shist_, 0, kSelBuckets * sizeof(uint32_t), s));
  k_sel_hist<<<1024, 512, 0, s>>>(ptab_, pcap_, min_freq, shist_);
  WL_OK(hipGetLastError());
  std::vector<uint32_t> hist(kSelBuckets);
  WL_OK(hipMemcpyAsync(hist.data(), shist_, kSelBuckets * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  WL_OK(hipStreamSynchronize(s));
  uint64_t acc = 0;
  uint32_t bstar = kSelBuckets;
  for (uint32_t b = kSelBuckets; b-- > 0;) {
    if (!hist[b]) continue;
    acc += hist[b];
    bstar = b;
    if (acc >= kSelK) break;
  }
  uint32_t st[kSelStats] = {};
  WL_OK(hipMemcpyAsync(st, sst_dev_, sizeof(st), hipMemcpyDeviceToHost, s));
  WL_OK(hipStreamSynchronize(s));
  u64 thr[2] = {~0ull, 0ull};
  uint32_t nf = 0;
  if (acc > 0) {
    if (acc > scol_cap_) {
      if (scol_) WL_OK(hipFree(scol_));
      scol_cap_ = std::max<uint64_t>(2 * acc, 1 << 16);
      scol_ = wl_alloc<uint32_t>(scol_cap_ + 1, &bytes_);
    }
    uint32_t* ncol = scol_ + scol_cap_;
    WL_OK(hipMemsetAsync(ncol, 0, sizeof(uint32_t), s));
    k_sel_collect<<<1024, 512, 0, s>>>(ptab_, pcap_, min_freq, bstar, scol_, ncol, scol_cap_);
    WL_OK(hipGetLastError());
    uint32_t nc = 0;
    WL_OK(hipMemcpyAsync(&nc, ncol, sizeof(nc), hipMemcpyDeviceToHost, s));
    WL_OK(hipStreamSynchronize(s));
    if (nc != acc) fatal("tiebreak=device: the frontier's collect disagrees with its histogram");
    if (nc <= kSelK) {  // every pair of the top buckets: the threshold is their lowest count
      nf = nc;
      k_sel_pick<<<64, 256, 0, s>>>(scol_, nullptr, nf, fr_[0]);
      WL_OK(hipGetLastError());
      thr[0] = std::max<u64>(sel_bucket_lo(bstar), min_freq);
      thr[1] = ~0ull;
    } else {  // the top kSelK in (count desc, key asc) order: sort by key, then stably by count
      size_t acc2 = 0;
      u64* key = wl_alloc<u64>(nc, &acc2);
      u64* key2 = wl_alloc<u64>(nc, &acc2);
      u64* negc = wl_alloc<u64>(nc, &acc2);
      u64* negc2 = wl_alloc<u64>(nc, &acc2);
      uint32_t* idx = wl_alloc<uint32_t>(nc, &acc2);
      uint32_t* idx2 = wl_alloc<uint32_t>(nc, &acc2);
      k_sel_gather<<<256, 256, 0, s>>>(scol_, nc, ptab_, key, negc, idx);
      WL_OK(hipGetLastError());
      size_t tb = 0, tb2 = 0;
      WL_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key2, idx, idx2, (int)nc, 0, 64, s));
      WL_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, negc, negc2, idx, idx2, (int)nc, 0, 64, s));
      void* tmp = wl_alloc<uint8_t>(std::max(tb, tb2), &acc2);
      WL_OK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key2, idx, idx2, (int)nc, 0, 64, s));
      // counts in key order, then a stable sort by ~count
      k_sel_gather<<<256, 256, 0, s>>>(scol_, nc, ptab_, key, negc, idx);  // key/negc of slot order
      WL_OK(hipGetLastError());
      std::vector<uint32_t> order(nc);
      std::vector<u64> kc(nc), nn(nc);
      WL_OK(hipMemcpyAsync(order.data(), idx2, nc * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      WL_OK(hipMemcpyAsync(nn.data(), negc, nc * sizeof(u64), hipMemcpyDeviceToHost, s));
      WL_OK(hipMemcpyAsync(kc.data(), key, nc * sizeof(u64), hipMemcpyDeviceToHost, s));
      WL_OK(hipStreamSynchronize(s));
      // (host) ~count in key order, sorted stably on the device
      std::vector<u64> nk(nc);
      for (uint32_t i = 0; i < nc; ++i) nk[i] = nn[order[i]];
      WL_OK(hipMemcpyAsync(negc, nk.data(), nc * sizeof(u64), hipMemcpyHostToDevice, s));
      WL_OK(hipMemcpyAsync(idx, order.data(), nc * sizeof(uint32_t), hipMemcpyHostToDevice, s));
      WL_OK(hipcub::DeviceRadixSort::SortPairs(tmp, tb2, negc, negc2, idx, idx2, (int)nc, 0, 64, s));
      nf = kSelK;
      k_sel_pick<<<64, 256, 0, s>>>(scol_, idx2, nf, fr_[0]);
      WL_OK(hipGetLastError());
      uint32_t last = 0;
      WL_OK(hipMemcpyAsync(&last, idx2 + (nf - 1), sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      WL_OK(hipStreamSynchronize(s));
      thr[0] = ~nn[last];
      thr[1] = kc[last];
      for (void* q : {(void*)key, (void*)key2, (void*)negc, (void*)negc2, (void*)idx, (void*)idx2, tmp}) WL_OK(hipFree(q));
    }
  }
  st[kSelNF] = nf;
  st[kSelBuf] = 0;
  st[kSelStatus] = 0;
  WL_OK(hipMemcpyAsync(sst_dev_, st, sizeof(st), hipMemcpyHostToDevice, s));
  WL_OK(hipMemcpyAsync(thr_, thr, sizeof(thr), hipMemcpyHostToDevice, s));
  WL_OK(hipStreamSynchronize(s));
  sst_.rebuilds += 1;
  sst_.rebuild_ms += 1e3 * (now_seconds() - t0);
  sst_.frontier_max = std::max<uint64_t>(sst_.frontier_max, nf);
  return nf > 0;
}

int WordLoop::run_select(const std::vector<PairCount>& pairs, int32_t X0, uint32_t n_max, uint64_t min_freq,
                         std::vector<SelectedMerge>* out) {
  out->clear();
  if (!ready_ || !posted_.empty()) return -1;
  WL_OK(hipSetDevice(ordinal_));
  stop();
  if (n_max == 0) return 0;
  reserve(X0 + (int32_t)n_max);
  hipStream_t s = S(stream_);
  // the table: room for the initial pairs and ~64 new pairs a merge (C3 makes 62), 1.5x over;
  // past 3/4 full it is grown 4x between launches.  Round 5, with the table updated from a log
  // per launch: a smaller table is faster -- its rebuild histogram reads fewer slots and its
  // updates stay in L2 / MALL (C3 A/B on one box: 33.5 M slots 57.4-57.5 k merges/s, 8.4 M
  // 59.8-60.1 k, 4.2 M 60.3-60.4 k; profiles/r05_c3_tiebreak_table_ab.txt)
  uint64_t want = 1 << 16;
  while (want < 3 * ((uint64_t)pairs.size() + 64ull * n_max) / 2) want <<= 1;
  if (const char* e = std::getenv("SHREDWORD_SELECT_TABLE_SLOTS")) {  // tests: a table that must grow
    const uint64_t t = std::strtoull(e, nullptr, 10);
    if (t >= 1024) {  // never below what the initial pairs need (they must all fit)
      want = 1024;
      while (want < t || want < 2 * (uint64_t)pairs.size()) want <<= 1;
    }
  }
  if (!fr_[0]) {
    fcap_ = 16384;
    fr_[0] = wl_alloc<uint32_t>(fcap_, &bytes_);
    fr_[1] = wl_alloc<uint32_t>(fcap_, &bytes_);
    sst_dev_ = wl_alloc<uint32_t>(kSelWords, &bytes_);
    thr_ = wl_alloc<u64>(2, &bytes_);
    shist_ = wl_alloc<uint32_t>(kSelBuckets, &bytes_);
  }
  if (2ull * n_max > sout_cap_) {
    if (sout_) WL_OK(hipFree(sout_));
    sout_cap_ = 2ull * n_max;
    sout_ = wl_alloc<u64>(sout_cap_, &bytes_);
  }
  // the table-change log: many merges' records between two applications (a launch ends early
  // when one more merge might not fit)
  const uint64_t need_log = std::max<uint64_t>(1ull << 22, 16ull * ((uint64_t)cap_ + 2));
  if (need_log > upd_cap_) {
    if (upd_) WL_OK(hipFree(upd_));
    upd_cap_ = need_log;
    upd_ = wl_alloc<uint32_t>(4 * upd_cap_, &bytes_);  // (key, delta) u64 pairs
  }
  WL_OK(hipMemsetAsync(sst_dev_, 0, kSelWords * sizeof(uint32_t), s));
  SelParams q{};
  auto table_from = [&](const PairCount* dp, size_t np, uint64_t cap) {  // a fresh table holding dp
    if (cap != pcap_) {
      if (ptab_) WL_OK(hipFree(ptab_));
      pcap_ = cap;
      ptab_ = wl_alloc<u64>(2 * pcap_, &bytes_);
    }
    k_sel_clear<<<1024, 256, 0, s>>>(ptab_, pcap_);
    WL_OK(hipGetLastError());
    q.tab = ptab_;
    q.pmask = pcap_ - 1;
    q.fr[0] = fr_[0];
    q.fr[1] = fr_[1];
    q.fcap = fcap_;
    q.st = sst_dev_;
    q.thr = thr_;
    q.out = sout_;
    q.log = reinterpret_cast<u64*>(upd_);
    q.log_cap = upd_cap_;
    q.X0 = X0;
    q.n_max = n_max;
    q.min_freq = min_freq;
    q.fill_max = (uint32_t)std::min<uint64_t>(3 * pcap_ / 4, 0xFFFFFFF0ull);
    if (const char* e = std::getenv("SHREDWORD_SEL_PROBE")) q.probe = (uint32_t)std::atoi(e);
    uint32_t zero = 0;
    WL_OK(hipMemcpyAsync(sst_dev_ + kSelIns, &zero, sizeof(zero), hipMemcpyHostToDevice, s));
    WL_OK(hipMemcpyAsync(sst_dev_ + kSelErr, &zero, sizeof(zero), hipMemcpyHostToDevice, s));
    if (np) {
      k_sel_insert<<<512, 256, 0, s>>>(dp, np, q);
      WL_OK(hipGetLastError());
    }
    WL_OK(hipStreamSynchronize(s));
    uint32_t err = 0;  // a pair that found no slot within the probe bound would be a lost count
    WL_OK(hipMemcpy(&err, sst_dev_ + kSelErr, sizeof(err), hipMemcpyDeviceToHost));
    if (err) fatal("tiebreak=device: the pair table's initial pairs overran the probe bound");
  };
  {
    size_t acc = 0;
    PairCount* dp = pairs.empty() ? nullptr : wl_alloc<PairCount>(pairs.size(), &acc);
    if (dp) WL_OK(hipMemcpyAsync(dp, pairs.data(), pairs.size() * sizeof(PairCount), hipMemcpyHostToDevice, s));
    table_from(dp, pairs.size(), want);
    if (dp) WL_OK(hipFree(dp));
  }
  sst_.table_slots = pcap_;
  uint32_t m = 0;
  if (sel_rebuild(min_freq)) {
    WlParams p{};
    p.wtok = wtok_;
    p.weight = weight_;
    p.pool = reinterpret_cast<WEnt*>(pool_);
    p.pool_cap = pool_cap_;
    p.dkey = dkey_;
    p.dval = dval_;
    p.dir_mask = dir_cap_ - 1;
    p.lst = lst_;
    p.lseq = lseq_;
    p.id_cap = id_cap_;
    p.dsum = dsum_;
    p.dft = dft_;
    p.dlist = dlist_;
    p.dstate = dstate_;
    p.cap = cap_;
    p.unk = unk_;
    p.fast = fast_ ? 1u : 0u;  // small merges through the small-merge body (then the pair-table tail)
    p.sel = q;
    dirty_ = true;
    int stalls = 0;
    for (;;) {
      p.seq0 = seq_ + 1;
      WL_OK(hipEventRecord((hipEvent_t)ev_[0], s));
      switch (probes_) {
        case 0: k_word_loop<true, 0><<<1, kWlThreads, 0, s>>>(p); break;
        case 1: k_word_loop<true, 1><<<1, kWlThreads, 0, s>>>(p); break;
        default: k_word_loop<true, kProbesDefault><<<1, kWlThreads, 0, s>>>(p); break;
      }
      WL_OK(hipGetLastError());
      WL_OK(hipEventRecord((hipEvent_t)ev_[1], s));
      WL_OK(hipStreamSynchronize(s));
      float ms = 0;
      WL_OK(hipEventElapsedTime(&ms, (hipEvent_t)ev_[0], (hipEvent_t)ev_[1]));
      sst_.kernel_ms += ms;
      sst_.launches += 1;
      uint32_t st[kSelWords];
      WL_OK(hipMemcpy(st, sst_dev_, sizeof(st), hipMemcpyDeviceToHost));
      uint32_t ds[8];
      WL_OK(hipMemcpy(ds, dstate_, sizeof(ds), hipMemcpyDeviceToHost));
      if (ds[kStError]) {
        std::fprintf(stderr, "[ERROR]\t k_word_loop<true>: error code %u\n", ds[kStError]);
        fatal("tiebreak=device merge loop failed");
      }
      if (sel_report_)
        std::fprintf(stderr, "[SELECT] launch %llu: merges %u..%u in %.3f ms (%.2f us/merge), status %u, table %u, "
                     "%u LDS compactions\n", (unsigned long long)sst_.launches, m, st[kSelM], ms,
                     st[kSelM] > m ? 1e3 * ms / (st[kSelM] - m) : 0.0, st[kSelStatus], st[kSelIns], st[kSelBuf]);
      const bool progressed = st[kSelM] != m;
      m = st[kSelM];
      // the launch's logged changes into the table
      const u64 logn = *reinterpret_cast<const u64*>(st + kSelLogW);
      if (logn) {
        const double tl = now_seconds();
        k_sel_apply_log<<<1024, 256, 0, s>>>(reinterpret_cast<const u64*>(upd_), logn, q);
        WL_OK(hipGetLastError());
        WL_OK(hipMemsetAsync(sst_dev_ + kSelLogW, 0, sizeof(u64), s));
        WL_OK(hipMemcpyAsync(st + kSelIns, sst_dev_ + kSelIns, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        WL_OK(hipStreamSynchronize(s));
        sst_.log_ms += 1e3 * (now_seconds() - tl);
        sst_.log_entries += logn;
      }
      // a change whose pair found no table slot within the probe bound would be lost: the table
      // would no longer be the corpus's count, so there is nothing exact to grow from
      if (st[kSelErr]) fatal("tiebreak=device: a pair-table update overran the probe bound");
      const uint32_t status = st[kSelStatus];
      if (status == kSelDone) break;
      // a rebuild that merged nothing is not a full table: only kSelFull and the
      // inserts past the bound grow it.  Right after a rebuild the frontier holds entries at or
      // above the threshold, so two such launches in a row would be a loop that cannot progress.
      if (status == kSelRebuild && !progressed) {
        if (++stalls > 1) fatal("tiebreak=device: two launches in a row ended for a rebuild without a merge");
      } else {
        stalls = 0;
      }
      // the table past 3/4 full, or without room for one more merge's new pairs: 4x, live pairs moved
      if (st[kSelIns] > q.fill_max || status == kSelFull) {
        size_t acc = 0;
        PairCount* dp = wl_alloc<PairCount>(pcap_, &acc);
        uint32_t* dn = wl_alloc<uint32_t>(1, &acc);
        WL_OK(hipMemsetAsync(dn, 0, sizeof(uint32_t), s));
        k_sel_export<<<1024, 256, 0, s>>>(ptab_, pcap_, dp, dn);
        WL_OK(hipGetLastError());
        uint32_t np = 0;
        WL_OK(hipMemcpyAsync(&np, dn, sizeof(np), hipMemcpyDeviceToHost, s));
        WL_OK(hipStreamSynchronize(s));
        // the exported pairs must survive the old table's release: keep them in their own buffer
        const uint64_t grown = 4 * pcap_;
        u64* old = ptab_;
        ptab_ = nullptr;
        pcap_ = 0;
        table_from(dp, np, grown);
        WL_OK(hipFree(old));
        WL_OK(hipFree(dp));
        WL_OK(hipFree(dn));
        ++sst_.grows;
        p.sel = q;
        if (!sel_rebuild(min_freq)) break;
        continue;
      }
      if (status != kSelRebuild) fatal("tiebreak=device: the merge loop ended without a status");
      if (!sel_rebuild(min_freq)) break;
    }
    uint32_t st[kSelWords];
    WL_OK(hipMemcpy(st, sst_dev_, sizeof(st), hipMemcpyDeviceToHost));
    const u64* t64 = reinterpret_cast<const u64*>(st + kSelStats);
    sst_.select_us += 1e-2 * (double)t64[0];
    sst_.merge_us += 1e-2 * (double)t64[1];
    sst_.listed += t64[2];
    sst_.changed += t64[3];
    sst_.occurrences += t64[4];
    sst_.new_pairs += t64[5];
    sst_.table_us += 1e-2 * (double)t64[6];
    sst_.rec_us += 1e-2 * (double)t64[8];
    sst_.append_us += 1e-2 * (double)t64[9];
    sst_.tail_us += 1e-2 * (double)t64[10];
    if (sel_report_ && m)
      std::fprintf(stderr, "[SELECT] %u merges: device select %.2f us, merge %.2f us (of it table + frontier %.2f us: "
                   "records %.2f, appends %.2f, tail %.2f) per merge; %llu LDS compactions, %llu listed / %llu changed "
                   "words\n", m, 1e-2 * (double)t64[0] / m, 1e-2 * (double)t64[1] / m, 1e-2 * (double)t64[6] / m,
                   1e-2 * (double)t64[8] / m, 1e-2 * (double)t64[9] / m, 1e-2 * (double)t64[10] / m, (unsigned long long)t64[7],
                   (unsigned long long)t64[2], (unsigned long long)t64[3]);
    sst_.table_pairs = st[kSelIns];
  }
  sst_.table_slots = pcap_;
  sst_.merges += m;
  std::vector<u64> o(2 * (size_t)m);
  if (m) WL_OK(hipMemcpy(o.data(), sout_, o.size() * sizeof(u64), hipMemcpyDeviceToHost));
  out->resize(m);
  for (uint32_t i = 0; i < m; ++i)
    (*out)[i] = SelectedMerge{(int32_t)(uint32_t)(o[2 * i] >> 32), (int32_t)(uint32_t)o[2 * i], o[2 * i + 1]};
  return (int)m;
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
  k_words_to_tiles<<<std::max(grid, 1), 256, 0, S(stream_)>>>(wtok_, woff_, tile_first_, tile_nw_, ntiles_, tok,
                                                           tile_off, tile_len);
  WL_OK(hipGetLastError());
  dirty_ = false;
}

}  // namespace shred
