// MI355X (gfx950) kernels of the BPE merge loop and the Device class that drives them.
//
// Integer-only, HBM/LDS-bound work (no MFMA).  Every kernel walks the tiled token stream of
// device.h with 256-thread workgroups (4 wave64s), 16 consecutive tokens per lane, one 4096-token
// chunk per iteration; a tile longer than one chunk (a word of > 4095 tokens) is walked chunk by
// chunk with carries, so no word length is special.
//
//   k_pair_count   K1  weighted pair histogram + first touch     (reference bpe.cpp:187-206)
//   k_merge        K2+K3 match (a,b), emit the 4 neighbour deltas per occurrence, rewrite the
//                  chunk compacted in place                      (reference bpe.cpp:259-296)
//   k_collect      K4  touched delta slots -> host records       (FreqChangeMap, bpe.cpp:9-50)
//   k_token_freq   K6  final weighted token histogram            (reference bpe.cpp:409-415)
//
// Deltas and pair counts are staged in per-workgroup LDS hash tables and spilled to HBM tables
// with 64-bit atomics (sum) and atomicMin (first touch), so the reduction is order-free and the
// result bit-identical run to run.
#include <hip/hip_runtime.h>

#ifndef SHRED_MAX_GROUPS
#define SHRED_MAX_GROUPS 256
#endif
#ifndef SHRED_DELTA_LDS
#define SHRED_DELTA_LDS 2048
#endif

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../host/common.h"
#include "../host/device.h"
#include "../host/dist.h"

namespace shred {

#define HIP_OK(expr)                                                                        \
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

constexpr int kThreads = 256;
constexpr int kPer = 16;
constexpr int kChunk = kThreads * kPer;  // 4096 tokens = 16 KiB per chunk
constexpr int kPairLds = 2048;           // per-workgroup pair-count staging slots
constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;
constexpr unsigned long long kEmpty64 = ~0ull;
constexpr int32_t kPad = INT32_MIN;      // beyond the tile; also looks like a header

typedef unsigned long long u64;

__device__ __forceinline__ bool is_hdr(int32_t t) { return t < kHeaderLimit; }
__device__ __forceinline__ uint32_t hdr_rank(int32_t t) { return (uint32_t)(t - kHeaderBase); }

__device__ __forceinline__ u64 mix64(u64 k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  k *= 0xC4CEB9FE1A85EC53ull;
  k ^= k >> 33;
  return k;
}

// One exclusive block scan of a packed header key (max) and a counter (sum) over 256 lanes.
struct ScanLds {
  u64 hdr[4];
  int cnt[4];
};

__device__ __forceinline__ void block_scan_hdr_cnt(u64 hdr, int cnt, ScanLds& s, u64* hdr_excl, int* cnt_excl,
                                                   u64* hdr_tot, int* cnt_tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  u64 h = hdr;
  int c = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    u64 hy = __shfl_up(h, d, 64);
    int cy = __shfl_up(c, d, 64);
    if (lane >= d) {
      h = hy > h ? hy : h;
      c += cy;
    }
  }
  if (lane == 63) {
    s.hdr[w] = h;
    s.cnt[w] = c;
  }
  __syncthreads();
  u64 hp = 0;
  int cp = 0;
  for (int i = 0; i < w; ++i) {
    hp = s.hdr[i] > hp ? s.hdr[i] : hp;
    cp += s.cnt[i];
  }
  u64 ht = 0;
  int ct = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ht = s.hdr[i] > ht ? s.hdr[i] : ht;
    ct += s.cnt[i];
  }
  u64 hx = __shfl_up(h, 1, 64);
  int cx = __shfl_up(c, 1, 64);
  if (lane == 0) {
    hx = 0;
    cx = 0;
  }
  *hdr_excl = hx > hp ? hx : hp;
  *cnt_excl = cx + cp;
  *hdr_tot = ht;
  *cnt_tot = ct;
  __syncthreads();
}

// Loads this lane's 16 tokens of chunk [cs, cs+cl) (kPad beyond cl).  16-byte loads where the
// whole quad is in range: tiles start 16-byte aligned and chunks are 4096 tokens.
__device__ __forceinline__ void load_chunk(const int32_t* base, uint32_t cs, uint32_t cl, int p0, int32_t (&v)[kPer]) {
#pragma unroll
  for (int q = 0; q < kPer / 4; ++q) {
    const int idx = p0 + 4 * q;
    if (idx + 4 <= (int)cl) {
      const int4 x = *reinterpret_cast<const int4*>(base + cs + idx);
      v[4 * q] = x.x;
      v[4 * q + 1] = x.y;
      v[4 * q + 2] = x.z;
      v[4 * q + 3] = x.w;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * q + r] = (idx + r < (int)cl) ? base[cs + idx + r] : kPad;
    }
  }
}

// Token following this lane's 16 (from the next lane, or from memory at a wave edge).
__device__ __forceinline__ int32_t next_token(const int32_t* base, uint32_t cs, uint32_t len, int p0, int32_t v0) {
  int32_t nx = __shfl_down(v0, 1, 64);
  if ((threadIdx.x & 63) == 63) nx = (cs + p0 + kPer < len) ? base[cs + p0 + kPer] : kPad;
  return nx;
}

// ------------------------------------------------------------------------------------------
// K2+K3(+K4): merge scan, one wavefront per tile.
//
// A wave owns a tile (<= 1024 tokens, or one longer word walked in 1024-token chunks): each lane
// holds 16 consecutive tokens, occurrences / run parity / word headers / output offsets are
// wave-level scans (no workgroup barrier on the tile path), the 4 neighbour deltas of every
// occurrence go to a workgroup LDS hash shared by the 4 waves, and a changed chunk is compacted
// in LDS and written back in place.  The last workgroup to finish (agent-scope release/acquire
// on a ticket) turns the touched delta slots into host records and raises a host-visible flag,
// so one launch + one flag wait is the whole device side of a merge.
constexpr int kWaveTok = 64 * kPer;  // 1024 tokens per wave chunk
constexpr int kWaves = kThreads / 64;
constexpr int kDeltaLdsW = SHRED_DELTA_LDS;
constexpr uint32_t kFusedCollectMax = 4096;  // beyond this the host launches k_collect
constexpr uint32_t kNeedCollect = 0x80000000u;
constexpr uint32_t kTimingStride = 8;
constexpr uint32_t kInlineTiles = 768;     // candidate tiles that fit the kernel arguments
constexpr int kMaxMergeGroups = SHRED_MAX_GROUPS;  // fat persistent grid: waves walk tiles with prefetch

struct MergeParams {
  int32_t* tok;
  const uint64_t* tile_off;
  uint32_t* tile_len;
  uint32_t ntiles;
  const uint64_t* weight;
  int32_t a, b, X;
  uint32_t slot_cap;
  u64* dsum;
  u64* dft;
  uint32_t* dlist;
  uint32_t* dcount;
  u64* stats;         // [0] occurrences merged, [1] tokens rewritten
  uint32_t* done;     // completion tickets: [0..7] per blockIdx % 8 group, [8] top
  int fused;          // 1: last workgroup collects; 0: leave the tables (multi-GPU exchange)
  DeltaRecord* out;   // host-visible records
  uint32_t* hcount;   // host-visible: [0] record count (| kNeedCollect), [1] flag = seq, [2] matched tiles
  u64* hstats;        // host-visible: [0] occurrences, [1] tokens rewritten
  uint32_t* mlist;    // host-visible: tiles where the merge matched (-> tiles(X) of the index)
  uint32_t* mcount;   // device counter for mlist
  uint32_t seq;
  uint32_t nlist;     // 0: visit every tile; else visit list[0 .. nlist)
  uint32_t list[kInlineTiles];  // candidate tiles (tile skipping), passed in the kernel arguments
};

struct DeltaLds {
  uint32_t key[kDeltaLdsW];
  u64 sum[kDeltaLdsW];
  u64 ft[kDeltaLdsW];
};

__device__ __forceinline__ void delta_global(const MergeParams& p, uint32_t key, u64 w, u64 ft) {
  atomicAdd(&p.dsum[key], w);
  const u64 old = atomicMin(&p.dft[key], ft);
  if (old == kEmpty64) {  // exactly one toucher sees MAX
    atomicExch(&p.dlist[atomicAdd(p.dcount, 1u)], key);
  }
}

__device__ __forceinline__ void delta_emit(DeltaLds& h, const MergeParams& p, uint32_t key, u64 w, u64 ft) {
  uint32_t s = (key * 2654435761u) >> (32 - __builtin_ctz(kDeltaLdsW));
  for (int probe = 0; probe < 16; ++probe) {
    const uint32_t prev = atomicCAS(&h.key[s], kEmpty32, key);
    if (prev == kEmpty32 || prev == key) {
      atomicAdd(&h.sum[s], w);
      atomicMin(&h.ft[s], ft);
      return;
    }
    s = (s + 1) & (kDeltaLdsW - 1);
  }
  delta_global(p, key, w, ft);
}

__device__ __forceinline__ uint32_t slot_of(int32_t id, uint32_t cap) {
  return (uint32_t)id < cap ? (uint32_t)id + 1u : 0u;
}

// Orders this wave's LDS accesses across lanes (LDS executes one wave's ops in order; this
// keeps the compiler from moving them and drains lgkmcnt).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <class T>
__device__ __forceinline__ T wave_incl_max(T x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T y = __shfl_up(x, d, 64);
    if (lane >= d) x = y > x ? y : x;
  }
  return x;
}

__device__ __forceinline__ int wave_incl_sum(int x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

template <bool kWeighted>
__global__ __launch_bounds__(kThreads) void k_merge(MergeParams p) {
  __shared__ int32_t s_tok[kWaves][kWaveTok + 8];  // [2 + j] = chunk position j; [0],[1] = -2,-1
  __shared__ DeltaLds h;
  __shared__ uint32_t s_last;
  __shared__ u64 s_cnt[2];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int32_t* st = s_tok[wid];
  for (int i = threadIdx.x; i < kDeltaLdsW; i += kThreads) {
    h.key[i] = kEmpty32;
    h.sum[i] = 0;
    h.ft[i] = kEmpty64;
  }
  if (threadIdx.x < 2) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const int32_t a = p.a, b = p.b, X = p.X;
  const bool same = (a == b);
  const int p0 = lane * kPer;
  u64 n_merged = 0, n_written = 0;  // wave-uniform

  const uint32_t n_iter = p.nlist ? p.nlist : p.ntiles;
  const uint32_t stride = gridDim.x * kWaves;
  uint32_t it = blockIdx.x * kWaves + wid;
  // first chunk of the wave's next tile, loaded one tile ahead (latency hiding)
  uint32_t f_tile = 0, f_len = 0;
  int32_t* f_base = p.tok;
  int32_t fv[kPer];
  int32_t f_nx = kPad;
  auto fetch = [&](uint32_t i) {
    f_tile = p.nlist ? p.list[i] : i;
    f_len = p.tile_len[f_tile];
    f_base = p.tok + p.tile_off[f_tile];
    load_chunk(f_base, 0, min((uint32_t)kWaveTok, f_len), p0, fv);
    f_nx = next_token(f_base, 0, f_len, p0, fv[0]);
  };
  if (it < n_iter) fetch(it);
  for (; it < n_iter; it += stride) {
    const uint32_t tile = f_tile, len = f_len;
    int32_t* base = f_base;
    int32_t v0[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) v0[j] = fv[j];
    const int32_t nx0 = f_nx;
    if (it + stride < n_iter) fetch(it + stride);
    uint64_t tile_hits = 0;
    long long c_nona = -1;  // last tile index whose token != a (a == b only)
    u64 c_hdr = 0;          // ((index + 1) << 32) | rank of the last header, 0 = none
    bool c_m1 = false, c_m2 = false;
    int32_t c_t1 = kPad, c_t2 = kPad;
    uint32_t c_out = 0;
    bool dirty = false;
    for (uint32_t cs = 0; cs < len; cs += kWaveTok) {
      const uint32_t cl = min((uint32_t)kWaveTok, len - cs);
      const bool more = cs + cl < len;
      int32_t v[kPer];
      int32_t nx;
      if (cs == 0) {
#pragma unroll
        for (int j = 0; j < kPer; ++j) v[j] = v0[j];
        nx = nx0;
      } else {
        load_chunk(base, cs, cl, p0, v);
        nx = next_token(base, cs, len, p0, v[0]);
      }
      bool any = false;
#pragma unroll
      for (int j = 0; j < kPer; ++j) any |= (v[j] == a) & ((j + 1 < kPer ? v[j + 1] : nx) == b);
      if (!__any(any) && !dirty && !more) break;  // rest of the tile is unchanged

      // ---- stage the chunk with 2 tokens of left context and 2 of lookahead
#pragma unroll
      for (int j = 0; j < kPer; ++j) st[2 + p0 + j] = v[j];
      if (lane == 0) {
        st[0] = c_t2;
        st[1] = c_t1;
      }
      if (lane == 63) {
        st[2 + kWaveTok] = (cs + kWaveTok < len) ? base[cs + kWaveTok] : kPad;
        st[3 + kWaveTok] = (cs + kWaveTok + 1 < len) ? base[cs + kWaveTok + 1] : kPad;
      }
      wave_lds_sync();
      const int32_t last1 = st[2 + cl - 1];
      const int32_t last2 = st[2 + cl - 2];  // st[1] when cl == 1

      // ---- occurrences, greedy left to right (runs of a == b pair up from the run start)
      uint32_t mask = 0;
      long long nona_tot = -1;
      if (same) {
        long long nl = -1;
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if (v[j] != a) nl = (long long)(cs + p0 + j);
        const long long inc = wave_incl_max(nl);
        nona_tot = __shfl(inc, 63, 64);
        long long last = __shfl_up(inc, 1, 64);
        if (lane == 0) last = -1;
        last = last > c_nona ? last : c_nona;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const long long gi = (long long)(cs + p0 + j);
          if (v[j] != a) last = gi;
          else if ((j + 1 < kPer ? v[j + 1] : nx) == a && ((gi - last - 1) & 1) == 0) mask |= 1u << j;
        }
      } else {
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if (v[j] == a && (j + 1 < kPer ? v[j + 1] : nx) == b) mask |= 1u << j;
      }
      uint32_t prevm = __shfl_up(mask, 1, 64);
      if (lane == 0) prevm = (c_m1 ? 1u << 15 : 0u) | (c_m2 ? 1u << 14 : 0u);
      const uint32_t m_ext = (mask << 2) | ((prevm >> 14) & 3u);  // bit k <-> position p0 - 2 + k
      const uint32_t removed = (m_ext >> 1) & 0xFFFFu;           // bit j <-> match at p0 + j - 1
      const int valid = max(0, min(kPer, (int)cl - p0));
      const uint32_t vmask = valid >= kPer ? 0xFFFFu : ((1u << valid) - 1u);
      const int kc = __popc(~removed & vmask);
      const int nm = __popc(mask);
      uint32_t hmask = 0;  // word headers among this lane's valid positions
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (is_hdr(v[j])) hmask |= 1u << j;
      hmask &= vmask;
      u64 hl = 0;
      if (hmask) {
        const int j = 31 - __clz(hmask);
        hl = ((u64)(cs + p0 + j + 1) << 32) | hdr_rank(st[2 + p0 + j]);
      }
      const u64 hinc = wave_incl_max(hl);
      u64 hdr_ex = __shfl_up(hinc, 1, 64);
      if (lane == 0) hdr_ex = 0;
      const u64 hdr_tot = __shfl(hinc, 63, 64);
      const int cinc = wave_incl_sum(kc | (nm << 16));
      const int ctot = __shfl(cinc, 63, 64);
      const int kc_ex = (cinc - (kc | (nm << 16))) & 0xFFFF;
      const int kept = ctot & 0xFFFF;
      const int matches = ctot >> 16;

      // ---- neighbour deltas, 4 per occurrence (bpe.cpp:274-290)
      if (mask) {
        const u64 hdr_in = hdr_ex > c_hdr ? hdr_ex : c_hdr;
        for (uint32_t mrem = mask; mrem; mrem &= mrem - 1) {
          const int j = __ffs(mrem) - 1;
          const uint32_t hb = hmask & ((2u << j) - 1u);  // headers at or before j in this lane
          u64 hdr = hdr_in;
          if (hb) {
            const int jh = 31 - __clz(hb);
            hdr = ((u64)(cs + p0 + jh + 1) << 32) | hdr_rank(st[2 + p0 + jh]);
          }
          const uint32_t hidx = (uint32_t)(hdr >> 32) - 1u;
          const uint32_t rank = (uint32_t)hdr;
          const uint32_t gi = cs + p0 + j;
          const u64 w = kWeighted ? p.weight[rank] : 1ull;
          const u64 ftb = ((u64)rank << 32) | ((u64)(gi - hidx - 1u) << 2);
          if (gi - 1u > hidx) {  // left neighbour inside the word; X if it was just merged
            const int32_t left = ((m_ext >> j) & 1u) ? X : st[1 + p0 + j];
            const uint32_t sl = slot_of(left, p.slot_cap) << 2;
            delta_emit(h, p, sl | kOldLeft, w, ftb | kOldLeft);
            delta_emit(h, p, sl | kNewLeft, w, ftb | kNewLeft);
          }
          const int32_t right = st[4 + p0 + j];  // original token after b
          if (!is_hdr(right)) {
            const uint32_t sr = slot_of(right, p.slot_cap) << 2;
            delta_emit(h, p, sr | kOldRight, w, ftb | kOldRight);
            delta_emit(h, p, sr | kNewRight, w, ftb | kNewRight);
          }
        }
      }
      const bool write = dirty || matches > 0 || kept != (int)cl;
      if (write) {
        wave_lds_sync();  // every neighbour read is done: compact in place
        int o = kc_ex;
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if (j < valid && !((removed >> j) & 1u)) st[2 + o++] = ((mask >> j) & 1u) ? X : v[j];
        wave_lds_sync();
        for (int j = lane; j < kept; j += 64) base[c_out + j] = st[2 + j];
        dirty = true;
        n_written += (u64)kept;
      }
      n_merged += (u64)matches;
      tile_hits += (u64)matches;
      // ---- carries to the next chunk of this tile
      c_out += (uint32_t)kept;
      c_m1 = (__shfl(mask, (int)((cl - 1) / kPer), 64) >> ((cl - 1) % kPer)) & 1u;
      c_m2 = cl >= 2 ? ((__shfl(mask, (int)((cl - 2) / kPer), 64) >> ((cl - 2) % kPer)) & 1u) : c_m1;
      c_t1 = last1;
      c_t2 = last2;
      c_hdr = hdr_tot > c_hdr ? hdr_tot : c_hdr;
      if (same) c_nona = nona_tot > c_nona ? nona_tot : c_nona;
      wave_lds_sync();  // the copy-out reads st before the next chunk overwrites it
    }
    if (dirty && lane == 0) p.tile_len[tile] = c_out;
    if (tile_hits && lane == 0) p.mlist[atomicAdd(p.mcount, 1u)] = tile;
  }
  if (lane == 0) {
    if (n_merged) atomicAdd(&s_cnt[0], n_merged);
    if (n_written) atomicAdd(&s_cnt[1], n_written);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kDeltaLdsW; i += kThreads)
    if (h.key[i] != kEmpty32) delta_global(p, h.key[i], h.sum[i], h.ft[i]);
  if (threadIdx.x == 0) {
    if (s_cnt[0]) atomicAdd(&p.stats[0], s_cnt[0]);
    if (s_cnt[1]) atomicAdd(&p.stats[1], s_cnt[1]);
  }
  // ---- completion: the slot tables are only ever touched by device-scope atomics (performed
  // at the memory side), so every wave draining its own vmcnt before the ticket is the whole
  // hand-off; the collector reads them with atomics too (MI355X_MICROARCH.md, valid forms).
  // Tickets are sharded by blockIdx % 8 so no counter sees more than gridDim/8 arrivals.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t g = blockIdx.x & 7u;
    const uint32_t in_group = (gridDim.x - g + 7u) >> 3;
    bool last = false;
    if (atomicAdd(&p.done[g], 1u) == in_group - 1u) {
      atomicExch(&p.done[g], 0u);
      const uint32_t groups = gridDim.x < 8u ? gridDim.x : 8u;
      last = atomicAdd(&p.done[8], 1u) == groups - 1u;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) s_cnt[0] = atomicAdd(p.dcount, 0u);
  __syncthreads();
  const uint32_t n = (uint32_t)s_cnt[0];
  const bool collect = p.fused && n <= kFusedCollectMax;
  if (collect) {
    for (uint32_t i0 = 0; i0 < n; i0 += kThreads * 4) {
      uint32_t key[4];
      u64 sum[4], ft[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t i = i0 + k * kThreads + threadIdx.x;
        key[k] = i < n ? atomicOr(&p.dlist[i], 0u) : 0u;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t i = i0 + k * kThreads + threadIdx.x;
        if (i < n) {
          sum[k] = atomicExch(&p.dsum[key[k]], 0ull);
          ft[k] = atomicExch(&p.dft[key[k]], kEmpty64);
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t i = i0 + k * kThreads + threadIdx.x;
        if (i < n) {
          DeltaRecord r;
          r.key = key[k];
          r.pad = 0;
          r.sum = sum[k];
          r.ft = ft[k];
          p.out[i] = r;
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (p.fused) {
      if (collect) atomicExch(p.dcount, 0u);
      p.hstats[0] = atomicExch(&p.stats[0], 0ull);
      p.hstats[1] = atomicExch(&p.stats[1], 0ull);
      p.hcount[0] = collect ? n : (n | kNeedCollect);
    }
    p.hcount[2] = atomicExch(p.mcount, 0u);
    atomicExch(&p.done[8], 0u);
    __threadfence_system();
    __hip_atomic_store(&p.hcount[1], p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// K4: touched slots -> records in host-visible memory; clears the slots for the next merge.
__global__ __launch_bounds__(kThreads) void k_collect(uint32_t* dcount, const uint32_t* dlist, u64* dsum, u64* dft,
                                                       DeltaRecord* out) {
  const uint32_t n = *dcount;
  for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
    const uint32_t key = dlist[i];
    DeltaRecord r;
    r.key = key;
    r.pad = 0;
    r.sum = dsum[key];
    r.ft = dft[key];
    out[i] = r;
    dsum[key] = 0;
    dft[key] = kEmpty64;
  }
}

__global__ void k_zero_u32(uint32_t* p) { *p = 0; }

// K4 (multi-GPU): after the all-reduce every rank scans the dense prefix instead of its own list.
__global__ __launch_bounds__(kThreads) void k_collect_dense(uint32_t nkeys, u64* dsum, u64* dft, DeltaRecord* out,
                                                             uint32_t* out_count) {
  for (uint32_t key = blockIdx.x * kThreads + threadIdx.x; key < nkeys; key += gridDim.x * kThreads) {
    const u64 ft = dft[key];
    if (ft == kEmpty64) continue;
    DeltaRecord r;
    r.key = key;
    r.pad = 0;
    r.sum = dsum[key];
    r.ft = ft;
    out[atomicAdd(out_count, 1u)] = r;
    dsum[key] = 0;
    dft[key] = kEmpty64;
  }
}

// ------------------------------------------------------------------------------------------
// K1: pair count
struct CountParams {
  const int32_t* tok;
  const uint64_t* tile_off;
  const uint32_t* tile_len;
  uint32_t ntiles;
  const uint64_t* weight;
  int32_t unk;
  u64* tkey;
  u64* tcnt;
  u64* tft;
  u64 tmask;
  uint32_t* overflow;
};

struct PairLds {
  u64 key[kPairLds];
  u64 cnt[kPairLds];
  u64 ft[kPairLds];
};

__device__ __forceinline__ void pair_global(const CountParams& p, u64 key, u64 c, u64 ft) {
  u64 s = mix64(key) & p.tmask;
  for (u64 probe = 0; probe <= p.tmask; ++probe) {
    const u64 prev = atomicCAS(&p.tkey[s], kEmpty64, key);
    if (prev == kEmpty64 || prev == key) {
      atomicAdd(&p.tcnt[s], c);
      atomicMin(&p.tft[s], ft);
      return;
    }
    s = (s + 1) & p.tmask;
  }
  atomicOr(p.overflow, 1u);
}

__device__ __forceinline__ void pair_emit(PairLds& h, const CountParams& p, u64 key, u64 c, u64 ft) {
  uint32_t s = (uint32_t)(mix64(key) >> 53);  // 11 bits
  for (int probe = 0; probe < 16; ++probe) {
    const u64 prev = atomicCAS(&h.key[s], kEmpty64, key);
    if (prev == kEmpty64 || prev == key) {
      atomicAdd(&h.cnt[s], c);
      atomicMin(&h.ft[s], ft);
      return;
    }
    s = (s + 1) & (kPairLds - 1);
  }
  pair_global(p, key, c, ft);
}

template <bool kWeighted>
__global__ __launch_bounds__(kThreads) void k_pair_count(CountParams p) {
  __shared__ PairLds h;
  __shared__ ScanLds s_scan;
  const int tid = threadIdx.x;
  for (int i = tid; i < kPairLds; i += kThreads) {
    h.key[i] = kEmpty64;
    h.cnt[i] = 0;
    h.ft[i] = kEmpty64;
  }
  __syncthreads();
  const int p0 = tid * kPer;
  for (uint32_t tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    const uint32_t len = p.tile_len[tile];
    const int32_t* base = p.tok + p.tile_off[tile];
    u64 c_hdr = 0;
    for (uint32_t cs = 0; cs < len; cs += kChunk) {
      const uint32_t cl = min((uint32_t)kChunk, len - cs);
      int32_t v[kPer];
      load_chunk(base, cs, cl, p0, v);
      const int32_t nx = next_token(base, cs, len, p0, v[0]);
      u64 hl = 0;
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (is_hdr(v[j]) && p0 + j < (int)cl) hl = ((u64)(cs + p0 + j + 1) << 32) | hdr_rank(v[j]);
      u64 hdr_ex, hdr_tot;
      int cx, ct;
      block_scan_hdr_cnt(hl, 0, s_scan, &hdr_ex, &cx, &hdr_tot, &ct);
      u64 hdr = hdr_ex > c_hdr ? hdr_ex : c_hdr;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int32_t x = v[j];
        const int32_t y = j + 1 < kPer ? v[j + 1] : nx;
        if (is_hdr(x)) {
          if (p0 + j < (int)cl) hdr = ((u64)(cs + p0 + j + 1) << 32) | hdr_rank(x);
          continue;
        }
        if (is_hdr(y) || x == p.unk || y == p.unk) continue;
        const uint32_t hidx = (uint32_t)(hdr >> 32) - 1u;
        const uint32_t rank = (uint32_t)hdr;
        const u64 w = kWeighted ? p.weight[rank] : 1ull;
        const u64 key = ((u64)(uint32_t)x << 32) | (uint32_t)y;
        pair_emit(h, p, key, w, ((u64)rank << 32) | (u64)(cs + p0 + j - hidx - 1u));
      }
      c_hdr = hdr_tot > c_hdr ? hdr_tot : c_hdr;
    }
  }
  __syncthreads();
  for (int i = tid; i < kPairLds; i += kThreads)
    if (h.key[i] != kEmpty64) pair_global(p, h.key[i], h.cnt[i], h.ft[i]);
}

__global__ __launch_bounds__(kThreads) void k_pair_collect(const u64* tkey, const u64* tcnt, const u64* tft, u64 cap,
                                                            PairCount* out, uint32_t out_cap, uint32_t* n) {
  for (u64 i = (u64)blockIdx.x * kThreads + threadIdx.x; i < cap; i += (u64)gridDim.x * kThreads) {
    const u64 k = tkey[i];
    if (k == kEmpty64) continue;
    PairCount pc;
    pc.a = (int32_t)(uint32_t)(k >> 32);
    pc.b = (int32_t)(uint32_t)k;
    pc.count = tcnt[i];
    pc.ft = tft[i];
    const uint32_t i_out = atomicAdd(n + 1, 1u);
    if (i_out < out_cap) out[i_out] = pc;
    else atomicOr(n, 2u);
  }
}

// ------------------------------------------------------------------------------------------
// K6: final token histogram over ids [0, T) (the unk count lands on unk_id when it is in range)
template <bool kWeighted>
__global__ __launch_bounds__(kThreads) void k_token_freq(const int32_t* tok, const uint64_t* tile_off,
                                                          const uint32_t* tile_len, uint32_t ntiles,
                                                          const uint64_t* weight, uint32_t T, u64* freq) {
  __shared__ ScanLds s_scan;
  const int p0 = threadIdx.x * kPer;
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint32_t len = tile_len[tile];
    const int32_t* base = tok + tile_off[tile];
    u64 c_hdr = 0;
    for (uint32_t cs = 0; cs < len; cs += kChunk) {
      const uint32_t cl = min((uint32_t)kChunk, len - cs);
      int32_t v[kPer];
      load_chunk(base, cs, cl, p0, v);
      u64 hl = 0;
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (is_hdr(v[j]) && p0 + j < (int)cl) hl = ((u64)(cs + p0 + j + 1) << 32) | hdr_rank(v[j]);
      u64 hdr_ex, hdr_tot;
      int cx, ct;
      block_scan_hdr_cnt(hl, 0, s_scan, &hdr_ex, &cx, &hdr_tot, &ct);
      u64 hdr = hdr_ex > c_hdr ? hdr_ex : c_hdr;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if (is_hdr(v[j])) {
          if (p0 + j < (int)cl) hdr = ((u64)(cs + p0 + j + 1) << 32) | hdr_rank(v[j]);
          continue;
        }
        if ((uint32_t)v[j] >= T) continue;
        atomicAdd(&freq[v[j]], kWeighted ? weight[(uint32_t)hdr] : 1ull);
      }
      c_hdr = hdr_tot > c_hdr ? hdr_tot : c_hdr;
    }
  }
}

__global__ void k_sum_len(const uint32_t* tile_len, uint32_t n, u64* out) {
  u64 s = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += tile_len[i];
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_down(s, d, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

inline hipStream_t S(void* s) { return (hipStream_t)s; }
inline u64* U(uint64_t* p) { return reinterpret_cast<u64*>(p); }

template <class T>
T* dalloc(size_t n, size_t* acc) {
  void* p = nullptr;
  if (n == 0) n = 1;
  HIP_OK(hipMalloc(&p, n * sizeof(T)));
  *acc += n * sizeof(T);
  return (T*)p;
}

}  // namespace

// ==========================================================================================
bool Device::available(std::string* why) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    if (why) *why = e != hipSuccess ? std::string("hipGetDeviceCount: ") + hipGetErrorString(e) : "no HIP device";
    return false;
  }
  return true;
}

Device::Device(int device_ordinal) : ordinal_(device_ordinal) {
  HIP_OK(hipSetDevice(ordinal_));
  hipStream_t s;
  HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  stream_ = s;
  for (auto& e : ev_) {
    hipEvent_t ev;
    HIP_OK(hipEventCreate(&ev));
    e = ev;
  }
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, ordinal_));
  cu_count_ = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  HIP_OK(hipHostMalloc((void**)&host_count_, 64, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(host_count_, 0, 64);
  HIP_OK(hipHostGetDevicePointer(&dev_count_, host_count_, 0));
  merge_params_ = new MergeParams();
  if (const char* e = std::getenv("SHREDWORD_TILE_SKIP")) skip_ = std::atoi(e) != 0;
  int nb = 0;  // resident workgroups of k_merge per CU
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(&k_merge<true>), kThreads, 0));
  merge_blocks_per_cu_ = nb > 0 ? nb : 4;
}

void Device::free_all() {
  void* ptrs[] = {tok_, tok0_, tile_off_, tile_len_, tile_len0_, weight_, dsum_, dft_, dlist_, dcount_};
  for (void* p : ptrs)
    if (p) HIP_OK(hipFree(p));
  tok_ = tok0_ = nullptr;
  tile_off_ = nullptr;
  tile_len_ = tile_len0_ = nullptr;
  weight_ = nullptr;
  dsum_ = dft_ = nullptr;
  dlist_ = dcount_ = nullptr;
  if (host_recs_) HIP_OK(hipHostFree(host_recs_));
  host_recs_ = nullptr;
  host_recs_cap_ = 0;
  slot_cap_ = 0;
  ntiles_ = 0;
  bytes_alloc_ = 0;
  uploaded_ = false;
}

Device::~Device() {
  (void)hipSetDevice(ordinal_);
  (void)hipStreamSynchronize(S(stream_));
  free_all();
  if (host_count_) (void)hipHostFree(host_count_);
  if (host_mlist_) (void)hipHostFree(host_mlist_);
  delete static_cast<MergeParams*>(merge_params_);
  for (auto e : ev_)
    if (e) (void)hipEventDestroy((hipEvent_t)e);
  if (stream_) (void)hipStreamDestroy(S(stream_));
}

void Device::upload(const TiledStream& ts, Layout layout, const std::vector<uint64_t>& weights, int32_t max_id) {
  HIP_OK(hipSetDevice(ordinal_));
  HIP_OK(hipStreamSynchronize(S(stream_)));
  free_all();
  layout_ = layout;
  ntiles_ = ts.num_tiles();
  tok_elems_ = ts.elems;
  live_tokens0_ = ts.live;
  live_tokens_est_ = ts.live;
  nentries_ = ts.entries;
  tok_ = dalloc<int32_t>(ts.elems + 4, &bytes_alloc_);
  tok0_ = dalloc<int32_t>(ts.elems + 4, &bytes_alloc_);
  tile_off_ = dalloc<uint64_t>(ntiles_, &bytes_alloc_);
  tile_len_ = dalloc<uint32_t>(ntiles_, &bytes_alloc_);
  tile_len0_ = dalloc<uint32_t>(ntiles_, &bytes_alloc_);
  HIP_OK(hipMemcpyAsync(tok0_, ts.tok.data(), (ts.elems + 4) * sizeof(int32_t), hipMemcpyHostToDevice, S(stream_)));
  if (ntiles_) {
    HIP_OK(hipMemcpyAsync(tile_off_, ts.off.data(), ntiles_ * sizeof(uint64_t), hipMemcpyHostToDevice, S(stream_)));
    HIP_OK(hipMemcpyAsync(tile_len0_, ts.len.data(), ntiles_ * sizeof(uint32_t), hipMemcpyHostToDevice, S(stream_)));
  }
  if (layout == Layout::kTypes) {
    weight_ = dalloc<uint64_t>(weights.size(), &bytes_alloc_);
    if (!weights.empty())
      HIP_OK(hipMemcpyAsync(weight_, weights.data(), weights.size() * sizeof(uint64_t), hipMemcpyHostToDevice,
                            S(stream_)));
  }
  HIP_OK(hipStreamSynchronize(S(stream_)));
  if (host_mlist_) HIP_OK(hipHostFree(host_mlist_));
  HIP_OK(hipHostMalloc((void**)&host_mlist_, (ntiles_ + 1) * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
  HIP_OK(hipHostGetDevicePointer(&dev_mlist_, host_mlist_, 0));
  index_.build(ts);
  max_id_seen_ = max_id;
  uploaded_ = true;
  reset_tokens();
}

void Device::reset_tokens() {
  HIP_OK(hipSetDevice(ordinal_));
  if (!uploaded_) return;
  HIP_OK(hipMemcpyAsync(tok_, tok0_, (tok_elems_ + 4) * sizeof(int32_t), hipMemcpyDeviceToDevice, S(stream_)));
  if (ntiles_)
    HIP_OK(hipMemcpyAsync(tile_len_, tile_len0_, ntiles_ * sizeof(uint32_t), hipMemcpyDeviceToDevice, S(stream_)));
  live_tokens_est_ = live_tokens0_;
  index_.reset();
}

uint64_t Device::live_tokens() {
  HIP_OK(hipSetDevice(ordinal_));
  if (!ntiles_) return 0;
  u64* d = dalloc<u64>(1, &bytes_alloc_);
  HIP_OK(hipMemsetAsync(d, 0, sizeof(u64), S(stream_)));
  k_sum_len<<<64, 256, 0, S(stream_)>>>(tile_len_, (uint32_t)ntiles_, d);
  u64 h = 0;
  HIP_OK(hipMemcpyAsync(&h, d, sizeof(u64), hipMemcpyDeviceToHost, S(stream_)));
  HIP_OK(hipStreamSynchronize(S(stream_)));
  HIP_OK(hipFree(d));
  bytes_alloc_ -= sizeof(u64);
  return h;
}

void Device::ensure_slots(uint32_t need) {
  if (need <= slot_cap_ && dsum_) return;
  uint32_t cap = std::max<uint32_t>(slot_cap_ ? slot_cap_ : 1024, 1024);
  while (cap < need) cap *= 2;
  HIP_OK(hipStreamSynchronize(S(stream_)));
  if (dsum_) {
    HIP_OK(hipFree(dsum_));
    HIP_OK(hipFree(dft_));
    HIP_OK(hipFree(dlist_));
    HIP_OK(hipFree(dcount_));
    HIP_OK(hipHostFree(host_recs_));
  }
  const size_t keys = 4 * ((size_t)cap + 1);
  dsum_ = dalloc<uint64_t>(keys + 2, &bytes_alloc_);  // + 2 stats words at the end
  dft_ = dalloc<uint64_t>(keys, &bytes_alloc_);
  dlist_ = dalloc<uint32_t>(keys, &bytes_alloc_);
  dcount_ = dalloc<uint32_t>(16, &bytes_alloc_);  // [0] count, [1..9] tickets, [10] matched tiles
  HIP_OK(hipMemsetAsync(dsum_, 0, (keys + 2) * sizeof(u64), S(stream_)));
  HIP_OK(hipMemsetAsync(dft_, 0xFF, keys * sizeof(u64), S(stream_)));
  HIP_OK(hipMemsetAsync(dcount_, 0, 16 * sizeof(uint32_t), S(stream_)));
  HIP_OK(hipHostMalloc((void**)&host_recs_, keys * sizeof(DeltaRecord), hipHostMallocMapped | hipHostMallocCoherent));
  HIP_OK(hipHostGetDevicePointer(&dev_recs_, host_recs_, 0));
  host_recs_cap_ = keys;
  slot_cap_ = cap;
  HIP_OK(hipStreamSynchronize(S(stream_)));
}

void Device::count_pairs(int32_t unk_id, std::vector<PairCount>* out) {
  HIP_OK(hipSetDevice(ordinal_));
  out->clear();
  if (!ntiles_) {
    dist_merge_pairs(out);
    return;
  }
  // distinct pairs <= live tokens and <= (ids in play)^2
  const uint64_t live = live_tokens();
  const uint64_t ids = (uint64_t)std::max<int32_t>(max_id_seen_, kBaseVocab) + 2;
  uint64_t bound = std::min<uint64_t>(live, ids * ids);
  uint64_t cap = 1024;
  while (cap < 2 * bound && cap < (1ull << 27)) cap *= 2;
  size_t acc = 0;
  u64* tkey = dalloc<u64>(cap, &acc);
  u64* tcnt = dalloc<u64>(cap, &acc);
  u64* tft = dalloc<u64>(cap, &acc);
  uint32_t* flags = dalloc<uint32_t>(2, &acc);
  HIP_OK(hipMemsetAsync(tkey, 0xFF, cap * sizeof(u64), S(stream_)));
  HIP_OK(hipMemsetAsync(tcnt, 0, cap * sizeof(u64), S(stream_)));
  HIP_OK(hipMemsetAsync(tft, 0xFF, cap * sizeof(u64), S(stream_)));
  HIP_OK(hipMemsetAsync(flags, 0, 2 * sizeof(uint32_t), S(stream_)));
  CountParams cp{tok_, tile_off_, tile_len_, (uint32_t)ntiles_, weight_, unk_id, tkey, tcnt, tft, cap - 1, flags};
  const int grid = (int)std::min<size_t>(ntiles_, (size_t)cu_count_ * 2);
  if (timing_) HIP_OK(hipEventRecord((hipEvent_t)ev_[2], S(stream_)));
  if (layout_ == Layout::kStream) k_pair_count<false><<<grid, kThreads, 0, S(stream_)>>>(cp);
  else k_pair_count<true><<<grid, kThreads, 0, S(stream_)>>>(cp);
  HIP_OK(hipGetLastError());
  if (timing_) HIP_OK(hipEventRecord((hipEvent_t)ev_[3], S(stream_)));
  const uint32_t out_cap = (uint32_t)std::min<uint64_t>(cap, bound + 1);
  PairCount* dout = dalloc<PairCount>(out_cap, &acc);
  k_pair_collect<<<512, kThreads, 0, S(stream_)>>>(tkey, tcnt, tft, cap, dout, out_cap, flags);
  HIP_OK(hipGetLastError());
  uint32_t hflags[2];
  HIP_OK(hipMemcpyAsync(hflags, flags, sizeof(hflags), hipMemcpyDeviceToHost, S(stream_)));
  HIP_OK(hipStreamSynchronize(S(stream_)));
  if (hflags[0]) fatal("pair table overflow in k_pair_count / k_pair_collect");
  out->resize(hflags[1]);
  if (hflags[1])
    HIP_OK(hipMemcpy(out->data(), dout, hflags[1] * sizeof(PairCount), hipMemcpyDeviceToHost));
  if (timing_) {
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, (hipEvent_t)ev_[2], (hipEvent_t)ev_[3]));
    times_.count_ms += ms;
    times_.count_launches += 1;
    // tokens + headers read once, plus the per-word weight in the types layout
    // 4 B per token and per word header (the boundary), 8 B weight per word in the types
    // layout, 12 B of tile descriptor per tile
    times_.count_bytes += 4.0 * (double)live + 12.0 * (double)ntiles_ +
                          (layout_ == Layout::kTypes ? 8.0 * (double)nentries_ : 0.0);
  }
  for (void* p : {(void*)tkey, (void*)tcnt, (void*)tft, (void*)flags, (void*)dout}) HIP_OK(hipFree(p));
  dist_merge_pairs(out);
}

void Device::flush_timing() {
  if (!timing_pending_) return;
  timing_pending_ = false;
  HIP_OK(hipEventSynchronize((hipEvent_t)ev_[1]));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, (hipEvent_t)ev_[0], (hipEvent_t)ev_[1]));
  times_.merge_ms += ms;
  times_.merge_launches += 1;
  times_.merge_bytes += pending_bytes_;
}

void Device::merge_scan(int32_t a, int32_t b, int32_t X) {
  HIP_OK(hipSetDevice(ordinal_));
  max_id_seen_ = std::max(max_id_seen_, X);
  ensure_slots((uint32_t)X + 1);
  flush_timing();
  launched_ = false;
  if (!ntiles_) return;  // an empty shard still joins collect()'s exchange
  ++seq_;
  launched_ = true;
  MergeParams& mp = *static_cast<MergeParams*>(merge_params_);
  mp.tok = tok_;
  mp.tile_off = tile_off_;
  mp.tile_len = tile_len_;
  mp.ntiles = (uint32_t)ntiles_;
  mp.weight = weight_;
  mp.a = a;
  mp.b = b;
  mp.X = X;
  mp.slot_cap = slot_cap_;
  mp.dsum = U(dsum_);
  mp.dft = U(dft_);
  mp.dlist = dlist_;
  mp.dcount = dcount_;
  mp.stats = U(dsum_) + 4 * ((size_t)slot_cap_ + 1);
  mp.done = dcount_ + 1;
  mp.fused = exchange_ ? 0 : 1;
  mp.out = (DeltaRecord*)dev_recs_;
  mp.hcount = (uint32_t*)dev_count_;
  mp.hstats = (u64*)((char*)dev_count_ + 16);
  mp.mlist = (uint32_t*)dev_mlist_;
  mp.mcount = dcount_ + 10;
  mp.seq = seq_;
  mp.nlist = 0;
  // tile skipping: visit only tiles(a) ∩ tiles(b) when that list is short
  if (skip_ && index_.candidates(a, b, &cand_) && cand_.size() <= kInlineTiles) {
    mp.nlist = (uint32_t)cand_.size();
    std::memcpy(mp.list, cand_.data(), cand_.size() * sizeof(uint32_t));
  }
  const size_t n_iter = mp.nlist ? mp.nlist : ntiles_;
  visited_tiles_ += n_iter;
  const size_t groups = (n_iter + kWaves - 1) / kWaves;
  const int grid = (int)std::min<size_t>(groups, (size_t)kMaxMergeGroups);
  // HIP events bracket every kTimingStride-th launch (an unbiased sample of launch durations
  // that keeps event overhead out of the timed loop)
  const bool sample = timing_ && (seq_ % kTimingStride == 0);
  if (sample) HIP_OK(hipEventRecord((hipEvent_t)ev_[0], S(stream_)));
  if (layout_ == Layout::kStream) k_merge<false><<<grid, kThreads, 0, S(stream_)>>>(mp);
  else k_merge<true><<<grid, kThreads, 0, S(stream_)>>>(mp);
  HIP_OK(hipGetLastError());
  if (sample) {
    HIP_OK(hipEventRecord((hipEvent_t)ev_[1], S(stream_)));
    timing_pending_ = true;
    // algorithmic bytes of this launch: the visited tiles' live tokens (estimated from the
    // mean tile length) + their descriptors
    const double frac = ntiles_ ? (double)n_iter / (double)ntiles_ : 0.0;
    pending_bytes_ = frac * 4.0 * (double)live_tokens_est_ + 12.0 * (double)n_iter;
  }
}

// Spins on the host-visible flag the last workgroup raises (much cheaper than a stream sync).
void Device::wait_flag() {
  volatile uint32_t* flag = host_count_ + 1;
  const double t0 = now_seconds();
  unsigned spins = 0;
  while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq_) {
    __builtin_ia32_pause();
    if (++spins % 4096 == 0 && now_seconds() - t0 > 120.0) {
      const hipError_t e = hipStreamQuery(S(stream_));
      if (e != hipSuccess && e != hipErrorNotReady) HIP_OK(e);
      if (now_seconds() - t0 > 600.0) fatal("k_merge did not signal completion within 600 s");
    }
  }
}

size_t Device::collect(int32_t X, const DeltaRecord** recs) {
  HIP_OK(hipSetDevice(ordinal_));
  (void)X;
  *recs = host_recs_;
  if (!ntiles_ && !exchange_) return 0;
  DeltaRecord* drec = (DeltaRecord*)dev_recs_;
  if (launched_) {
    wait_flag();
    index_.set_tiles(X, host_mlist_, host_count_[2]);
  }
  launched_ = false;
  const u64* hs = (const u64*)(host_count_ + 4);
  size_t n;
  u64* stats = U(dsum_) + 4 * ((size_t)slot_cap_ + 1);
  if (exchange_) {
    // multi-GPU: all-reduce the live prefix of the slot tables, then every rank scans it
    const uint32_t unk_slot = (unk_ >= 0 && (uint32_t)unk_ < slot_cap_) ? (uint32_t)unk_ : 0u;
    const size_t top = std::max<uint32_t>((uint32_t)X, unk_slot);
    const size_t nkeys = 4 * (std::min<size_t>(slot_cap_, top + 1) + 1);
    exchange_(exchange_ctx_, dsum_, dft_, nkeys, stream_);
    HIP_OK(hipMemsetAsync(dcount_, 0, sizeof(uint32_t), S(stream_)));
    k_collect_dense<<<256, kThreads, 0, S(stream_)>>>((uint32_t)nkeys, U(dsum_), U(dft_), drec, dcount_);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(host_count_, dcount_, sizeof(uint32_t), hipMemcpyDeviceToHost, S(stream_)));
    HIP_OK(hipMemcpyAsync((u64*)(host_count_ + 4), stats, 2 * sizeof(u64), hipMemcpyDeviceToHost, S(stream_)));
    HIP_OK(hipMemsetAsync(dcount_, 0, sizeof(uint32_t), S(stream_)));
    HIP_OK(hipMemsetAsync(stats, 0, 2 * sizeof(u64), S(stream_)));
    HIP_OK(hipStreamSynchronize(S(stream_)));
    n = host_count_[0];
  } else {
    n = host_count_[0];
    if (n & kNeedCollect) {  // too many touched slots for one workgroup: a wide collect pass
      n &= ~kNeedCollect;
      k_collect<<<256, kThreads, 0, S(stream_)>>>(dcount_, dlist_, U(dsum_), U(dft_), drec);
      HIP_OK(hipGetLastError());
      k_zero_u32<<<1, 1, 0, S(stream_)>>>(dcount_);
      HIP_OK(hipGetLastError());
      HIP_OK(hipStreamSynchronize(S(stream_)));
    }
  }
  live_tokens_est_ -= hs[0];
  records_total_ += n;
  records_max_ = std::max<uint64_t>(records_max_, n);
  return n;
}

void Device::token_freq(size_t T, std::vector<uint64_t>* freq) {
  HIP_OK(hipSetDevice(ordinal_));
  freq->assign(T, 0);
  if (!ntiles_ || !T) {
    dist_allreduce_host(freq->data(), T, false);
    return;
  }
  size_t acc = 0;
  u64* d = dalloc<u64>(T, &acc);
  HIP_OK(hipMemsetAsync(d, 0, T * sizeof(u64), S(stream_)));
  const int grid = (int)std::min<size_t>(ntiles_, (size_t)cu_count_ * 4);
  if (layout_ == Layout::kStream)
    k_token_freq<false><<<grid, kThreads, 0, S(stream_)>>>(tok_, tile_off_, tile_len_, (uint32_t)ntiles_, weight_, (uint32_t)T, d);
  else
    k_token_freq<true><<<grid, kThreads, 0, S(stream_)>>>(tok_, tile_off_, tile_len_, (uint32_t)ntiles_, weight_, (uint32_t)T, d);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(freq->data(), d, T * sizeof(u64), hipMemcpyDeviceToHost, S(stream_)));
  HIP_OK(hipStreamSynchronize(S(stream_)));
  HIP_OK(hipFree(d));
  dist_allreduce_host(freq->data(), T, false);
}

void Device::download_tokens(std::vector<int32_t>* out) {
  HIP_OK(hipSetDevice(ordinal_));
  out->clear();
  if (!ntiles_) return;
  std::vector<int32_t> all(tok_elems_ + 4);
  std::vector<uint64_t> off(ntiles_);
  std::vector<uint32_t> lens(ntiles_);
  HIP_OK(hipMemcpyAsync(all.data(), tok_, all.size() * sizeof(int32_t), hipMemcpyDeviceToHost, S(stream_)));
  HIP_OK(hipMemcpyAsync(off.data(), tile_off_, ntiles_ * sizeof(uint64_t), hipMemcpyDeviceToHost, S(stream_)));
  HIP_OK(hipMemcpyAsync(lens.data(), tile_len_, ntiles_ * sizeof(uint32_t), hipMemcpyDeviceToHost, S(stream_)));
  HIP_OK(hipStreamSynchronize(S(stream_)));
  for (size_t t = 0; t < ntiles_; ++t) out->insert(out->end(), all.begin() + off[t], all.begin() + off[t] + lens[t]);
}

}  // namespace shred
