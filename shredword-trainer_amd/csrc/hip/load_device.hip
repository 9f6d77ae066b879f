// GPU word count of the corpus load (replaces the O(tokens · W / 4096) word
// counting of reference bpe.cpp:110-153 / hash.cpp:29-72 on the device).
//
// The file's bytes are uploaded once; then, on gfx950:
//   k_word_count   one thread per 64-byte chunk takes the words that START in its chunk (maximal
//                  runs of bytes outside "\t\r\n "), hashes each (64-bit FNV-1a + length mix)
//                  with its djb2 & 4095 (the reference StrMap bucket), and counts it in a
//                  per-workgroup LDS table (count, min first offset) that spills to, and is
//                  flushed into, one open-addressing HBM table with 64-bit atomics;
//   k_word_verify  every occurrence is compared byte for byte with its entry's first occurrence,
//                  so a 64-bit key collision is detected (the count is then repeated with another
//                  seed) and the table is exact;
//   k_word_compact entries -> (bucket << 52 | first offset) keys, radix-sorted (hipCUB): the
//                  reference word order, since first offsets are distinct;
//   k_word_gather  rank -> {first, count, length} records for the host.
// The host keeps the fgets/strlen path for files with NUL bytes (corpus.cpp) and builds the word
// table (spellings, coverage, symbols) from the records.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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
constexpr int kLoadThreads = 256;
constexpr int kLdsSlots = 2048;      // per-workgroup staging table (57 KB: two workgroups per CU)
constexpr int kLdsProbes = 8;
constexpr size_t kPadBytes = 256;    // ' ' past the corpus: every word scan ends inside the buffer

__device__ __forceinline__ bool delim(uint32_t c) { return c == 9u || c == 13u || c == 10u || c == 32u; }

struct Table {
  u64* key;       // 0 = empty; else mix(hash, len, seed) | 1
  u64* cnt;
  u64* first;     // min first offset
  uint32_t* len;
  uint32_t* bkt;  // djb2 & 4095
  u64 mask;       // capacity - 1
  uint32_t* nkeys;
  uint32_t* flags;  // [0] table too full, [1] key collision
};

__device__ __forceinline__ u64 word_key(u64 h, uint32_t len, u64 seed) {
  h ^= (u64)len * 0x9E3779B97F4A7C15ull ^ seed;
  h ^= h >> 31;
  h *= 0xD6E8FEB86659FD93ull;
  h ^= h >> 32;
  return h | 1ull;
}

// The word starting at d[pos]: its key, djb2 bucket and length.
__device__ __forceinline__ void scan_word(const uint8_t* d, u64 pos, u64 seed, u64* key, uint32_t* bkt, uint32_t* len) {
  u64 h = 0xCBF29CE484222325ull ^ seed;
  uint32_t dj = 5381u;  // djb2 in 32 bits: its & 4095 equals the reference's 64-bit value's
  uint32_t l = 0;
  for (;; ++l) {
    const uint32_t c = d[pos + l];
    if (delim(c)) break;
    h = (h ^ c) * 0x100000001B3ull;
    dj = dj * 33u + c;
  }
  *key = word_key(h, l, seed);
  *bkt = dj & 4095u;
  *len = l;
}

__device__ __forceinline__ void table_add(const Table& t, u64 key, uint32_t bkt, uint32_t len, u64 cnt, u64 first) {
  u64 s = key & t.mask;
  for (u64 probe = 0; probe <= t.mask; ++probe) {
    const u64 prev = atomicCAS(&t.key[s], 0ull, key);
    if (prev == 0ull) {
      t.len[s] = len;
      t.bkt[s] = bkt;
      if (atomicAdd(t.nkeys, 1u) > (uint32_t)((t.mask + 1) / 4 * 3)) atomicOr(&t.flags[0], 1u);
    }
    if (prev == 0ull || prev == key) {
      atomicAdd(&t.cnt[s], cnt);
      atomicMin(&t.first[s], first);
      return;
    }
    s = (s + 1) & t.mask;
  }
  atomicOr(&t.flags[0], 1u);
}

__global__ __launch_bounds__(kLoadThreads) void k_word_count(const uint8_t* d, u64 n, Table t, u64 seed) {
  __shared__ u64 s_key[kLdsSlots];
  __shared__ u64 s_first[kLdsSlots];
  __shared__ uint32_t s_cnt[kLdsSlots];
  __shared__ uint32_t s_len[kLdsSlots];
  __shared__ uint32_t s_bkt[kLdsSlots];
  for (int i = threadIdx.x; i < kLdsSlots; i += kLoadThreads) {
    s_key[i] = 0;
    s_first[i] = ~0ull;
    s_cnt[i] = 0;
  }
  __syncthreads();
  const u64 nchunks = (n + kChunkBytes - 1) / kChunkBytes;
  for (u64 c = (u64)blockIdx.x * kLoadThreads + threadIdx.x; c < nchunks; c += (u64)gridDim.x * kLoadThreads) {
    const u64 c0 = c * kChunkBytes;
    const u64 c1 = c0 + kChunkBytes < n ? c0 + kChunkBytes : n;
    uint32_t prev = c0 ? d[c0 - 1] : 32u;
    for (u64 i = c0; i < c1; ++i) {
      const uint32_t b = d[i];
      if (!delim(b) && delim(prev)) {
        u64 key;
        uint32_t bkt, len;
        scan_word(d, i, seed, &key, &bkt, &len);
        uint32_t s = (uint32_t)(key >> 40) & (kLdsSlots - 1);
        bool done = false;
        for (int probe = 0; probe < kLdsProbes && !done; ++probe) {
          const u64 old = atomicCAS(&s_key[s], 0ull, key);
          if (old == 0ull || old == key) {
            if (old == 0ull) {
              s_len[s] = len;
              s_bkt[s] = bkt;
            }
            atomicAdd(&s_cnt[s], 1u);
            atomicMin(&s_first[s], i);
            done = true;
          } else {
            s = (s + 1) & (kLdsSlots - 1);
          }
        }
        if (!done) table_add(t, key, bkt, len, 1ull, i);
      }
      prev = b;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLdsSlots; i += kLoadThreads)
    if (s_key[i]) table_add(t, s_key[i], s_bkt[i], s_len[i], s_cnt[i], s_first[i]);
}

// Every occurrence against its entry's first occurrence: a mismatch is a 64-bit key collision.
__global__ __launch_bounds__(kLoadThreads) void k_word_verify(const uint8_t* d, u64 n, Table t, u64 seed) {
  const u64 nchunks = (n + kChunkBytes - 1) / kChunkBytes;
  for (u64 c = (u64)blockIdx.x * kLoadThreads + threadIdx.x; c < nchunks; c += (u64)gridDim.x * kLoadThreads) {
    const u64 c0 = c * kChunkBytes;
    const u64 c1 = c0 + kChunkBytes < n ? c0 + kChunkBytes : n;
    uint32_t prev = c0 ? d[c0 - 1] : 32u;
    for (u64 i = c0; i < c1; ++i) {
      const uint32_t b = d[i];
      if (!delim(b) && delim(prev)) {
        u64 key;
        uint32_t bkt, len;
        scan_word(d, i, seed, &key, &bkt, &len);
        u64 s = key & t.mask;
        bool found = false;
        for (u64 probe = 0; probe <= t.mask; ++probe) {
          const u64 k = t.key[s];
          if (k == key) {
            found = true;
            break;
          }
          if (k == 0ull) break;
          s = (s + 1) & t.mask;
        }
        bool same = found && t.len[s] == len;
        if (same) {
          const u64 f = t.first[s];
          for (uint32_t k = 0; k < len && same; ++k) same = d[f + k] == d[i + k];
        }
        if (!same) atomicOr(&t.flags[1], 1u);
      }
      prev = b;
    }
  }
}

__global__ void k_word_compact(Table t, u64* okey, uint32_t* oslot, uint32_t* nout) {
  for (u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x; s <= t.mask; s += (u64)gridDim.x * blockDim.x) {
    if (!t.key[s]) continue;
    const uint32_t i = atomicAdd(nout, 1u);
    okey[i] = ((u64)t.bkt[s] << 52) | t.first[s];
    oslot[i] = (uint32_t)s;
  }
}

__global__ void k_word_gather(Table t, const uint32_t* slot, uint32_t W, WordRec* out) {
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < W; r += gridDim.x * blockDim.x) {
    const uint32_t s = slot[r];
    WordRec w;
    w.first = t.first[s];
    w.count = t.cnt[s];
    w.len = t.len[s];
    w.pad = 0;
    out[r] = w;
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

static double wall() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool gpu_count_words(int device, const uint8_t* d, size_t n, std::vector<WordRec>* out, std::string* why) {
  out->clear();
  const bool report = std::getenv("SHREDWORD_LOAD_REPORT") != nullptr;
  const double t0 = wall();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
    if (why) *why = "no HIP device";
    return false;
  }
  if (n == 0) return true;
  if (n >= (1ull << 52)) {
    if (why) *why = "corpus larger than 2^52 bytes";
    return false;
  }
  LOAD_OK(hipSetDevice(device));
  hipStream_t st;
  LOAD_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
  } sg{st};
  hipDeviceProp_t prop;
  LOAD_OK(hipGetDeviceProperties(&prop, device));
  const int cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;

  DevBuf dd;
  LOAD_OK(hipMalloc(&dd.p, n + kPadBytes));
  uint8_t* db = static_cast<uint8_t*>(dd.p);
  LOAD_OK(hipMemsetAsync(db + n, ' ', kPadBytes, st));
  LOAD_OK(hipMemcpyAsync(db, d, n, hipMemcpyHostToDevice, st));
  if (report) LOAD_OK(hipStreamSynchronize(st));
  const double t1 = wall();

  // table capacity: a power of two >= n / 64 (grown while it overflows)
  u64 cap = 1ull << 20;
  while (cap < (u64)(n / 64) && cap < (1ull << 31)) cap <<= 1;
  const u64 nchunks = (n + kChunkBytes - 1) / kChunkBytes;
  const int grid = (int)std::min<u64>((nchunks + kLoadThreads - 1) / kLoadThreads, (u64)cus * 2);
  for (int attempt = 0; attempt < 6; ++attempt) {
    const u64 seed = 0x51ED270B27A1F4A3ull * (u64)(attempt + 1);
    DevBuf bkey, bcnt, bfirst, blen, bbkt, bmeta;
    LOAD_OK(hipMalloc(&bkey.p, cap * 8));
    LOAD_OK(hipMalloc(&bcnt.p, cap * 8));
    LOAD_OK(hipMalloc(&bfirst.p, cap * 8));
    LOAD_OK(hipMalloc(&blen.p, cap * 4));
    LOAD_OK(hipMalloc(&bbkt.p, cap * 4));
    LOAD_OK(hipMalloc(&bmeta.p, 64));
    LOAD_OK(hipMemsetAsync(bkey.p, 0, cap * 8, st));
    LOAD_OK(hipMemsetAsync(bcnt.p, 0, cap * 8, st));
    LOAD_OK(hipMemsetAsync(bfirst.p, 0xFF, cap * 8, st));
    LOAD_OK(hipMemsetAsync(bmeta.p, 0, 64, st));
    Table t;
    t.key = (u64*)bkey.p;
    t.cnt = (u64*)bcnt.p;
    t.first = (u64*)bfirst.p;
    t.len = (uint32_t*)blen.p;
    t.bkt = (uint32_t*)bbkt.p;
    t.mask = cap - 1;
    t.nkeys = (uint32_t*)bmeta.p;
    t.flags = (uint32_t*)bmeta.p + 4;
    k_word_count<<<grid, kLoadThreads, 0, st>>>(db, n, t, seed);
    LOAD_OK(hipGetLastError());
    k_word_verify<<<(int)std::min<u64>((nchunks + kLoadThreads - 1) / kLoadThreads, (u64)cus * 8), kLoadThreads, 0,
                    st>>>(db, n, t, seed);
    LOAD_OK(hipGetLastError());
    uint32_t meta[16];
    LOAD_OK(hipMemcpyAsync(meta, bmeta.p, 64, hipMemcpyDeviceToHost, st));
    LOAD_OK(hipStreamSynchronize(st));
    const double t2 = wall();
    const uint32_t W = meta[0];
    if (meta[4]) {  // too full: a bigger table
      if (cap >= (1ull << 33)) break;
      cap <<= 2;
      continue;
    }
    if (meta[5]) continue;  // a 64-bit key collision: another seed
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
    size_t tmp_bytes = 0;
    LOAD_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, (u64*)bk.p, (u64*)bk2.p, (uint32_t*)bs.p,
                                               (uint32_t*)bs2.p, (int)W, 0, 64, st));
    LOAD_OK(hipMalloc(&btmp.p, tmp_bytes + 16));
    LOAD_OK(hipcub::DeviceRadixSort::SortPairs(btmp.p, tmp_bytes, (u64*)bk.p, (u64*)bk2.p, (uint32_t*)bs.p,
                                               (uint32_t*)bs2.p, (int)W, 0, 64, st));
    LOAD_OK(hipMalloc(&brec.p, (size_t)W * sizeof(WordRec) + sizeof(WordRec)));
    k_word_gather<<<cus * 4, 256, 0, st>>>(t, (const uint32_t*)bs2.p, W, (WordRec*)brec.p);
    LOAD_OK(hipGetLastError());
    out->resize(W);
    if (W) LOAD_OK(hipMemcpyAsync(out->data(), brec.p, (size_t)W * sizeof(WordRec), hipMemcpyDeviceToHost, st));
    LOAD_OK(hipStreamSynchronize(st));
    if (report)
      std::fprintf(stderr, "[LOAD] %zu bytes: upload %.1f ms, count+verify %.1f ms, order+gather %.1f ms, %u words\n", n,
                   1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (wall() - t2), W);
    return true;
  }
  if (why) *why = "the device word table did not converge";
  return false;
}

}  // namespace shred
