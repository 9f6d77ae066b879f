// Shared constants and helpers of the shredword MI355X BPE trainer (host side).
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace shred {

constexpr int32_t kBaseVocab = 256;          // reference bpe.h:20 INITIAL_VOCAB_SIZE
constexpr uint64_t kDefaultMinPairFreq = 2000;  // reference bpe.h:23 MIN_PAIR_FREQ
constexpr int kPairBuckets = 4096;           // reference bpe.cpp:183 bimap_init(MIN_HEAP_SIZE)
constexpr int kDeltaBuckets = 1024;          // reference bpe.cpp:16 FREQ_CHANGE_BUCKETS

// In-band word header of the device token stream: header(rank) = INT32_MIN + rank.  Real ids
// are >= -2^30 (unk_id must be >= kMinUnkId), so any value below kHeaderLimit is a header.
constexpr int32_t kHeaderBase = INT32_MIN;
constexpr int32_t kHeaderLimit = -(1 << 30);
constexpr int32_t kMinUnkId = -(1 << 30);
constexpr uint32_t kMaxRank = (1u << 30) - 1;

inline double now_seconds() {
  using clk = std::chrono::steady_clock;
  return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
}

[[noreturn]] inline void fatal(const char* what) {
  std::fprintf(stderr, "[ERROR]\t %s\n", what);
  std::fflush(stderr);
  std::exit(EXIT_FAILURE);
}

// FNV-1a 32 over the little-endian bytes of (first, second): reference hash.cpp:7-16.
inline uint32_t pair_fnv(int32_t a, int32_t b) {
  uint32_t h = 2166136261u;
  uint32_t ua = (uint32_t)a, ub = (uint32_t)b;
  for (int i = 0; i < 4; ++i) { h ^= (ua >> (8 * i)) & 0xFF; h *= 16777619u; }
  for (int i = 0; i < 4; ++i) { h ^= (ub >> (8 * i)) & 0xFF; h *= 16777619u; }
  return h;
}

inline uint64_t pack_pair(int32_t a, int32_t b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }
inline int32_t pair_first(uint64_t k) { return (int32_t)(uint32_t)(k >> 32); }
inline int32_t pair_second(uint64_t k) { return (int32_t)(uint32_t)k; }

}  // namespace shred
