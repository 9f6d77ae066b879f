// Shared pieces of the BPE encoder (include/shredword_encode.h): the merge-rank table layout that
// the host builds and the gfx950 kernels probe, and the device half's interface.  No HIP type
// appears here so host C++ can include it; encode_device.hip implements EncodeDevice.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace shred {

// Open-addressing table, one u64 per slot: key (first << 20 | second, 40 bits) << 20 | rank.
// Capacity is a power of two >= 2 x merges (load factor <= 1/2); linear probing from
// enc_slot(key).  Ids outside [0, 2^20) never merge; an empty slot is all ones.
constexpr uint64_t kEncEmpty = ~0ull;
constexpr int32_t kEncIdLimit = 1 << 20;
constexpr int kEncMaxWord = 1024;  // SHRED_ENCODE_MAX_WORD

inline uint64_t enc_key(int32_t a, int32_t b) { return (uint64_t)(uint32_t)a << 20 | (uint64_t)(uint32_t)b; }
inline uint64_t enc_slot(uint64_t key) { return (key * 0x9E3779B97F4A7C15ull) >> 24; }

// Builds the table; the first (lowest-rank) entry of a repeated pair wins, like the replay.
std::vector<uint64_t> enc_build_table(const std::vector<int32_t>& first, const std::vector<int32_t>& second);

class EncodeDevice {
 public:
  // Uploads the table and byte map to `device`; *why says what failed.
  static EncodeDevice* create(int device, const std::vector<uint64_t>& table, const int32_t* byte_map,
                              std::string* why);
  ~EncodeDevice();
  // text / out on the device; stream = hipStream_t or nullptr.  Returns ids, -1 device error,
  // -2 cap too small, -3 word longer than kEncMaxWord.
  int64_t encode(const uint8_t* text, size_t n, int32_t* out, size_t cap, void* stream, double* kernel_ms);
  // Host buffers: staged through cached device buffers in pieces of <= kHostPiece bytes cut at
  // delimiters (device memory ~14 B per piece byte, whatever n is).
  static constexpr size_t kHostPiece = size_t(256) << 20;
  int64_t encode_host(const uint8_t* text, size_t n, int32_t* out, size_t cap);
  // Calls that fell back from the word cache to the direct path (overflow or hash collision).
  uint64_t fallbacks() const { return fallbacks_; }

 private:
  EncodeDevice() = default;
  bool reserve(size_t n, std::string* why);
  bool reserve_host(size_t n);
  int device_ = 0;
  void* stream_ = nullptr;      // hipStream_t
  uint64_t* table_ = nullptr;
  uint64_t mask_ = 0;
  bool packed_ = false;         // 16-bit LDS strips (ids < 0xFFFF)
  int32_t* byte_map_ = nullptr;
  // scratch sized for the largest text seen: ids per word span, rank cache of long words,
  // per-thread counts, per-block counts / offsets, total + error word
  size_t cap_bytes_ = 0;
  int32_t* pad_ = nullptr;
  int32_t* rank_ = nullptr;
  uint32_t* tcnt_ = nullptr;
  uint64_t* bcnt_ = nullptr;    // [0, nb) block counts, [nb, 2 nb) inclusive sums
  void* scan_tmp_ = nullptr;     // hipCUB scan scratch
  size_t scan_tmp_bytes_ = 0;
  uint64_t* misc_ = nullptr;    // [0] total ids, [1] flags: 1 long word, 2 probe window full, 4 collision,
                                // 8 arena full; [2] word-cache arena top
  // word cache (one 16-byte slot per distinct word): 64-bit word hash, payload (an occurrence's
  // offset, then arena offset | length << 32 | id count << 48); the arena is rank_
  size_t ccap_ = 0, ccap_min_ = 0;  // allocated slots; slots a call starts with
  uint64_t* cslot_ = nullptr;
  uint64_t* host_misc_ = nullptr;  // pinned
  // host-path staging
  size_t host_cap_ = 0;
  uint8_t* dtext_ = nullptr;
  int32_t* dout_ = nullptr;
  void* ev_[4] = {nullptr, nullptr, nullptr, nullptr};
  uint64_t fallbacks_ = 0;
};

}  // namespace shred
