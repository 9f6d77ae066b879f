// Corpus loading for the BPE path: raw text -> reference-ordered table of distinct words.
//
// Semantics follow the reference bpe_load_corpus (shredword/csrc/bpe/bpe.cpp:110-185) exactly
// (SURVEY.md Appendix A.1-A.2):
//  * the file is read with fgets into a buffer that starts at 4096 bytes and doubles, and each
//    buffer is cut at its first NUL (strlen) before strtok on "\t\r\n " (bpe.cpp:131-153);
//  * distinct words are ordered by (djb2(word) & 4095, first occurrence) — the iteration order
//    of the reference's fixed 4096-bucket StrMap (hash.cpp:29-72);
//  * the byte histogram counts each distinct word's bytes once (histogram.cpp:30-36), candidates
//    are taken in StrMap(256) order ((c + 165) & 255), stable-sorted by count descending, and the
//    first (size_t)((float)n * coverage) bytes are kept; other bytes map to unk_id.
// The implementation is parallel (thread-local hash maps merged by hash partition); the result
// does not depend on the thread count.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace shred {

struct WordTable {
  // Distinct words in reference word order ("rank" order).
  std::vector<uint8_t> bytes;    // concatenated spellings
  std::vector<uint64_t> offset;  // size W+1: word w occupies bytes/symbols [offset[w], offset[w+1])
  std::vector<uint64_t> count;   // occurrences of each word
  std::vector<int32_t> symbols;  // initial symbol ids (byte value or unk_id), same offsets as bytes
  uint64_t total_occurrences = 0;
  size_t distinct_bytes = 0;     // `c` of bpe.cpp:165
  size_t kept_bytes = 0;         // `keep` of bpe.cpp:169
  bool keep[256] = {};
  // Stream layout (optional): the type rank of every word occurrence, in corpus order.
  std::vector<uint32_t> occurrence_rank;
  bool counted_on_gpu = false;   // the distinct words were counted on the device (load_device.hip)

  size_t num_words() const { return count.size(); }
  size_t num_symbols() const { return symbols.size(); }
};

// All-gather of a byte buffer across the ranks of a sharded load: returns every rank's buffer,
// concatenated in rank order (*out_bytes = total), valid until the next call.
typedef const void* (*LoadGather)(void* ctx, const void* send, size_t nbytes, size_t* out_bytes);

struct LoadOptions {
  int32_t unk_id = 0;
  float coverage = 0.995f;
  bool want_stream = false;  // also fill occurrence_rank
  int threads = 0;           // 0: hardware concurrency (capped at 32)
  int gpu_device = -1;       // >= 0: count words on this HIP device (types layout, NUL-free files)
  size_t gpu_min_bytes = 1 << 20;  // smaller files take the host path
  // Sharded load (types layout, NUL-free files; SURVEY.md §8 f2 multi-GPU): rank r of `world`
  // counts the words starting in its byte range only (on its GPU, or the host path); the ranks'
  // distinct-word lists are all-gathered and merged (counts summed, first occurrence min,
  // spellings compared byte for byte), so every rank builds the identical, full table.
  int shard_rank = 0, shard_world = 1;
  LoadGather gather = nullptr;
  void* gather_ctx = nullptr;
};

// One distinct word found by the device count: its first offset in the file, its occurrence
// count and its length (hip/load_device.hip).
struct WordRec {
  uint64_t first;
  uint64_t count;
  uint32_t len;
  uint32_t pad;
};

// GPU word count: the distinct words of d[0, n) in reference word order
// (djb2(word) & 4095, first occurrence).  d must not contain NUL bytes (those files keep the
// host's fgets/strlen path).  False (reason in *why) when no device is usable.
// staged: d is a range inside a larger mapping (a sharded load): uploaded through pinned buffers.
bool gpu_count_words(int device, const uint8_t* d, size_t n, std::vector<WordRec>* out, std::string* why,
                     bool staged = false);

// The same count read straight from an open file (no mapping): reader threads pread() into
// pinned buffers and DMA each chunk to HBM; the device also gathers the spellings in rank order
// (*spell: the word table's byte array).  *nul: the file holds a NUL byte (false is returned; the
// caller takes the host's fgets/strlen path).
// [base, base + n) of the file (a sharded load's byte range): records carry file offsets.
bool gpu_count_file(int device, int fd, uint64_t base, size_t n, std::vector<WordRec>* out,
                    std::vector<uint8_t>* spell, bool* nul, std::string* why);

// Returns 0 on success, -1 if the file cannot be opened/mapped (message in *err).
int load_corpus(const char* path, const LoadOptions& opt, WordTable* out, std::string* err);

// Builds a WordTable from in-memory text (same rules); used by tests and tools.
// 0, or -1 with *err set (a sharded load whose word-list all-gather failed).
// fd >= 0: the same bytes as an open file (the device count of a sharded load reads its range
// from it instead of the mapping).
int load_corpus_bytes(const uint8_t* data, size_t n, const LoadOptions& opt, WordTable* out, std::string* err = nullptr,
                      int fd = -1);

}  // namespace shred
