// The indexed merge loop (types layout, one GPU): K2+K3 of SURVEY.md §7.1 driven by an exact
// pair -> words occurrence index instead of a scan of the whole token table (§8 f3 "tile
// skipping ... or an occurrence index").
//
// Why an index.  A merge of (a, b) only changes the words that hold (a, b).  The reference finds
// them by walking every symbol of every word twice per merge (recompute_freq bpe.cpp:52-65 and
// the merge scan bpe.cpp:265-296); on C3 that is 15 M symbols per merge for ~280 words that
// actually change.  Two facts make an exact index cheap to keep:
//  * a merge creates adjacencies only next to its new id X: (p, X) and (X, n) (bpe.cpp:274-290),
//    so the words holding a pair (c, d) are all listed either by the initial index (every pair of
//    the table when the index was built) or by the one merge that created max(c, d);
//  * lists may over-approximate (a listed word that no longer holds the pair is scanned and left
//    alone), so nothing is ever removed from them.
// The device therefore holds, in HBM: the table as one int32 run per word (rank order, capacity =
// initial length, live length beside it), a pool of word ids, and an open-addressing directory
// pair -> (pool offset, count, creating command).  Merge X scans only the words its pair lists,
// emits the reference's four neighbour deltas per occurrence (reduced per (neighbour, category)
// with the minimum first touch, exactly as k_resident/k_merge do), compacts each word in place,
// hands the records to the host, and then appends the words of every new pair (p, X) / (X, n) to
// the pool under a directory entry of its own.
//
// Execution: one persistent workgroup of 1024 threads (k_word_loop) polls a command ring in
// pinned host memory, so a merge costs a handful of dependent memory round trips instead of a
// fan-out to 256 workgroups and a fan-in.  One workgroup is always co-resident, so the launch
// cannot deadlock on partial residency whatever else holds the GPU.  Speculative guesses are
// undone exactly (UNMERGE expands X back into (a, b) in the words of (a, b)'s list; the guess's
// directory entries are invalidated by its command number).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "selector.h"
#include "tiles.h"

namespace shred {

struct WordLoopStats {
  uint64_t merges = 0;        // merges collected
  uint64_t undos = 0;         // guesses undone
  uint64_t candidates = 0;    // Σ listed words scanned by collected merges
  uint64_t changed = 0;       // Σ words a collected merge changed
  uint64_t occurrences = 0;   // Σ occurrences merged
  uint64_t launches = 0;      // persistent launches
  double kernel_ms = 0;       // Σ launch durations (HIP events)
  double dev_us = 0;          // Σ device time command seen -> flag raised (s_memrealtime)
  double wait_us = 0;         // Σ host time post -> flag seen
  uint64_t build_rounds = 0;  // index build rounds (> merges when a merge had > 2048 new pairs)
};

class WordLoop {
 public:
  static constexpr int kSlots = 4;  // merges in flight: the current one and up to 3 guesses

  WordLoop(int ordinal, void* stream, int32_t unk_id);
  ~WordLoop();
  WordLoop(const WordLoop&) = delete;
  WordLoop& operator=(const WordLoop&) = delete;

  // Builds the per-word table of a types-layout tile stream (entries = words in rank order),
  // uploads it with a pristine copy, and builds the index of its pairs.  d_weight: the device's
  // u64 weight per rank.  False when the table does not suit the loop (it then stays unused).
  bool upload(const TiledStream& ts, const uint64_t* d_weight);
  bool ready() const { return ready_; }
  // Back to the uploaded table and its initial index.
  void reset();
  // Replaces the current words (not the pristine copy) by a tile stream of the same table whose
  // words were merged elsewhere (the tile path), and re-indexes them.  False if it does not fit.
  bool load_current(const TiledStream& ts);
  // Re-indexes the current words (the initial index then describes them).
  void rebuild() { build_index(); }
  // Delta slots and id tables for ids <= max_id (stops the launch if they must grow).
  void reserve(int32_t max_id);

  // Queues merge (a, b) -> X (the persistent launch starts on the first post).
  void post_merge(int32_t a, int32_t b, int32_t X);
  // The records of the oldest posted merge, which must be X (waits for its flag).
  size_t collect(int32_t X, const DeltaRecord** recs);
  // Undoes every posted merge with id >= X, newest first (queued; nothing waits).
  void rollback(int32_t X);
  size_t in_flight() const { return posted_.size(); }
  // Ends the persistent launch (nothing may be in flight).
  void stop();
  bool running() const { return running_; }

  // Writes the current words back into the tile stream (headers + tokens, tile_len), so the tile
  // kernels (K1, K6, downloads) see the merged table.  No-op when nothing changed since.
  void sync_tiles(int32_t* tok, const uint64_t* tile_off, uint32_t* tile_len);
  bool tiles_dirty() const { return dirty_; }
  void mark_tiles_current() { dirty_ = false; }

  const WordLoopStats& stats() const { return st_; }
  void clear_stats() { st_ = WordLoopStats(); }
  void set_timing(bool on) { timing_ = on; }
  size_t device_bytes() const { return bytes_; }
  uint32_t words() const { return nwords_; }
  uint64_t initial_keys() const { return init_keys_n_; }
  uint64_t pool_used() const;  // diagnostic (stops nothing; reads the device counter)

 private:
  struct Slot {
    DeltaRecord* host_recs = nullptr;  // pinned, device-visible
    void* dev_recs = nullptr;
    uint32_t* host_hdr = nullptr;      // pinned: [0] records, [1] flag = command seq, [2..] stats
    void* dev_hdr = nullptr;
    uint32_t rec_cap = 0;
  };
  struct Post {
    int32_t X, a, b;
    uint32_t seq;
    double t_post;
  };
  void free_all();
  void build_index();
  void restore_index();
  void launch();
  uint32_t post(uint32_t op, int32_t a, int32_t b, int32_t X);
  void wait_flag(const Slot& s, uint32_t seq);
  void ensure_slots(uint32_t cap);

  int ordinal_ = 0;
  void* stream_ = nullptr;
  int32_t unk_ = 0;
  bool ready_ = false, running_ = false, dirty_ = false, timing_ = false;

  uint32_t nwords_ = 0;
  uint64_t nsym_ = 0;          // Σ word capacities
  uint32_t ntiles_ = 0;
  int32_t* wtok_ = nullptr;    // tokens, word w at [woff[w], woff[w] + wcap)
  int32_t* wtok0_ = nullptr;   // pristine copy
  uint32_t* woff_ = nullptr;   // W + 1
  std::vector<uint32_t> woff_h_;
  uint32_t* wlen_ = nullptr;   // live length
  uint32_t* wlen0_ = nullptr;
  uint32_t* wmark_ = nullptr;  // last command that claimed the word (duplicate list entries)
  const unsigned long long* weight_ = nullptr;
  uint32_t* tile_first_ = nullptr;  // per tile: first word, count (sync_tiles)
  uint32_t* tile_nw_ = nullptr;
  // index
  uint32_t* pool_ = nullptr;
  uint64_t pool_cap_ = 0;
  unsigned long long* dkey_ = nullptr;   // directory: pair key (EMPTY = ~0)
  unsigned long long* dval_ = nullptr;   //            pool offset | count << 32
  uint32_t* dseq_ = nullptr;   //            creating command (0 = initial index)
  uint64_t dir_cap_ = 0;
  unsigned long long* init_key_ = nullptr;   // the initial index as sorted runs (restore on reset)
  unsigned long long* init_val_ = nullptr;
  uint64_t init_keys_n_ = 0;
  uint64_t init_pool_n_ = 0;
  uint32_t* valid_seq_ = nullptr;  // per id: the command whose directory entries are valid
  uint32_t id_cap_ = 0;
  unsigned long long* stage_key_[2] = {};    // per merge: new pairs (key, word), and the deferred round
  uint32_t* stage_w_[2] = {};
  uint32_t* stage_slot_ = nullptr;
  uint64_t stage_cap_ = 0;
  unsigned long long* dsum_ = nullptr;       // delta spill tables (keys past the LDS hash), 4 x (cap + 1)
  unsigned long long* dft_ = nullptr;
  uint32_t* dlist_ = nullptr;
  uint32_t* dstate_ = nullptr;     // [0] spill count, [1] pool top, [2] directory keys, [3] error
  uint32_t cap_ = 0;               // delta slots: ids < cap_ have slot id + 1

  Slot slot_[kSlots];
  void* ring_ = nullptr;           // pinned command ring
  void* ring_dev_ = nullptr;
  uint32_t* status_ = nullptr;     // pinned: [0] exit reason, [1] error code
  void* status_dev_ = nullptr;
  uint32_t seq_ = 0;
  std::vector<Post> posted_;
  void* ev_[2] = {};
  WordLoopStats st_;
  size_t bytes_ = 0;
};

}  // namespace shred
