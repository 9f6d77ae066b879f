// The indexed merge loop (types layout, one GPU): K2+K3 of SURVEY.md §7.1 driven by an exact
// word index instead of a scan of the whole token table (§8 f3 "tile skipping ... or an
// occurrence index").
//
// Why an index.  A merge of (a, b) only changes the words that hold (a, b).  The reference finds
// them by walking every symbol of every word twice per merge (recompute_freq bpe.cpp:52-65 and
// the merge scan bpe.cpp:265-296); on C3 that is 15 M symbols per merge for ~300 words that
// actually change.  Two facts give an index that costs nothing to extend:
//  * only merge X creates the id X (bpe.cpp:274-290), so every word that ever holds X is one of
//    the words merge X changed: that list ("words of X") is a superset of the holders of X for
//    the rest of the run;
//  * a merge never makes two older ids adjacent (it only puts X next to its neighbours), so a
//    pair of ids that predate the index occurs only where it occurred when the index was built.
// Hence the words of pair (c, d): the shorter words-of list of c and d when either was created by
// the loop, else the initial pair index (every adjacent pair of the table at build time, grouped
// by pair).  Lists may over-approximate (a listed word that no longer holds the pair is scanned
// and left alone), so nothing is ever removed from them.
//
// Device layout, in HBM: one run per word in rank order, 16-B aligned, [live length][tokens ...]
// (capacity = the initial length); a pool of u64 word entries (run offset << 32 | word id); the
// initial pair index as an open-addressing directory pair -> (pool offset, count); per id X the
// words-of list (pool offset, count) and the command that made it.  Merge X scans the words its
// pair lists, emits the reference's four neighbour deltas per occurrence (reduced per
// (neighbour, category) with the minimum first touch, as k_resident/k_merge do), compacts each
// word in place, appends the words it changed to the pool as the words of X, and hands the
// records to the host.  A wrong guess is undone exactly: UNMERGE expands X back into (a, b) in
// the words of X and releases its list.
//
// Execution: one persistent workgroup of 1024 threads (k_word_loop) polls a command ring in
// pinned host memory, so a merge costs a handful of dependent memory round trips instead of a
// fan-out to 256 workgroups and a fan-in.  One workgroup is always co-resident, so the launch
// cannot deadlock on partial residency whatever else holds the GPU.
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
  uint64_t candidates = 0;    // Σ listed words of collected merges
  uint64_t scanned = 0;       //   of which: words whose runs were read (signature hits)
  uint64_t changed = 0;       // Σ words a collected merge changed
  uint64_t occurrences = 0;   // Σ occurrences merged
  uint64_t launches = 0;      // persistent launches
  double kernel_ms = 0;       // Σ launch durations (HIP events)
  double dev_us = 0;          // Σ device time command seen -> flag raised (s_memrealtime)
  double dev_lookup_us = 0;   //   of which: command seen -> word list known
  double dev_scan_us = 0;     //   of which: word list known -> every listed word merged
  double wait_us = 0;         // Σ host time post -> flag seen
  double build_us = 0;        // Σ device time building pair groups (after the flags)
  uint64_t no_sub = 0;        // merges whose pair groups were not built (their words-of list serves)
  uint64_t staged = 0;        // Σ pair-group entries written
  uint64_t run_ints_read = 0;     // Σ ints of the scanned words' runs (length + tokens)
  uint64_t run_ints_written = 0;  // Σ ints of the changed words' runs written back
  uint64_t records = 0;           // Σ delta records handed to the host
  uint64_t raw_records = 0;       // Σ delta records of the merges (before the device's combine)
  uint64_t finalized = 0;         // merges whose records left as ordered changes
  double dev_rel_us = 0;          // Σ device time of the flags' system release (L2 write-back), diagnostic
  double dev_out_us = 0;          // Σ device time handing the records out (raw, or gathered + finalized)
  double dev_fin_us = 0;          //   of which: the merges whose records were finalized
  uint64_t fin_records = 0;       //   their raw records
  uint64_t spill_merges = 0;      // merges whose delta keys overflowed the LDS hash (HBM spill tables)
  uint64_t spill_keys = 0;        // Σ their spilled keys
};

struct SelectStats {
  uint64_t merges = 0, launches = 0, rebuilds = 0;
  double kernel_ms = 0, rebuild_ms = 0;  // launches of k_word_loop<true>; frontier rebuilds (host wall)
  double select_us = 0, merge_us = 0;    // device time: selecting, merging + table update (s_memrealtime)
  double table_us = 0;                   // of merge_us: the pair table + frontier update
  double rec_us = 0, append_us = 0, tail_us = 0;  // of table_us: records, appends, compaction + bookkeeping
  double log_ms = 0;                     // the table-change logs applied between launches (host wall)
  uint64_t log_entries = 0;
  uint64_t listed = 0, changed = 0, occurrences = 0, new_pairs = 0;
  uint64_t table_slots = 0, table_pairs = 0, frontier_max = 0;
  uint64_t grows = 0;  // pair tables grown 4x (past 3/4 full) between launches
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
  // The current words from the device tile stream of the same table (tok, tile_off, tile_len in
  // device memory; the tile path merged them), then re-indexed: all on the device.
  void load_tiles(const int32_t* tok, const uint64_t* tile_off, const uint32_t* tile_len);
  // Back to the uploaded words without restoring the initial index (a load_tiles follows).
  void reset_words();
  // Delta slots and id tables for ids <= max_id (stops the launch if they must grow).
  void reserve(int32_t max_id);

  // Queues merge (a, b) -> X (the persistent launch starts on the first post).
  void post_merge(int32_t a, int32_t b, int32_t X);
  // The records of the oldest posted merge, which must be X (waits for its flag).  When
  // last_changes() is true afterwards they are Selector::Change entries instead (K4 on the device:
  // combined per pair key, in the reference's application order; word_loop.hip finalize_changes).
  size_t collect(int32_t X, const DeltaRecord** recs);
  bool last_changes() const { return last_changes_; }
  // K4 on the device for merges of at most n records (0: off; SHREDWORD_WL_FINALIZE overrides).
  void set_finalize(uint32_t n) { fin_max_ = n; }
  uint32_t finalize_max() const { return fin_max_; }
  // Non-blocking: X is the oldest posted merge and its flag is up (records as collect() gives them).
  bool peek(int32_t X, const DeltaRecord** recs, size_t* n) const;
  // Undoes every posted merge with id >= X, newest first (queued; nothing waits).
  void rollback(int32_t X);
  size_t in_flight() const { return posted_.size(); }
  uint32_t id_room() const { return cap_; }  // merges may post ids X with X + 2 <= id_room()
  // tiebreak=device: merges X0 .. X0 + n_max - 1 selected and applied on the device, with no
  // host round trip per merge (k_word_loop<true>).  `pairs`: the current words' pair counts (K1,
  // pairs holding unk excluded).  Each merge takes the pair of largest count, ties to the smaller
  // key ((u32)a << 32 | (u32)b), while that count is >= min_freq.  Returns the merges done (out:
  // in order), or -1 when the loop is not usable.  The words are merged in place as by post_merge.
  int run_select(const std::vector<PairCount>& pairs, int32_t X0, uint32_t n_max, uint64_t min_freq,
                 std::vector<SelectedMerge>* out);
  const SelectStats& select_stats() const { return sst_; }
  // Ends the persistent launch (nothing may be in flight).
  void stop();
  bool running() const { return running_; }
  // Later work goes to this stream (nothing may be in flight).
  void set_stream(void* s) {
    if (running_) stop();
    stream_ = s;
  }

  // Writes the current words back into the tile stream (headers + tokens, tile_len), so the tile
  // kernels (K1, K6, downloads) see the merged table.  No-op when nothing changed since.
  void sync_tiles(int32_t* tok, const uint64_t* tile_off, uint32_t* tile_len);
  bool tiles_dirty() const { return dirty_; }
  void mark_tiles_current() { dirty_ = false; }

  const WordLoopStats& stats() const { return st_; }
  void clear_stats() {
    st_ = WordLoopStats();
    const uint64_t slots = sst_.table_slots;
    sst_ = SelectStats();
    sst_.table_slots = slots;
    trace_.clear();
  }
  // Per collected merge while timing is on, kTraceFields u32 each: X, listed words, scanned
  // words, changed words, occurrences, device ns command -> flag, of which lookup ns, scan ns;
  // then thread 0's stamps (ns after the command): pool entries loaded, first run loaded, first
  // word merged; and the delta keys spilled past the LDS hash to HBM; then the device ns
  // outside merges since the previous merge's flag (waiting for commands; undoing guesses), and
  // the host ns from posting this merge to seeing its flag; then absolute clocks: host post and
  // flag seen (10 ns since the loop was made), device command seen and wait begun (100 MHz
  // ticks), low 32 bits each.
  static constexpr int kTraceFields = 37;
  const std::vector<uint32_t>& trace() const { return trace_; }
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
  void launch(uint32_t seq0);  // the first command the launch takes
  void recover_timeout();
  // Writes one command; (loff, lcnt1): the words-of list of max(a, b) if known (count + 1; 0: none).
  uint32_t post(uint32_t op, int32_t a, int32_t b, int32_t X, uint32_t loff = 0, uint32_t lcnt1 = 0);
  void wait_flag(const Slot& s, uint32_t seq);
  bool handed_over(const Slot& s, uint32_t seq) const;  // the small-merge path's checksummed hand-off
  void ensure_slots(uint32_t cap);

  int ordinal_ = 0;
  void* stream_ = nullptr;
  int32_t unk_ = 0;
  bool ready_ = false, running_ = false, dirty_ = false, timing_ = false;
  // per id: the words-of list a collected merge wrote (offset | (count + 1) << 32; 0: none) --
  // exactly the device's lst[] for confirmed merges, so a merge's command carries its list
  std::vector<uint64_t> lists_;
  double t_epoch_ = now_seconds();  // the trace's host clock origin

  uint32_t nwords_ = 0;
  uint64_t nint_ = 0;          // int32 elements of the word runs (lengths + tokens + padding)
  uint64_t ntok_ = 0;          // Σ initial word lengths
  uint32_t ntiles_ = 0;
  int32_t* wtok_ = nullptr;    // word w: run at woff[w] (16-B aligned) = [live length][tokens]
  int32_t* wtok0_ = nullptr;   // pristine copy
  uint32_t* woff_ = nullptr;   // W + 1
  std::vector<uint32_t> woff_h_;
  const unsigned long long* weight_ = nullptr;
  uint32_t* tile_first_ = nullptr;  // per tile: first word, count (sync_tiles)
  uint32_t* tile_nw_ = nullptr;
  // index
  unsigned long long* pool_ = nullptr;   // word entries {run offset << 32 | word id, id signature}
  uint64_t pool_cap_ = 0;
  unsigned long long* dkey_ = nullptr;   // initial pair directory: pair key (EMPTY = ~0)
  unsigned long long* dval_ = nullptr;   //   pool offset | count << 32
  uint64_t dir_cap_ = 0;
  unsigned long long* init_key_ = nullptr;   // the initial index as sorted runs (restore on reset)
  unsigned long long* init_val_ = nullptr;
  uint64_t init_keys_n_ = 0;
  uint64_t init_pool_n_ = 0;
  unsigned long long* lst_ = nullptr;    // per id: words-of list, pool offset | count << 32
  uint32_t* lseq_ = nullptr;             // per id: the command that made the list (~0: none)
  uint32_t id_cap_ = 0;
  unsigned long long* dsum_ = nullptr;   // delta spill tables (keys past the LDS hash), 4 x (cap + 1)
  unsigned long long* dft_ = nullptr;
  uint32_t* dlist_ = nullptr;
  uint32_t* dstate_ = nullptr;     // [0] spill count, [1] pool top, [2] sub top, [3] error, [4..7] stats
  uint32_t cap_ = 0;               // delta slots: ids < cap_ have slot id + 1

  Slot slot_[kSlots];
  void* ring_ = nullptr;           // pinned command ring
  void* ring_dev_ = nullptr;
  uint32_t* status_ = nullptr;     // pinned: [0] exit reason, [1] error code
  void* status_dev_ = nullptr;
  uint32_t seq_ = 0;
  uint32_t idle_polls_ = 1u << 22;  // ~10 s without a command: the launch ends itself (relaunched on demand)
  bool sel_report_ = false;         // SHREDWORD_SELECT_REPORT=1: one stderr line per k_word_loop<true> launch
  // K4 on the device up to this many records (<= 64: one wave; up to kFinMax: the workgroup).  Off
  // by default: measured on C3 it costs the device more than it saves the host
  uint32_t fin_max_ = 0;
  // SHREDWORD_WL_FIN_MIN: K4 only for merges of at least this many records (the large ones; the
  // small-merge path then stays on for the rest)
  uint32_t fin_min_ = 0;
  // the next command read while the records go out (SHREDWORD_WL_PREFETCH=0 turns it off): C3 A/B
  // on one box, 2 rounds: 54.2-54.3 k off, 55.0-55.2 k on (profiles/r05_c3_command_prefetch_ab.txt)
  bool prefetch_ = true;
  // SHREDWORD_WL_DRAIN=1: every merge barrier drains the stores (the round-4 barriers)
  bool drain_ = false;
  // SHREDWORD_WL_PROBES=0 / 1 (tests): the kernel instance whose LDS delta hash spills every key /
  // most keys to the HBM tables (a template argument: the default kernel pays nothing for it)
  int probes_ = 32;
  // the small-merge path for merges listing <= 512 words (SHREDWORD_WL_FAST=0: the queued path only)
  bool fast_ = true;
  bool last_changes_ = false;
  std::vector<Post> posted_;
  // tiebreak=device: pair table, frontier, state (see word_loop.hip SelParams)
  void sel_free();
  bool sel_rebuild(uint64_t min_freq);  // false: no pair at or above min_freq is left
  unsigned long long* ptab_ = nullptr;  // tiebreak=device pair table: 16-B slots (key, count | pos)
  uint64_t pcap_ = 0;
  uint32_t* fr_[2] = {nullptr, nullptr};
  uint32_t fcap_ = 0;
  uint32_t* sst_dev_ = nullptr;
  unsigned long long* thr_ = nullptr;
  unsigned long long* sout_ = nullptr;
  uint64_t sout_cap_ = 0;
  uint32_t* upd_ = nullptr;
  uint64_t upd_cap_ = 0;
  uint32_t* shist_ = nullptr;
  uint32_t* scol_ = nullptr;
  uint64_t scol_cap_ = 0;
  SelectStats sst_;
  void* ev_[2] = {};
  WordLoopStats st_;
  std::vector<uint32_t> trace_;
  size_t bytes_ = 0;
};

}  // namespace shred
