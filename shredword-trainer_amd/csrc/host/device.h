// HBM-resident state and kernel launches of the BPE merge loop on one MI355X (gfx950).
//
// Layout in HBM (see DESIGN.md "Data layout"):
//   tok       int32 token stream, cut into tiles of whole words (<= 4096 tokens, or one word
//             that is longer); every word is preceded by an in-band header INT32_MIN + rank.
//   tile_off  u64 element offset of each tile (16-byte aligned), tile_len u32 live length.
//   weight    u64 occurrence count per word rank ("types" layout; the "stream" layout keeps
//             every occurrence with weight 1 and needs no weight array).
//   dsum/dft  u64 per (neighbour slot, category): summed weight and min first-touch of the
//             current merge's neighbour-pair deltas; dlist/dcount: the touched keys.  Two sets
//             (merge parity), so a speculative merge X+1 can run while merge X is consumed.
// No HIP type appears here so host C++ can include it; bpe_device.hip implements it.
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstdint>
#include <string>
#include <vector>

#include "corpus.h"
#include "engine.h"
#include "selector.h"
#include "tiles.h"
#include "word_loop.h"

namespace shred {

struct KernelTimes {
  double merge_ms = 0;   // Σ k_merge durations (HIP events on the trainer stream)
  double compact_ms = 0; // Σ k_compact_deltas durations
  double count_ms = 0;   // Σ k_pair_count durations
  uint64_t merge_launches = 0;
  uint64_t count_launches = 0;
  double merge_bytes = 0;  // Σ algorithmic bytes of k_merge launches (4 B per live token read)
  double count_bytes = 0;  // Σ algorithmic bytes of k_pair_count (tokens + boundaries + weights)
  double hist_ms = 0;      // Σ k_pair_hist durations (stream layout K1 bulk: counts only)
  double hist_bytes = 0;   // Σ its algorithmic bytes (4 B per token + 12 B per tile)
  uint64_t hist_launches = 0;
  uint64_t res_merges = 0;  // merges collected from k_resident
  double res_bytes = 0;     // their algorithmic bytes: 4 B per live token per merge
  double res_k3_bytes = 0;  // K3: 4 B read + 4 B written per token of the tiles a merge rewrote
  double res_ms = 0;        // Σ durations of the k_resident launches that merged (HIP events)
};

class Device : public Backend {
 public:
  // True when a HIP device is usable; otherwise *why says what is missing.
  static bool available(std::string* why);
  // Achievable HBM bandwidth on `ordinal` (streaming read and copy of `bytes`, `reps` timed
  // launches each, HIP events); GB/s of bytes moved.  0, or -1 without a device.
  static int hbm_probe(int ordinal, size_t bytes, int reps, double* read_gbps, double* copy_gbps);
  // Diagnostic: fills every wave slot of all CUs but `free_cus` with a spinning kernel on its own
  // stream (returns once it runs) until release() or max_seconds; tests the resident loop's
  // co-residency check.
  static void* occupy(int ordinal, int free_cus, double max_seconds);
  static void release(void* handle);

  explicit Device(int device_ordinal);
  ~Device();
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;

  // Uploads a packed tile stream (types: one entry per distinct word, weights = counts; stream:
  // one entry per occurrence, weight 1) and keeps a pristine copy for reset_tokens().
  void upload(const TiledStream& ts, Layout layout, const std::vector<uint64_t>& weights, int32_t max_id);
  // Restores the token stream to its uploaded (unmerged) state.
  void reset_tokens();
  bool has_tokens() const { return ntiles_ > 0 || uploaded_; }

  // K1: weighted pair histogram with first touch, pairs holding unk skipped (bpe.cpp:187-206);
  // under RCCL the per-rank lists are merged (sum, min first touch).
  void count_pairs(int32_t unk_id, std::vector<PairCount>* out) override;
  // K5 check (debug): K1 again, reduced on the device (k_pair_max) to the largest pair count and
  // (a, b)'s count.
  void pair_max(int32_t unk_id, int32_t a, int32_t b, uint64_t* max_freq, uint64_t* ab_freq) override;

  // K2+K3 for a chain of merges (ab[2i], ab[2i+1]) -> X0 + i: one k_merge launch applies them in
  // order per tile and reduces each merge's neighbour deltas separately.
  void merge_chain(const int32_t* ab, int n, int32_t X0) override;
  // tiebreak=device on the indexed loop (WordLoop::run_select).
  int device_select(const std::vector<PairCount>& pairs, int32_t X0, int n, uint64_t min_freq,
                    std::vector<SelectedMerge>* out) override;
  // The early merges run on the whole-chip resident loop (host-selected) until the hybrid switch.
  bool device_select_now() const override { return !hybrid_resident_phase() || switch_pending_; }
  // Multi-GPU: every launch's compacted records are all-gathered (fixed buckets of
  // `bucket_records` records per rank, RCCL over xGMI, queued behind k_merge on the stream);
  // collect() then returns the concatenation of all ranks' records, which the host combines
  // (sum of weights, min first touch) exactly like one rank's duplicate records.
  struct Exchange {
    int rank = 0, world = 1;
    void* comm = nullptr;
    // in-place-free all-gather of `bytes` per rank from send into recv (world x bytes)
    void (*allgather)(void* comm, const void* send, void* recv, size_t bytes, void* stream) = nullptr;
    uint32_t bucket_records = 1024;
  };
  void set_exchange(const Exchange& x);
  // K4: merge X's records (host memory); the first collect of a chain waits for the launch.
  size_t collect(int32_t X, const DeltaRecord** recs) override;
  bool records_are_changes() const override { return last_changes_; }
  // The indexed loop's finished merge X, without collecting it (Engine's apply helper).
  bool peek(int32_t X, const DeltaRecord** recs, size_t* n) override;
  static constexpr int kChainMax = 8;
  int max_chain() const override {
    return speculate_ && !resident_eligible() && !index_eligible() ? kChainMax : 1;
  }
  bool index_id_room(int32_t max_id) const;
  bool can_overlap() const override {
    if (switch_pending_) return false;  // drain the resident loop: the indexed loop takes over
    // the indexed loop's delta slots grow only with nothing in flight: no guess runs past them
    // (the next merge is then posted alone, and reserves room first)
    if (index_eligible()) return speculate_ && index_id_room(max_id_seen_ + 1 + spec_depth_);
    return speculate_ && (!resident_eligible() || (uint32_t)max_id_seen_ + 3 < min_slot_cap());
  }
  // k_resident takes up to kResSlots merges in flight (the current one and the guesses behind
  // it); the launch path two launches.
  static constexpr int kResSlots = 4;
  int overlap_depth() const override { return resident_eligible() || index_eligible() ? spec_depth_ : 1; }
  // k_resident and the indexed loop queue up to kResSlots / WordLoop::kSlots merges; the launch
  // path's two launches hold one guess behind the current merge.
  int max_guesses() const override { return resident_eligible() || index_eligible() ? kResSlots - 1 : 1; }
  void set_spec_depth(int d) { spec_depth_ = std::max(1, std::min(d, kResSlots - 1)); }
  uint32_t min_slot_cap() const {
    uint32_t c = UINT32_MAX;
    for (const MergeSlot& s : slot_) c = std::min(c, s.cap);
    return c;
  }
  void reserve_ids(int32_t max_id) override;
  uint64_t exchange_overflows() const { return x_overflows_; }
  // Undoes the chain's uncollected merges >= X with k_unmerge (newest first), host-free.
  void rollback(int32_t X) override;
  // LDS-resident merge loop (k_resident): when the types table fits the chip's LDS, single
  // merges run in one persistent launch that holds the table in LDS; quiesce() ends it and
  // leaves the HBM stream current.  Results are identical with it on or off.
  void quiesce() override { park(); }
  void park();
  void set_resident(bool on);
  bool resident() const { return resident_on_; }
  bool resident_eligible() const { return resident_on_ && resident_ok_ && !exchange_ && !index_eligible(); }
  // The indexed merge loop (word_loop.h): the default for the types layout on one GPU.
  void set_index(bool on);
  bool index_on() const { return index_on_; }
  // Hybrid: the first merges (each changes many words) run on k_resident, which spreads a merge
  // over every CU; once kSwitchWindow merges in a row changed fewer than switch_occ_ table
  // entries each, the indexed loop (one workgroup, a few round trips per merge) takes over for
  // the rest of train().
  bool hybrid_resident_phase() const {
    return hybrid_ && !idx_phase_ && resident_on_ && resident_ok_ && !exchange_ && ntiles_ > 0;
  }
  bool index_eligible() const {
    return index_on_ && wl_ && wl_->ready() && !exchange_ && !hybrid_resident_phase();
  }
  void set_hybrid(bool on) {
    park();
    hybrid_ = on;
  }
  void set_switch_occurrences(uint64_t n) { switch_occ_ = n; }
  // The indexed loop's K4 on the device for merges of at most n records (0: off; -1 leaves the
  // loop's default); takes effect at the loop's next launch.
  void set_finalize(int64_t n) {
    fin_ = n;
    if (wl_ && n >= 0) {
      index_sync();
      wl_->set_finalize((uint32_t)n);
    }
  }
  int64_t switch_merge() const { return switch_x_; }
  double switch_ms() const { return switch_ms_; }
  const WordLoop* word_loop() const { return wl_; }
  uint64_t resident_launches() const { return res_launches_; }
  uint64_t resident_aborts() const { return res_aborts_; }
  bool resident_tokens_in_lds() const { return res_lds_tok_; }
  double resident_ms() const { return res_ms_; }
  // mean dispatch -> host flag time of a resident merge (device clock), us
  double resident_latency_us() const { return res_lat_n_ ? res_lat_us_ / (double)res_lat_n_ : 0.0; }
  void set_speculation(bool on) { speculate_ = on; }
  uint64_t rollbacks() const { return rollbacks_; }
  // Tuning: k_merge grid cap.
  void set_merge_groups(int groups);

  // K6: final weighted token histogram over ids [0, T); other ids are dropped.
  void token_freq(size_t T, std::vector<uint64_t>* freq) override;
  // Copies the live token stream back (tests): per entry, header then tokens.
  void download_tokens(std::vector<int32_t>* out);

  void set_timing(bool on) {
    timing_ = on;
    if (wl_) wl_->set_timing(on);
  }
  const KernelTimes& times() {
    flush_timing(true);
    return times_;
  }
  void set_unk(int32_t unk) { unk_ = unk; }
  uint64_t records_total() const { return records_total_; }
  uint64_t visited_tiles() const { return visited_tiles_; }
  uint64_t records_max() const { return records_max_; }
  void clear_times() {
    flush_timing(true);
    times_ = KernelTimes();
    records_total_ = records_max_ = 0;
    visited_tiles_ = 0;
    res_launches_ = 0;
    res_ms_ = res_lat_us_ = 0;
    res_lat_n_ = 0;
    if (wl_) {
      wl_->clear_stats();
      wl_ms_seen_ = 0;
      wl_kms_seen_ = 0;
    }
  }
  uint64_t live_tokens();  // Σ tile_len (headers included)
  size_t num_tiles() const { return ntiles_; }
  size_t device_bytes() const { return bytes_alloc_; }
  int ordinal() const { return ordinal_; }
  void* stream_handle() const { return stream_; }

 private:
  // Device tables and host-visible buffers of a merge launch.
  struct MergeSlot {
    uint32_t cap = 0;  // neighbour slots: id+1 for ids < cap, slot 0 for unk outside
    uint64_t* dsum = nullptr;  // kChainMax x 4 (cap + 1) keys + 2 stats words
    uint64_t* dft = nullptr;
    uint32_t* dlist = nullptr;
    uint32_t* dcount = nullptr;  // [0] touched-slot count, [1..9] completion tickets, [10] matched tiles
    DeltaRecord* host_recs = nullptr;  // pinned, device-visible
    void* dev_recs = nullptr;
    uint32_t* host_count = nullptr;    // pinned: [0] records (| need-collect), [1] flag, [2] matched tiles,
    void* dev_count = nullptr;         //         [3] k_collect offset, bytes 16..31: occurrences, tokens
    uint32_t* dmlist = nullptr;        // device: matched tiles beyond a workgroup's LDS list / multi-GPU
    uint32_t* rhdr = nullptr;          // device: per-workgroup regions of the fused completion
    uint64_t* rrec = nullptr;
    uint32_t* rtile = nullptr;
    uint32_t* host_mlist = nullptr;    // pinned: matched tiles (tile | chain index << 27)
    void* dev_mlist = nullptr;
    // multi-GPU: this rank's bucket (32-byte header, then records; records past the bucket
    // stay behind it for the overflow round), the gathered buckets, and their pinned copy
    uint8_t* xsend = nullptr;
    uint8_t* xrecv = nullptr;
    DeltaRecord* host_xrecs = nullptr;  // pinned: world x bucket records, concatenated
    void* dev_xrecs = nullptr;
    uint32_t* host_xhdr = nullptr;      // pinned: per rank [records | need-collect, k_collect offset]
    void* dev_xhdr = nullptr;
    std::vector<DeltaRecord> xall;      // all ranks' records when a bucket overflowed
    uint32_t grid = 0;
    uint32_t n_iter = 0;  // candidate tiles of the launch
    bool launched = false;
    uint32_t seq = 0;
  };
  // A launch: merges X0 .. X0+n-1, collected in order.  Up to two runs are in flight (the
  // second launched before the first is collected); run r uses slot_[r's slot].
  struct ChainRun {
    int slot = 0;
    int32_t X0 = 0;
    int n = 0;
    int collected = 0;
    bool waited = false;
    int32_t ab[2 * kChainMax] = {};
    // merge j's records and matched tiles: straight in the slot's pinned buffers for a single
    // merge, else split into the vectors below
    const DeltaRecord* rp[kChainMax] = {};
    size_t rn[kChainMax] = {};
    const uint32_t* tp[kChainMax] = {};
    size_t tn[kChainMax] = {};
    std::vector<DeltaRecord> recs[kChainMax];
    std::vector<uint32_t> tiles[kChainMax];
  };
  void ensure_slots(MergeSlot& s, uint32_t need);
  void free_slot(MergeSlot& s, bool keep_host);
  void free_all();
  void wait_flag(const MergeSlot& s);
  void finish_launch(ChainRun& run);
  size_t exchange_bucket_bytes() const { return 32 + (size_t)xchg_.bucket_records * 24; }
  void exchange_launch(MergeSlot& sl);
  size_t exchange_finish(MergeSlot& sl, const DeltaRecord** recs);
  void count_pairs_dense(int32_t unk_id, uint64_t live, std::vector<PairCount>* out);
  struct PairMaxQuery {
    int32_t a, b;
    uint64_t max_freq, ab_freq;
  };
  PairMaxQuery* pmq_ = nullptr;  // set by pair_max(): count_pairs reduces instead of collecting
  void reduce_pair_max(const PairCount* dout, uint32_t n);
  void unmerge_run(ChainRun& run, int j0);
  void unmerge_launch(ChainRun& run, const uint32_t* tiles, size_t n_tiles, int j0 = 0);
  void flush_timing(bool block);

  int ordinal_ = 0;
  void* stream_ = nullptr;
  void* aux_stream_ = nullptr;  // wide collect of a slot while the other slot's merge runs
  void* ev_[6] = {};            // [2],[3]: pair count, [4]: k_pair_hist start
  // sampled k_merge launch timing: a ring of event pairs read back without blocking
  static constexpr int kEvPairs = 16;
  void* mev_[kEvPairs][2] = {};
  struct PendingEv {
    int pair;
    double bytes;
  };
  std::vector<PendingEv> ev_pending_;
  std::vector<int> ev_free_;
  bool timing_ = false;
  KernelTimes times_;
  Exchange xchg_;
  bool exchange_ = false;  // xchg_ is set up: every launch is followed by the records exchange
  uint8_t* xrecv2_ = nullptr;  // overflow round: world x the largest remainder (grown on demand)
  size_t xrecv2_bytes_ = 0;
  std::vector<uint8_t> xstage_;
  uint64_t x_overflows_ = 0;
  int cu_count_ = 256;
  bool uploaded_ = false;
  Layout layout_ = Layout::kTypes;

  size_t ntiles_ = 0;
  size_t tok_elems_ = 0;
  int32_t* tok_ = nullptr;
  int32_t* tok0_ = nullptr;
  uint64_t* tile_off_ = nullptr;
  uint32_t* tile_len_ = nullptr;
  uint32_t* tile_len0_ = nullptr;
  uint64_t* weight_ = nullptr;
  uint64_t live_tokens0_ = 0;
  uint32_t* sig_ = nullptr;    // per-tile pair signature (Bloom filter), see k_merge
  unsigned long long* stamps_ = nullptr;  // SHRED_STAMPS diagnostic build only
  uint64_t nentries_ = 0;
  size_t ft_tiles_ = 0;         // tiles holding one occurrence of every type (TiledStream::ft_tiles)
  uint64_t ft_live_tokens_ = 0;
  uint64_t live_tokens_est_ = 0;

  MergeSlot slot_[kResSlots];  // the launch path uses slots 0 and 1
  ChainRun runs_[2];
  int run_head_ = 0, run_count_ = 0;  // runs_[run_head_] is the oldest in flight
  ChainRun& run_at(int k) { return runs_[(run_head_ + k) & 1]; }
  uint32_t keys_per_merge_ = 0;
  uint32_t* host_ulist_ = nullptr;  // pinned: tiles to unmerge
  void* dev_ulist_ = nullptr;
  std::vector<uint32_t> ulist_;
  bool unmerge_pending_ = false;  // a k_unmerge reading host_ulist_ may still run
  uint32_t seq_ = 0;            // launch sequence number echoed by the device flag
  int32_t unk_ = 0;
  uint64_t records_total_ = 0, records_max_ = 0;
  int32_t max_id_seen_ = 0;
  int32_t max_id0_ = 0;  // max id at upload (reset_tokens restores it)
  bool speculate_ = true;
  bool last_changes_ = false;  // the last collect() gave ordered changes (the indexed loop's K4)
  int64_t fin_ = -1;           // set_finalize (-1: the loop's default)
  uint64_t rollbacks_ = 0;

  void* merge_params_ = nullptr;        // MergeParams kernel arguments (with the inline tile list)
  void* unmerge_params_ = nullptr;      // UnmergeParams kernel arguments
  int max_groups_ = 256;                // k_merge grid cap (env SHREDWORD_MERGE_GROUPS)
  FILE* merge_log_ = nullptr;           // SHREDWORD_MERGE_LOG diagnostic
  TileIndex index_;                     // tile skipping (tiles.h)
  bool skip_ = true;
  std::vector<uint32_t> cand_, cand1_, cand2_;
  uint64_t visited_tiles_ = 0;
  int merge_blocks_per_cu_ = 4;

  size_t bytes_alloc_ = 0;

  // ---- the indexed merge loop (word_loop.h)
  void index_sync();               // ends the loop's launch, brings the tiles up to date
  void index_refresh();            // words_stale_: rebuild the loop's table from the tiles
  WordLoop* wl_ = nullptr;
  bool index_on_ = true;           // option (SHREDWORD_INDEX / set_option index)
  bool words_stale_ = false;       // a tile-path merge changed the tiles after the words
  bool wl_pristine_index_ = true;  // the loop's initial index is the uploaded table's
  bool hybrid_ = true;             // option (SHREDWORD_HYBRID / set_option hybrid)
  bool idx_phase_ = false;         // hybrid: the indexed loop has taken over this train()
  bool switch_pending_ = false;    // hybrid: a resident merge changed < switch_occ_ occurrences
  // option (SHREDWORD_SWITCH_OCC / set_option switch_occ); 2000 since round 6 (the small-merge word
  // loop made the late merges cheaper, the queued path's mid merges stay better on k_resident a
  // little longer: C3 A/Bs +0.5..+1.3% on three boxes, C5 10 GB within noise;
  // profiles/r06_c3_switch_ab.json)
  uint64_t switch_occ_ = 2000;
  static constexpr int kSwitchWindow = 64;
  uint64_t sw_win_[kSwitchWindow] = {};  // entries merged by the last resident merges
  uint64_t sw_n_ = 0;
  int64_t switch_x_ = -1;          // the first merge id the indexed loop ran (stats)
  double switch_ms_ = 0;           // Σ host time of the switches (tiles -> words + index build)
  int32_t reserved_max_id_ = 0;    // the last reserve_ids()
  void hybrid_switch(int32_t X);
  void resident_abort_fallback();
  std::vector<void*> retired_streams_;  // streams of aborted resident launches
  uint64_t res_aborts_ = 0;
  uint32_t* res_arrive_ = nullptr;      // k_resident: workgroups that started
  uint32_t res_arrive_polls_ = 20000;   // the leader's co-residency bound (~20 ms; env SHREDWORD_RESIDENT_ARRIVE_POLLS)
  uint32_t res_region_keys_ = 32;       // participants with more delta keys add them to the global tables
                                        // (env SHREDWORD_RESIDENT_REGION_KEYS)
  uint64_t wl_ms_seen_ = 0;        // merges already folded into times_
  double wl_kms_seen_ = 0;         // launch time already folded into times_

  // ---- k_resident state (bpe_device.hip "K2+K3 resident")
  struct ResPost {          // a merge posted to the resident loop and not yet collected
    int32_t X, a, b;
    uint32_t seq;
    int slot;
    uint32_t nparts;
    double t_post;
  };
  void plan_resident(const TiledStream& ts);
  void free_resident();
  void drain_retired();  // syncs and destroys retired_streams_ (before their buffers go)
  void start_resident();
  uint32_t post_resident(uint32_t op, int32_t a, int32_t b, int32_t X, int slot);
  bool wait_resident(const MergeSlot& sl, int32_t X);  // false: the launch aborted
  int pick_resident_slot();
  size_t collect_resident(int32_t X, const DeltaRecord** recs);
  [[noreturn]] void resident_dump(const char* why);
  bool resident_on_ = true;       // option (SHREDWORD_RESIDENT / set_option resident)
  bool resident_ok_ = false;      // the uploaded table fits (plan_resident)
  bool res_running_ = false;      // a k_resident launch is live
  bool res_lds_tok_ = true;       // the tokens are in LDS (else in HBM, LDS holds weights + signatures)
  std::vector<ResPost> res_posted_;  // oldest first (a merge and the guesses behind it)
  std::vector<uint32_t> res_post_parts_[kResSlots];  // participants of the posted merges, by slot
  int spec_depth_ = 1;               // guesses in flight behind the current merge (resident)
  int32_t res_abandoned_[kResSlots] = {-1, -1, -1, -1};  // by slot: an undone guess not yet completed
  int res_next_slot_ = 0;
  uint32_t res_grid_ = 0, res_tok_words_ = 0, res_w_words_ = 0;
  uint32_t res_sig_words_ = 0;   // LDS signature words per tile in this plan
  bool res_w_global_ = false;    // the plan reads word weights from HBM
  size_t res_shm_ = 0;
  uint32_t* res_wg_tiles_ = nullptr;   // device: grid + 1
  uint32_t* res_wg_rank_ = nullptr;    // device: grid + 1
  uint32_t* res_tile_lofs_ = nullptr;  // device: per tile
  std::vector<uint32_t> res_owner_;    // tile -> workgroup (0 dispatches and 1 gathers: they own none)
  std::vector<uint32_t> res_wg_ntiles_;
  std::vector<uint32_t> res_all_;      // every worker workgroup (1 .. grid-1)
  std::vector<uint32_t> res_wg_first_; // grid + 1: first tile of each workgroup
  std::vector<uint32_t> res_parts_;
  void* res_mbox_ = nullptr;           // pinned host ResMbox (command ring)
  void* res_mbox_dev_ = nullptr;
  uint32_t* res_cmd_ = nullptr;        // device command ring
  uint64_t* res_q_ = nullptr;          // device per-workgroup queues
  uint32_t* res_dbg_ = nullptr;        // device: per-workgroup progress (SHREDWORD_RESIDENT_DEBUG)
  uint64_t* res_stamps_ = nullptr;     // device: per-participant phase stamps (SHREDWORD_RESIDENT_STAMPS)
  double res_phase_[5] = {};
  double res_ph_[4] = {};  // diagnostic: the gatherer's phases
  uint64_t res_phase_n_ = 0;
  bool res_stamp_detail_ = false;
  double res_post_flag_last_ = 0;      // the last collected merge's post -> flag seen (µs)
  double res_host_wait_ = 0, res_parts_sum_ = 0, res_post_flag_us_ = 0;
  uint32_t* res_status_ = nullptr;     // pinned host status
  void* res_status_dev_ = nullptr;
  void* res_ev_[2] = {};
  uint64_t res_launches_ = 0;
  uint64_t res_merges_ = 0;            // merges collected in the current launch
  double res_ms_ = 0;                  // Σ k_resident launch durations (HIP events)
  double res_lat_us_ = 0;              // Σ per-merge dispatch -> flag times (device clock)
  uint64_t res_lat_n_ = 0;
};

}  // namespace shred
