// The BPE training driver: reference bpe_init / bpe_count_bigrams / bpe_merge_batch / bpe_train /
// bpe_save control flow (shredword/csrc/bpe/bpe.cpp:98-108, 187-432) over a Backend that owns the
// token stream.  The product backend is the HIP Device (device.h); there is no CPU backend in the
// product library (tests build a kernel-emulation backend of their own).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

#include "common.h"
#include "selector.h"

namespace shred {

class Backend {
 public:
  virtual ~Backend() = default;
  // K1: pair histogram with first touch over every rank's share, pairs holding unk skipped.
  virtual void count_pairs(int32_t unk_id, std::vector<PairCount>* out) = 0;
  // K2+K3: applies the merges (ab[2i], ab[2i+1]) -> X0 + i for i < n, in order, as one device
  // pass; K4: collect(X) then returns each merge's neighbour-delta records (all ranks), in order.
  virtual void merge_chain(const int32_t* ab, int n, int32_t X0) = 0;
  void merge_scan(int32_t a, int32_t b, int32_t X) {
    const int32_t ab[2] = {a, b};
    merge_chain(ab, 1, X);
  }
  // A guess: merge X posted before the merges ahead of it are confirmed.  The backend holds at
  // most max_guesses() unconfirmed guesses; one more is refused (fatal), never run: a backend
  // past its depth would miscount (the launch path with two guesses).
  void post_guess(int32_t a, int32_t b, int32_t X) {
    if (guesses_ >= max_guesses()) fatal("post_guess: more unconfirmed guesses than the backend holds");
    ++guesses_;
    merge_scan(a, b, X);
  }
  void guess_confirmed() {
    if (guesses_ > 0) --guesses_;
  }
  // Undoes every unconfirmed guess (rollback from the oldest, X).
  void undo_guesses(int32_t X) {
    rollback(X);
    guesses_ = 0;
  }
  int guesses_in_flight() const { return guesses_; }
  virtual size_t collect(int32_t X, const DeltaRecord** recs) = 0;
  // True when the last collect() handed out Selector::Change entries (combined per pair key, in
  // the reference's application order: K4 done on the device) instead of raw delta records.
  virtual bool records_are_changes() const { return false; }
  // Non-blocking look at the oldest outstanding merge X: true with its records once the device
  // has finished it (they stay valid until X is collected or rolled back).  Default: never.
  virtual bool peek(int32_t X, const DeltaRecord** recs, size_t* n) { return false; }
  // Longest chain the backend runs (1: one merge per pass, e.g. under a multi-GPU exchange).
  virtual int max_chain() const { return 1; }
  // True when a second launch may be issued before the first is collected (its merges run
  // after the first launch's on the device).
  virtual bool can_overlap() const { return false; }
  // How many guessed merges may be in flight behind the current one (overlap mode).
  virtual int overlap_depth() const { return 1; }
  // How many guesses the backend can hold in flight at all (the early guess needs 2).
  virtual int max_guesses() const { return 1; }
  // Undoes every launched merge with id >= X that was not collected, newest first (each
  // expands its X back into (a, b)), so the corpus is exactly as before those merges.
  virtual void rollback(int32_t X) {}
  // Ends any persistent device work (the merge loop's end): the corpus is then current in HBM.
  virtual void quiesce() {}
  // The merge loop will create ids up to max_id (tables can be sized once, up front).
  virtual void reserve_ids(int32_t max_id) {}
  // K6: final weighted token histogram over ids [0, T) (all ranks).
  virtual void token_freq(size_t T, std::vector<uint64_t>* freq) = 0;
  // tiebreak=device (K5 as the selector): merges X0 .. X0 + n - 1 chosen AND applied on the
  // device from its own pair table (`pairs`: the current K1 counts), each the pair of largest
  // count, ties to the smaller key, while that count is >= min_freq; no host round trip per
  // merge.  Returns the merges done (out: in order), -1 when the backend has no such loop.
  virtual int device_select(const std::vector<PairCount>& pairs, int32_t X0, int n, uint64_t min_freq,
                            std::vector<SelectedMerge>* out) {
    return -1;
  }
  // False while the backend's own loop serves merges better than device_select (the device's
  // whole-chip resident phase, before its switch to the indexed loop): train() in
  // tiebreak=device selects those merges on the host by the same rule (exact counts).
  virtual bool device_select_now() const { return true; }
  // K5 check (debug): a fresh K1 over the current corpus reduced to the largest pair count
  // (*max_freq) and the count of (a, b) (*ab_freq).  Default: reduced on the host.
  virtual void pair_max(int32_t unk_id, int32_t a, int32_t b, uint64_t* max_freq, uint64_t* ab_freq) {
    std::vector<PairCount> pc;
    count_pairs(unk_id, &pc);
    *max_freq = *ab_freq = 0;
    for (const PairCount& p : pc) {
      if (p.count > *max_freq) *max_freq = p.count;
      if (p.a == a && p.b == b) *ab_freq = p.count;
    }
  }

 private:
  int guesses_ = 0;
};

struct EngineTimes {
  double init_s = 0, train_s = 0;
  double select_s = 0, launch_s = 0, wait_s = 0, apply_s = 0;
  double wait_hit_s = 0, wait_miss_s = 0;  // wait_s of merges whose guess ran / had to be posted
  uint64_t n_hit = 0, n_miss = 0;
  // apply_s split: the records' combine on this thread, the late correction, the info walk and
  // heap pushes, the early guess, the helper hand-over
  double combine_s = 0, correct_s = 0, finish_s = 0, early_s = 0, offer_s = 0;
};

class Engine {
 public:
  void configure(size_t target_vocab_size, int32_t unk_id, uint64_t min_pair_freq);
  void reset_selection() {
    selector_stale_ = false;
    sel_.reset(unk_, min_freq_);
  }
  // bpe_load_corpus: the pair map starts fresh, the heap and the merges stay (bpe.cpp:176-183).
  void reload() { sel_.reset_info(); }
  void forget_merges();

  void count_bigrams(Backend& be);            // bpe_count_bigrams (bpe.cpp:187-230)
  int merge_batch(Backend& be, int batch);    // bpe_merge_batch (bpe.cpp:232-323)
  int train(Backend& be);                     // bpe_train (bpe.cpp:345-386), bpe_init included
  // bpe_save (bpe.cpp:388-432).  `freq` = final token histogram (size 256 + merges) or empty.
  void write_outputs(const std::vector<uint64_t>& freq, const char* model_path, const char* vocab_path) const;

  void set_log(int level) { log_ = level; }
  int log() const { return log_; }
  void set_trace(FILE* f) { trace_ = f; }
  size_t num_merges() const { return merge_a_.size(); }
  int32_t merge_first(size_t m) const { return merge_a_[m]; }
  int32_t merge_second(size_t m) const { return merge_b_[m]; }
  const Selector& selector() const { return sel_; }
  EngineTimes& times() { return times_; }
  // Speculation, in one of two modes (results are identical either way):
  //  * overlap (default): while the host consumes merge m, the backend already runs a second
  //    launch with the merge guessed to come next (Selector::predict_next);
  //  * chain (set_chain(n > 1)): the selected merge and up to n-1 guessed successors
  //    (Selector::predict_chain) run in one launch.
  // Guesses are confirmed one by one by the exact selection; a wrong tail is rolled back.
  void set_chain(int max_len, size_t window) {
    chain_max_ = max_len < 1 ? 1 : max_len;
    chain_window_ = window;
  }
  void set_speculation(bool on) { speculate_ = on; }
  // Late correction of the guess in flight once the current merge's records are known (default
  // on; SHREDWORD_CORRECT=0 turns it off).
  void set_correction(bool on) { correct_ = on; }
  // Early guess (opt-in; SHREDWORD_EARLY_GUESS=1 or option early_guess=1): the guess for X+2 is
  // posted right after X is applied, before the select of X+1 (see merge_one).  Measured on one
  // box: C3 within noise of off, C4 80 GB -3..-6% (a wrong second guess wastes a long merge).
  void set_early_guess(bool on) { early_guess_ = on; }
  // ... only after merges with at most this many delta records (default: always).
  void set_early_max_records(uint64_t n) { early_max_records_ = n; }
  // Apply helper (opt-in; SHREDWORD_APPLY_HELPER=1 or option apply_helper=1): a
  // second host thread combines and orders the records of the guess in flight (Selector::prepare)
  // while this thread selects; a confirmed guess then only has its changes walked and pushed.
  void set_apply_helper(bool on) { helper_on_ = on; }
  // Heap slots the overlap guess (Selector::predict_avoid) may look at (default 256;
  // SHREDWORD_PRED_WINDOW overrides).
  void set_pred_window(size_t n) { pred_window_ = n ? n : 1; }
  uint64_t helper_used() const { return helper_used_; }
  ~Engine();
  uint64_t corrections() const { return corrections_; }
  // K5 argmax verifier (debug): every `every` merges (0 = off), the selected pair's frequency is
  // checked against a device recount of the corpus (Backend::pair_max): it must be the largest
  // pair count and (a, b)'s own count.  Mismatches are counted and the first is printed.
  void set_verify(int every) { verify_every_ = every < 0 ? 0 : every; }
  // Merge selection of train(): the reference's heap replay (exact, default) or, opt-in, the
  // device's own argmax (Backend::device_select): NOT bit-exact with the reference (ties go to
  // the smaller pair key), every merge still the most frequent pair of the corpus at its step.
  void set_tiebreak_device(bool on) { tiebreak_device_ = on; }
  bool tiebreak_device() const { return tiebreak_device_; }
  uint64_t verify_checks() const { return verify_checks_; }
  // Debug: after every count / batch / train, while the selector claims its pair
  // info is the corpus's exact count, compare it with a fresh K1 (Selector::exact_mismatches).
  void set_verify_exact(bool on) { verify_exact_ = on; }
  uint64_t exact_checks() const { return exact_checks_; }
  uint64_t exact_failures() const { return exact_fail_; }
  uint64_t verify_failures() const { return verify_fail_; }
  uint64_t host_phase_merges() const { return host_phase_merges_; }  // tiebreak=device, selected on the host
  void finish_speculation(Backend& be);  // rolls back unconfirmed guesses (before any other access)
  uint64_t spec_hits() const { return spec_hits_; }
  uint64_t spec_misses() const { return spec_misses_; }
  uint64_t launches() const { return launches_; }
  // Diagnostic: record a predicted chain of k merges after every selection.
  void set_chain_probe(size_t k, size_t window) { probe_k_ = k; probe_window_ = window; }
  const std::vector<std::vector<int32_t>>& chain_log() const { return chain_log_; }

 private:
  bool merge_one(Backend& be, int remaining);
  void verify_selection(Backend& be, int32_t a, int32_t b, uint64_t freq);

  size_t target_vocab_ = 0;
  int32_t unk_ = 0;
  uint64_t min_freq_ = 2000;
  int log_ = 1;
  FILE* trace_ = nullptr;
  FILE* capture_ = nullptr;  // SHREDWORD_APPLY_CAPTURE (train(): counts + records)
  Selector sel_;
  std::vector<int32_t> merge_a_, merge_b_;
  EngineTimes times_;
  bool speculate_ = true;
  int chain_max_ = 1;
  size_t chain_window_ = 2048;
  size_t pred_window_ = 256;
  struct Guess {
    int32_t a, b, X;
    bool posted = false;  // its own launch (Backend::post_guess), not the tail of a chain
  };
  std::vector<Guess> pending_;  // launched guesses awaiting confirmation, oldest first
  std::vector<int32_t> used_;
  std::vector<int32_t> chain_ab_;
  uint64_t spec_hits_ = 0, spec_misses_ = 0, launches_ = 0;
  int verify_every_ = 0;
  bool tiebreak_device_ = false;
  int train_device(Backend& be, double t0);
  bool verify_exact_ = false;
  uint64_t exact_checks_ = 0, exact_fail_ = 0;
  void check_exact(Backend& be);
  bool selector_stale_ = false;         // tiebreak=device trained: the heap does not hold the corpus
  void refresh_selector(Backend& be);   // ... rebuilt from a fresh K1 before the next batch / count
  bool correct_ = true;
  bool early_guess_ = false;
  uint64_t early_max_records_ = ~0ull;
  uint64_t corrections_ = 0;
  uint64_t verify_checks_ = 0, verify_fail_ = 0;
  uint64_t host_phase_merges_ = 0;
  // the apply helper: one job at a time (0 idle, 1 submitted, 2 done, 3 quit)
  struct Helper {
    std::thread th;
    std::atomic<int> state{0};
    int32_t a = 0, b = 0, X = 0;
    const DeltaRecord* recs = nullptr;
    size_t n = 0;
    const void* pf = nullptr;
    uint64_t pfm = 0;
    Selector::Prepared out;
  };
  Helper* helper_ = nullptr;
  bool helper_on_ = false;  // C3 +0.7%, C4 80 GB -20% (profiles/r04_c4_80g_option_ab.json): off by default
  uint64_t helper_used_ = 0;
  void helper_start();
  void helper_stop();
  void helper_drain();                       // no job running (its result dropped)
  void helper_offer(Backend& be);            // submits the oldest guess's records if they are ready
  size_t probe_k_ = 0, probe_window_ = 256;
  std::vector<std::vector<int32_t>> chain_log_;
  // SHREDWORD_ENGINE_TRACE=<path>: per merge (hit, select, launch, wait, apply µs, records),
  // written at the end of train()
  struct MergeTime { float select_us, launch_us, wait_us, apply_us; uint32_t records; uint8_t hit; };
  std::vector<MergeTime> mtrace_;
  bool mtrace_on_ = false;
};

}  // namespace shred
