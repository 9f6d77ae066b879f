// The BPE training driver: reference bpe_init / bpe_count_bigrams / bpe_merge_batch / bpe_train /
// bpe_save control flow (shredword/csrc/bpe/bpe.cpp:98-108, 187-432) over a Backend that owns the
// token stream.  The product backend is the HIP Device (device.h); there is no CPU backend in the
// product library (tests build a kernel-emulation backend of their own).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "selector.h"

namespace shred {

class Backend {
 public:
  virtual ~Backend() = default;
  // K1: pair histogram with first touch over every rank's share, pairs holding unk skipped.
  virtual void count_pairs(int32_t unk_id, std::vector<PairCount>* out) = 0;
  // K2+K3: merge (a,b) -> X everywhere; K4: the merge's neighbour-delta records (all ranks).
  virtual void merge_scan(int32_t a, int32_t b, int32_t X) = 0;
  virtual size_t collect(int32_t X, const DeltaRecord** recs) = 0;
  // Speculation support: a backend that can keep two merges in flight (merge_scan may be called
  // for X+1 before collect(X)) and can exactly undo the oldest outstanding merge X (which must
  // be the only one in flight) — rollback expands every X back into (a, b).
  virtual bool can_speculate() const { return false; }
  virtual void rollback(int32_t a, int32_t b, int32_t X) {}
  // K6: final weighted token histogram over ids [0, T) (all ranks).
  virtual void token_freq(size_t T, std::vector<uint64_t>* freq) = 0;
};

struct EngineTimes {
  double init_s = 0, train_s = 0;
  double select_s = 0, launch_s = 0, wait_s = 0, apply_s = 0;
};

class Engine {
 public:
  void configure(size_t target_vocab_size, int32_t unk_id, uint64_t min_pair_freq);
  void reset_selection() { sel_.reset(unk_, min_freq_); }
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
  // Speculative pipelining: while the host applies merge m's deltas and replays the heap, the
  // backend already runs the predicted merge m+1; a wrong guess is rolled back exactly.
  void set_speculation(bool on) { speculate_ = on; }
  void finish_speculation(Backend& be);  // rolls back a pending guess (before any other access)
  uint64_t spec_hits() const { return spec_hits_; }
  uint64_t spec_misses() const { return spec_misses_; }

 private:
  bool merge_one(Backend& be, int remaining);

  size_t target_vocab_ = 0;
  int32_t unk_ = 0;
  uint64_t min_freq_ = 2000;
  int log_ = 1;
  FILE* trace_ = nullptr;
  Selector sel_;
  std::vector<int32_t> merge_a_, merge_b_;
  EngineTimes times_;
  bool speculate_ = true;
  size_t pred_window_ = 256;
  bool spec_active_ = false;
  int32_t spec_a_ = 0, spec_b_ = 0, spec_x_ = 0;
  uint64_t spec_hits_ = 0, spec_misses_ = 0;
};

}  // namespace shred
