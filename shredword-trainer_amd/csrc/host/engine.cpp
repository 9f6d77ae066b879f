// BPE training driver: see engine.h.
#include "engine.h"

#include <algorithm>
#include <string>
#include <unordered_map>

#include "common.h"

namespace shred {

void Engine::configure(size_t target_vocab_size, int32_t unk_id, uint64_t min_pair_freq) {
  target_vocab_ = target_vocab_size;
  unk_ = unk_id;
  min_freq_ = min_pair_freq;
  sel_.reset(unk_, min_freq_);
}

void Engine::forget_merges() {
  merge_a_.clear();
  merge_b_.clear();
  sel_.reset(unk_, min_freq_);
}

void Engine::refresh_selector(Backend& be) {
  if (!selector_stale_) return;
  selector_stale_ = false;
  sel_.reset(unk_, min_freq_);
  std::vector<PairCount> pairs;
  be.count_pairs(unk_, &pairs);
  sel_.add_counts(std::move(pairs));
}

void Engine::check_exact(Backend& be) {
  if (!verify_exact_ || !sel_.exact() || selector_stale_) return;
  std::vector<PairCount> fresh;
  be.count_pairs(unk_, &fresh);
  ++exact_checks_;
  const size_t bad = sel_.exact_mismatches(fresh);
  if (bad) {
    if (!exact_fail_)
      std::fprintf(stderr, "[ERROR]\t exactness check after %zu merges: %zu pair counts differ from a fresh K1\n",
                   merge_a_.size(), bad);
    ++exact_fail_;
  }
}

void Engine::count_bigrams(Backend& be) {
  refresh_selector(be);
  std::vector<PairCount> pairs;
  be.count_pairs(unk_, &pairs);
  const size_t unique = pairs.size();
  if (capture_) {  // SHREDWORD_APPLY_CAPTURE: the counts the selector starts from
    const uint64_t n = pairs.size();
    std::fwrite("P", 1, 1, capture_);
    std::fwrite(&n, 8, 1, capture_);
    std::fwrite(pairs.data(), sizeof(PairCount), n, capture_);
  }
  sel_.add_counts(std::move(pairs));
  check_exact(be);
  if (log_ >= 1)
    std::printf("[INFO]\t Counted %zu unique pairs\n[INFO]\t Added %zu pairs to heap (freq >= %llu)\n", unique,
                sel_.heap_size(), (unsigned long long)min_freq_);
}

Engine::~Engine() { helper_stop(); }

void Engine::helper_start() {
  if (helper_ || !helper_on_) return;
  helper_ = new Helper();
  Helper* h = helper_;
  const Selector* sel = &sel_;
  h->th = std::thread([h, sel] {
    unsigned idle = 0;
    for (;;) {
      const int st = h->state.load(std::memory_order_acquire);
      if (st == 1) {
        sel->prepare(h->a, h->b, h->X, h->recs, h->n, &h->out, h->pf, h->pfm);
        h->state.store(2, std::memory_order_release);
        idle = 0;
      } else if (st == 3) {
        return;
      } else if (++idle < (1u << 20)) {
        __builtin_ia32_pause();
      } else {
        std::this_thread::yield();
      }
    }
  });
}

void Engine::helper_stop() {
  if (!helper_) return;
  helper_drain();
  helper_->state.store(3, std::memory_order_release);
  helper_->th.join();
  delete helper_;
  helper_ = nullptr;
}

void Engine::helper_drain() {
  if (!helper_) return;
  while (helper_->state.load(std::memory_order_acquire) == 1) __builtin_ia32_pause();
  helper_->state.store(0, std::memory_order_relaxed);
}

void Engine::helper_offer(Backend& be) {
  if (!helper_ || pending_.empty() || helper_->state.load(std::memory_order_acquire) != 0) return;
  const Guess& g = pending_.front();
  const DeltaRecord* recs = nullptr;
  size_t n = 0;
  if (!be.peek(g.X, &recs, &n)) return;
  Helper* h = helper_;
  h->a = g.a;
  h->b = g.b;
  h->X = g.X;
  h->recs = recs;
  h->n = n;
  h->pf = sel_.table_base();
  h->pfm = sel_.table_mask();
  h->state.store(1, std::memory_order_release);
}

void Engine::finish_speculation(Backend& be) {
  if (pending_.empty()) return;
  helper_drain();  // the helper may be reading a guess's records: done before they are undone
  be.undo_guesses(pending_.front().X);
  pending_.clear();
  ++spec_misses_;
}

// K5 check: the guesses in flight are undone first (the device then holds exactly the corpus
// after the confirmed merges), so the next launch starts from the selected merge again.
void Engine::verify_selection(Backend& be, int32_t a, int32_t b, uint64_t freq) {
  if (!pending_.empty()) {
    helper_drain();
    be.undo_guesses(pending_.front().X);
    pending_.clear();
  }
  uint64_t mx = 0, fab = 0;
  be.pair_max(unk_, a, b, &mx, &fab);
  ++verify_checks_;
  if (mx != freq || fab != freq) {
    if (!verify_fail_)
      std::fprintf(stderr, "[ERROR]\t argmax check at merge %zu: selected (%d,%d) freq=%llu, device recount: max=%llu, "
                   "(%d,%d)=%llu\n", merge_a_.size(), a, b, (unsigned long long)freq, (unsigned long long)mx, a, b,
                   (unsigned long long)fab);
    ++verify_fail_;
  }
}

// One merge (bpe.cpp:244-318): false when the heap holds no valid candidate.  `remaining` = how
// many more merges the caller may still ask for (no guess runs past them).
bool Engine::merge_one(Backend& be, int remaining) {
  int32_t a, b;
  uint64_t freq;
  // A pair map that is not the corpus's count (call sequences such as count twice, or a batch
  // after a reload without a count): the select needs recompute_freq's rescan (bpe.cpp:251), so
  // no guess runs and the corpus's counts come from one device recount, kept current by the
  // merges' deltas.
  const bool exact = sel_.exact();
  if (!exact) {
    finish_speculation(be);
    if (!sel_.truth_live()) {
      std::vector<PairCount> pc;
      be.count_pairs(unk_, &pc);
      sel_.set_truth(pc);
    }
  }
  // the guess in flight for this merge, if the device has finished it: the helper combines and
  // orders its records while the select below runs
  if (exact) helper_offer(be);
  const double t0 = now_seconds();
  const bool ok = sel_.select(&a, &b, &freq);
  const double t1 = now_seconds();
  times_.select_s += t1 - t0;
  if (!ok) {
    finish_speculation(be);
    return false;
  }
  const int32_t X = kBaseVocab + (int32_t)merge_a_.size();
  if (verify_every_ && merge_a_.size() % (size_t)verify_every_ == 0) verify_selection(be, a, b, freq);
  if (log_ >= 2)
    std::printf("[MERGE]\t Merging (%d,%d) freq=%llu -> new_id=%d (merge %zu)\n", a, b, (unsigned long long)freq, X,
                merge_a_.size() + 1);
  if (trace_) std::fprintf(trace_, "M %d %d %llu %d\n", a, b, (unsigned long long)freq, X);
  merge_a_.push_back(a);
  merge_b_.push_back(b);
  if (probe_k_) {
    std::vector<int32_t> c(2 * probe_k_);
    c.resize(2 * sel_.predict_chain(a, b, probe_window_, probe_k_, c.data()));
    chain_log_.push_back(std::move(c));
  }
  bool launched = false;
  if (!pending_.empty()) {  // the oldest unconfirmed guess
    const Guess& g = pending_.front();
    if (g.X == X && g.a == a && g.b == b) {
      launched = true;
      if (g.posted) be.guess_confirmed();
      pending_.erase(pending_.begin());
      ++spec_hits_;
    } else {
      finish_speculation(be);
    }
  }
  const bool spec = speculate_ && exact;
  const int chain = spec ? std::max(1, std::min(std::min(chain_max_, be.max_chain()), remaining)) : 1;
  if (!launched) {
    chain_ab_.assign(2 * (size_t)chain, 0);
    chain_ab_[0] = a;
    chain_ab_[1] = b;
    const int n = 1 + (chain > 1 ? (int)sel_.predict_chain(a, b, chain_window_, (size_t)chain - 1, chain_ab_.data() + 2) : 0);
    for (int i = 1; i < n; ++i) pending_.push_back({chain_ab_[2 * i], chain_ab_[2 * i + 1], X + i});
    ++launches_;
    be.merge_chain(chain_ab_.data(), n, X);
  }
  // overlap: the next merges' guesses run while this one is consumed (up to the backend's depth;
  // each guess shares no token with this merge or the guesses before it)
  if (spec && chain == 1) {
    // early guess: one guess (X+1) in flight before the collect; the one after it (X+2) is made
    // once X is applied (below).  Otherwise the backend's depth, all guessed here.
    const size_t depth = early_guess_ ? 1 : (size_t)std::max(1, be.overlap_depth());
    while (pending_.size() < depth && (int)pending_.size() + 1 < remaining && be.can_overlap()) {
      used_.assign({a, b});
      for (const Guess& p : pending_) {
        used_.push_back(p.a);
        used_.push_back(p.b);
      }
      Guess g{0, 0, X + 1 + (int32_t)pending_.size(), true};
      if (!sel_.predict_avoid(used_.data(), used_.size(), pred_window_, &g.a, &g.b)) break;
      pending_.push_back(g);
      ++launches_;
      be.post_guess(g.a, g.b, g.X);
    }
  }
  const double t2 = now_seconds();
  const DeltaRecord* recs = nullptr;
  bool adopted = false;
  if (helper_) {
    const int st = helper_->state.load(std::memory_order_acquire);
    if (st != 0 && launched && helper_->X == X && helper_->a == a && helper_->b == b) {
      while (helper_->state.load(std::memory_order_acquire) == 1) __builtin_ia32_pause();
      be.collect(X, &recs);  // the flag is up: the helper read these records
      sel_.adopt(&helper_->out);
      helper_->state.store(0, std::memory_order_relaxed);
      adopted = true;
      ++helper_used_;
    } else if (st != 0) {
      helper_drain();
    }
  }
  const size_t n = adopted ? 0 : be.collect(X, &recs);
  const double t3 = now_seconds();
  if (capture_ && !adopted && !be.records_are_changes()) {  // one merge's records, for host replays
    const int32_t h[3] = {a, b, X};
    const uint64_t nn = n;
    std::fwrite("M", 1, 1, capture_);
    std::fwrite(h, 4, 3, capture_);
    std::fwrite(&nn, 8, 1, capture_);
    std::fwrite(recs, sizeof(DeltaRecord), n, capture_);
  }
  if (!adopted) {
    if (be.records_are_changes())
      sel_.apply_changes(a, b, X, reinterpret_cast<const Selector::Change*>(recs), n);
    else
      sel_.apply_combine(a, b, X, recs, n);
  }
  const double ta = now_seconds();
  // Late correction: with (a, b)'s changes known, a new pair holding X that is strictly more
  // frequent than the guess in flight (made before them; its own count is unchanged by this
  // merge) replaces it now, so the device undoes and redoes the guess while this merge is
  // applied and the next one selected.  The exact selection still confirms or rolls back.
  if (correct_ && spec && chain == 1 && pending_.size() == 1 && pending_.front().X == X + 1 && remaining > 1 &&
      be.can_overlap()) {
    const Guess g = pending_.front();
    int32_t pa, pb;
    uint64_t pf = 0, gf = 0;
    uint32_t gv = 0;
    sel_.lookup(g.a, g.b, &gf, &gv);
    if (sel_.predict_after(X, gf, &pa, &pb, &pf)) {
      helper_drain();
      be.undo_guesses(g.X);
      pending_.clear();
      pending_.push_back({pa, pb, X + 1, true});
      ++launches_;
      ++corrections_;
      be.post_guess(pa, pb, X + 1);
    }
  }
  const double tb = now_seconds();
  sel_.apply_finish(a, b, X);
  const double tc = now_seconds();
  // Early guess: with X applied, the guess for X+2 is made now, on the heap the coming selects
  // will pop (the guess for X+1 and every pair sharing its tokens counted as changing), and posted
  // at once, so the device has X+2 queued before it finishes X+1.  The selects of X+1 happen after
  // the post (the heap replay is off the device's path); a wrong guess for X+1 undoes both.
  // (merges with many records are device-heavy: a wrong second guess then wastes a long merge and
  // its undo on the device; early_max_records bounds where the early guess is made)
  if (early_guess_ && spec && chain == 1 && pending_.size() == 1 && pending_.front().X == X + 1 && remaining > 2 &&
      be.can_overlap() && be.max_guesses() >= 2 && (uint64_t)sel_.last_records() <= early_max_records_) {
    const Guess g1 = pending_.front();
    used_.assign({g1.a, g1.b});
    Guess g{0, 0, X + 2, true};
    if (sel_.predict_avoid(used_.data(), used_.size(), pred_window_, &g.a, &g.b)) {
      pending_.push_back(g);
      ++launches_;
      be.post_guess(g.a, g.b, g.X);
    }
  }
  const double td = now_seconds();
  if (spec) helper_offer(be);  // X+1's records, if they have landed
  times_.launch_s += t2 - t1;
  times_.wait_s += t3 - t2;
  if (launched) {
    times_.wait_hit_s += t3 - t2;
    ++times_.n_hit;
  } else {
    times_.wait_miss_s += t3 - t2;
    ++times_.n_miss;
  }
  const double t4 = now_seconds();
  times_.apply_s += t4 - t3;
  times_.combine_s += ta - t3;
  times_.correct_s += tb - ta;
  times_.finish_s += tc - tb;
  times_.early_s += td - tc;
  times_.offer_s += t4 - td;
  if (mtrace_on_)
    mtrace_.push_back(MergeTime{(float)(1e6 * (t1 - t0)), (float)(1e6 * (t2 - t1)), (float)(1e6 * (t3 - t2)),
                                (float)(1e6 * (t4 - t3)), (uint32_t)n, (uint8_t)(launched ? 1 : 0)});
  return true;
}

int Engine::merge_batch(Backend& be, int batch) {
  refresh_selector(be);
  if (sel_.heap_empty()) {
    if (log_ >= 2) std::printf("[INFO]\t Heap is empty, no more merges possible\n");
    return 0;
  }
  int done = 0;
  be.reserve_ids(kBaseVocab +
                 (int32_t)std::min<size_t>(merge_a_.size() + (size_t)batch,
                                           std::max<size_t>(target_vocab_, merge_a_.size() + kBaseVocab + 1)));
  while (done < batch && !sel_.heap_empty()) {
    if (!merge_one(be, batch - done)) break;
    ++done;
  }
  finish_speculation(be);
  be.quiesce();
  check_exact(be);
  return done;
}

// tiebreak=device: K1, then every merge selected and applied on the device.
int Engine::train_device(Backend& be, double t0) {
  sel_.reset(unk_, min_freq_);  // bpe_init; the heap stays empty (the device selects)
  std::vector<PairCount> pairs;
  be.count_pairs(unk_, &pairs);
  times_.init_s += now_seconds() - t0;
  const int target = (int)target_vocab_ - kBaseVocab;
  int n = 0;
  std::vector<SelectedMerge> sm;
  const int32_t X0 = kBaseVocab + (int32_t)merge_a_.size();
  bool exhausted = false;
  if (target > 0 && !be.device_select_now()) {
    // The early merges, while the backend's whole-chip loop serves them better than the one
    // workgroup of the device selector: the same rule (largest count, ties to the smaller key)
    // over exact host counts kept by each merge's delta records, then the device takes over
    // with those counts as its table.
    be.reserve_ids(X0 + target);
    std::unordered_map<uint64_t, uint64_t> cnt;
    cnt.reserve(2 * pairs.size() + 1024);
    // lazy max-heap on (count, ~key): an entry is live while its count is the pair's count
    std::vector<std::pair<uint64_t, uint64_t>> heap;
    heap.reserve(pairs.size());
    for (const PairCount& p : pairs) {
      const uint64_t k = pack_pair(p.a, p.b);
      cnt[k] = p.count;
      if (p.count >= min_freq_ && p.count > 0) heap.push_back({p.count, ~k});
    }
    std::make_heap(heap.begin(), heap.end());
    std::unordered_map<uint64_t, int64_t> net;
    while (n < target && !be.device_select_now()) {
      uint64_t best = 0, bk = 0;
      bool found = false;
      while (!heap.empty()) {
        std::pop_heap(heap.begin(), heap.end());
        const auto top = heap.back();
        heap.pop_back();
        const uint64_t k = ~top.second;
        const auto it = cnt.find(k);
        if (it == cnt.end() || it->second != top.first) continue;  // stale
        best = top.first;
        bk = k;
        found = true;
        break;
      }
      if (!found) {
        exhausted = true;
        break;
      }
      const int32_t a = pair_first(bk), b = pair_second(bk), X = X0 + n;
      if (verify_every_ > 0 && n % verify_every_ == 0) {  // K5: the pick is a fresh K1's maximum
        std::vector<PairCount> fresh;
        be.count_pairs(unk_, &fresh);
        uint64_t mc = 0, mk = ~0ull;
        for (const PairCount& p : fresh) {
          const uint64_t k = pack_pair(p.a, p.b);
          if (p.count > mc || (p.count == mc && k < mk)) {
            mc = p.count;
            mk = k;
          }
        }
        ++verify_checks_;
        if (mc != best || mk != bk) {
          if (!verify_fail_)
            std::fprintf(stderr, "[ERROR]\t tiebreak=device check at merge %d (host phase): selected (%d,%d) freq=%llu, "
                         "fresh K1 max (%d,%d) freq=%llu\n", n, a, b, (unsigned long long)best, pair_first(mk),
                         pair_second(mk), (unsigned long long)mc);
          ++verify_fail_;
        }
      }
      be.merge_scan(a, b, X);
      const DeltaRecord* recs = nullptr;
      const size_t nr = be.collect(X, &recs);
      // one net delta per pair first: a pair can take both signs in one merge ((X, a) of
      // "a b a b": -w as the second occurrence's left pair, +w as the first's right pair), and
      // the records come in any order
      net.clear();
      if (be.records_are_changes()) {  // already one change per pair key (reference keys: the pair's own
        const auto* ch = reinterpret_cast<const Selector::Change*>(recs);  // ids, as neither is unk here)
        for (size_t i = 0; i < nr; ++i) {
          const int32_t f = (int32_t)(uint32_t)(ch[i].hk >> 32), s = (int32_t)(uint32_t)ch[i].hk;
          if ((f == a && s == b) || f == unk_ || s == unk_) continue;
          net[pack_pair(f, s)] += ch[i].delta;
        }
      }
      for (size_t i = 0; i < nr && !be.records_are_changes(); ++i) {
        const uint32_t cat = recs[i].key & 3u, slot = recs[i].key >> 2;
        const int32_t id = slot == 0 ? unk_ : (int32_t)(slot - 1);
        int32_t f, s;
        switch (cat) {
          case kOldLeft: f = id; s = a; break;
          case kNewLeft: f = id; s = X; break;
          case kOldRight: f = b; s = id; break;
          default: f = X; s = id; break;
        }
        if ((f == a && s == b) || f == unk_ || s == unk_) continue;
        const int64_t d = (cat == kOldLeft || cat == kOldRight) ? -(int64_t)recs[i].sum : (int64_t)recs[i].sum;
        net[pack_pair(f, s)] += d;
      }
      for (const auto& kd : net) {
        if (kd.second == 0) continue;
        uint64_t& v = cnt[kd.first];
        v = kd.second < 0 ? (v >= (uint64_t)(-kd.second) ? v - (uint64_t)(-kd.second) : 0) : v + (uint64_t)kd.second;
        if (v >= min_freq_ && v > 0) {
          heap.push_back({v, ~kd.first});
          std::push_heap(heap.begin(), heap.end());
        }
      }
      cnt[bk] = 0;
      sm.push_back(SelectedMerge{a, b, best});
      ++n;
    }
    pairs.clear();
    for (const auto& kv : cnt)
      if (kv.second) pairs.push_back(PairCount{pair_first(kv.first), pair_second(kv.first), kv.second, 0});
    std::sort(pairs.begin(), pairs.end(), [](const PairCount& x, const PairCount& y) {
      return pack_pair(x.a, x.b) < pack_pair(y.a, y.b);
    });
    host_phase_merges_ += (uint64_t)n;
    if (verify_every_ > 0 && n > 0 && !exhausted) {  // the host counts must be the corpus's
      std::vector<PairCount> fresh;
      be.count_pairs(unk_, &fresh);
      std::sort(fresh.begin(), fresh.end(), [](const PairCount& x, const PairCount& y) {
        return pack_pair(x.a, x.b) < pack_pair(y.a, y.b);
      });
      bool same = fresh.size() == pairs.size();
      for (size_t i = 0; same && i < fresh.size(); ++i)
        same = fresh[i].a == pairs[i].a && fresh[i].b == pairs[i].b && fresh[i].count == pairs[i].count;
      ++verify_checks_;
      if (!same) {
        if (!verify_fail_)
          std::fprintf(stderr, "[ERROR]\t tiebreak=device: the host counts after %d merges differ from a fresh K1\n", n);
        ++verify_fail_;
      }
    }
  }
  // verify_argmax = k: the device selects k merges at a time from a table rebuilt from a fresh
  // K1 count; the first merge of each chunk must be that count's maximum (ties: the smaller key)
  const int chunk = verify_every_ > 0 ? verify_every_ : target;
  const int n_host = n;
  while (n < target && !exhausted) {
    if (n > n_host) {
      pairs.clear();
      be.count_pairs(unk_, &pairs);
    }
    const int want = std::min(chunk, target - n);
    std::vector<SelectedMerge> part;
    const int got = be.device_select(pairs, X0 + n, want, min_freq_, &part);
    if (got < 0) {
      std::fprintf(stderr, "[ERROR]\t tiebreak=device needs the device's indexed merge loop (types layout, one GPU, "
                   "index on)\n");
      return -1;
    }
    if (verify_every_ > 0 && got > 0) {
      uint64_t mc = 0, mk = ~0ull;
      for (const PairCount& p : pairs) {
        const uint64_t k = pack_pair(p.a, p.b);
        if (p.count > mc || (p.count == mc && k < mk)) {
          mc = p.count;
          mk = k;
        }
      }
      ++verify_checks_;
      if (part[0].freq != mc || pack_pair(part[0].a, part[0].b) != mk) {
        if (!verify_fail_)
          std::fprintf(stderr, "[ERROR]\t tiebreak=device check at merge %d: selected (%d,%d) freq=%llu, fresh K1 max "
                       "(%d,%d) freq=%llu\n", n, part[0].a, part[0].b, (unsigned long long)part[0].freq,
                       pair_first(mk), (int32_t)(uint32_t)mk, (unsigned long long)mc);
        ++verify_fail_;
      }
    }
    sm.insert(sm.end(), part.begin(), part.end());
    n += got;
    if (got < want) break;
  }
  {
    for (int i = 0; i < n; ++i) {
      if (log_ >= 2)
        std::printf("[MERGE]\t Merging (%d,%d) freq=%llu -> new_id=%d (merge %zu)\n", sm[i].a, sm[i].b,
                    (unsigned long long)sm[i].freq, X0 + i, merge_a_.size() + 1);
      if (trace_) std::fprintf(trace_, "M %d %d %llu %d\n", sm[i].a, sm[i].b, (unsigned long long)sm[i].freq, X0 + i);
      merge_a_.push_back(sm[i].a);
      merge_b_.push_back(sm[i].b);
    }
  }
  be.quiesce();
  // the host Selector never saw these merges: a later bpe_merge_batch / bpe_count_bigrams first
  // rebuilds it from a fresh K1 of the merged corpus, as bpe_init would
  selector_stale_ = true;
  if (trace_) std::fflush(trace_);
  times_.train_s += now_seconds() - t0;
  if (log_ >= 1) std::printf("[INFO]\t Training completed (tiebreak=device). Performed %d merges\n", n);
  return n;
}

int Engine::train(Backend& be) {
  const double t0 = now_seconds();
  if (log_ >= 1) std::printf("[INFO]\t Starting BPE training (target vocab size: %zu)\n", target_vocab_);
  if (tiebreak_device_) return train_device(be, t0);
  selector_stale_ = false;
  sel_.reset(unk_, min_freq_);  // bpe_init (bpe.cpp:98-108)
  mtrace_on_ = std::getenv("SHREDWORD_ENGINE_TRACE") != nullptr;
  // Diagnostic: the selector's inputs of this train() (the initial counts, every merge's records)
  // to a file, so the host half can be replayed and timed without a device (tools/apply_replay.cpp)
  if (const char* cp = std::getenv("SHREDWORD_APPLY_CAPTURE")) {
    capture_ = std::fopen(cp, "wb");
    if (capture_) {
      const int64_t h[2] = {unk_, (int64_t)min_freq_};
      std::fwrite("R", 1, 1, capture_);
      std::fwrite(h, 8, 2, capture_);
    }
  }
  if (const char* e = std::getenv("SHREDWORD_SIM_SELECT")) sel_.set_simulate_pops(std::atoi(e) != 0);
  mtrace_.clear();
  count_bigrams(be);
  helper_start();
  times_.init_s += now_seconds() - t0;
  int total = 0;
  const int target = (int)target_vocab_ - kBaseVocab;  // bpe.cpp:353
  // ids continue after the merges of earlier trainings (new_id = 256 + num_merges, bpe.cpp:259)
  if (target > 0) be.reserve_ids((int32_t)(kBaseVocab + merge_a_.size() + (size_t)target));
  while (total < target) {
    if (sel_.heap_empty()) {
      if (log_ >= 1) std::printf("[INFO]\t Heap exhausted, stopping training\n");
      break;
    }
    const uint64_t tf = sel_.heap_top_freq();
    int batch = tf > 50000 ? 10 : tf > 20000 ? 5 : tf > 10000 ? 3 : tf > 5000 ? 2 : 1;  // bpe.cpp:363-368
    if (batch > target - total) batch = target - total;
    if (trace_) std::fprintf(trace_, "B %d %d %zu %llu\n", batch, total, sel_.heap_size(), (unsigned long long)tf);
    if (log_ >= 2)
      std::printf("[INFO]\t Processing batch of %d merges (completed: %d/%d, heap size: %zu, top freq: %llu)\n", batch,
                  total, target, sel_.heap_size(), (unsigned long long)tf);
    int merged = 0;
    while (merged < batch && !sel_.heap_empty()) {
      if (!merge_one(be, target - total - merged)) break;
      ++merged;
    }
    if (merged <= 0) {
      if (log_ >= 1) std::printf("[WARNING]\t No merges performed, stopping\n");
      break;
    }
    total += merged;
  }
  finish_speculation(be);
  helper_stop();
  if (capture_) {
    std::fclose(capture_);
    capture_ = nullptr;
  }
  be.quiesce();
  if (trace_) std::fflush(trace_);
  times_.train_s += now_seconds() - t0;
  check_exact(be);
  if (log_ >= 1) std::printf("[INFO]\t Training completed. Performed %d merges\n", total);
  if (const char* tp = std::getenv("SHREDWORD_ENGINE_TRACE")) {
    if (FILE* f = std::fopen(tp, "w")) {
      for (size_t i = 0; i < mtrace_.size(); ++i) {
        const MergeTime& m = mtrace_[i];
        std::fprintf(f, "%zu %u %.2f %.2f %.2f %.2f %u\n", i, m.hit, m.select_us, m.launch_us, m.wait_us, m.apply_us,
                     m.records);
      }
      std::fclose(f);
    }
  }
  if (std::getenv("SHREDWORD_ENGINE_REPORT"))
    std::fprintf(stderr, "[ENGINE] merges %d: select %.2f us, apply %.2f us per merge; wait %.2f us per guessed merge (%llu), "
                 "%.2f us per posted merge (%llu); corrections %llu\n", total, 1e6 * times_.select_s / std::max(1, total),
                 1e6 * times_.apply_s / std::max(1, total), 1e6 * times_.wait_hit_s / std::max<uint64_t>(1, times_.n_hit),
                 (unsigned long long)times_.n_hit, 1e6 * times_.wait_miss_s / std::max<uint64_t>(1, times_.n_miss),
                 (unsigned long long)times_.n_miss, (unsigned long long)corrections_);
  return total;
}

void Engine::write_outputs(const std::vector<uint64_t>& freq, const char* model_path, const char* vocab_path) const {
  const size_t M = merge_a_.size(), T = kBaseVocab + M;
  std::vector<std::string> tok(T);
  for (size_t i = 1; i < (size_t)kBaseVocab; ++i) tok[i] = std::string(1, (char)i);  // tok[0]: "" as a C string
  for (size_t m = 0; m < M; ++m) tok[kBaseVocab + m] = tok[merge_a_[m]] + tok[merge_b_[m]];
  if (FILE* vf = std::fopen(vocab_path, "w")) {
    for (size_t i = 0; i < T; ++i) {
      std::fwrite(tok[i].data(), 1, tok[i].size(), vf);
      std::fprintf(vf, " %llu\n", (unsigned long long)(i < freq.size() ? freq[i] : 0));
    }
    std::fclose(vf);
  } else {
    std::fprintf(stderr, "[ERROR]\t Couldn't open file: %s\n", vocab_path);
  }
  if (FILE* mf = std::fopen(model_path, "wb")) {
    std::vector<int32_t> rec(3 * M);
    for (size_t m = 0; m < M; ++m) {
      rec[3 * m] = merge_a_[m];
      rec[3 * m + 1] = merge_b_[m];
      rec[3 * m + 2] = (int32_t)(kBaseVocab + m);
    }
    if (M) std::fwrite(rec.data(), sizeof(int32_t), rec.size(), mf);
    std::fclose(mf);
  } else {
    std::fprintf(stderr, "[ERROR]\t Couldn't open file: %s\n", model_path);
  }
  if (log_ >= 1)
    std::printf("[INFO]\tSaved %zu-token vocab to %s and %zu merges to %s\n", T, vocab_path, M, model_path);
}

}  // namespace shred
