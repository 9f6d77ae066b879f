#include <algorithm>
// Test-only harness: the product's host code (corpus loader, tile packing, Engine, Selector)
// driven by a CPU emulation of the device kernels, so the host logic and the multi-rank exchange
// can be checked without a GPU.  NOT part of the product library (built into
// tests/native/_build/libhostharness.so only).
//
// EmuBackend restates, sequentially, the semantics of k_pair_count / k_merge / k_token_freq over
// the tiled stream of tiles.h: greedy left-to-right occurrences (runs of a==b pair up from the
// run start), the left neighbour is X when it was just merged, the right neighbour is the original
// token, deltas keyed (slot, category) with first touch (rank << 32 | pos << 2 | category).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "corpus.h"
#include "engine.h"
#include "selector.h"
#include "tiles.h"

using namespace shred;

// Dense reduction (initial pair counts, final token histogram): sum into `sum`, min into `mn`.
typedef void (*ExchangeCb)(void* ctx, uint64_t* sum, uint64_t* mn, size_t n);
// Per-merge records exchange, as the device's RCCL all-gather: every rank's bytes concatenated
// in rank order; the returned buffer belongs to the callback and stays valid until its next call.
typedef const void* (*GatherCb)(void* ctx, const void* send, size_t nbytes, size_t* out_bytes);

namespace {

inline bool is_hdr(int32_t t) { return t < kHeaderLimit; }

class EmuBackend : public Backend {
 public:
  EmuBackend(const WordTable& wt, Layout layout, size_t begin, size_t end, uint32_t slot_cap)
      : wt_(wt), layout_(layout), cap_(slot_cap) {
    pack_tiles(wt, layout, begin, end, &ts_);
    index_.build(ts_);
    dsum_.assign(4 * ((size_t)cap_ + 1), 0);
    dft_.assign(4 * ((size_t)cap_ + 1), ~0ull);
  }
  void set_exchange(ExchangeCb cb, GatherCb gather, void* ctx) {
    cb_ = cb;
    gather_ = gather;
    ctx_ = ctx;
  }
  void set_speculation(bool on) { spec_ = on; }
  int max_chain() const override { return spec_ ? 64 : 1; }
  bool can_overlap() const override { return spec_; }

  uint64_t weight(uint32_t rank) const { return layout_ == Layout::kTypes ? wt_.count[rank] : 1; }

  // Any ids (a count after merges: a second train, a count without init): a hash map.
  void count_pairs_any(int32_t unk, std::vector<PairCount>* out) {
    std::unordered_map<uint64_t, std::pair<uint64_t, uint64_t>> m;  // pair -> (count, first touch)
    for (size_t t = 0; t < ts_.num_tiles(); ++t) {
      const int32_t* p = ts_.tok.data() + ts_.off[t];
      uint32_t hidx = 0, rank = 0;
      for (uint32_t i = 0; i < ts_.len[t]; ++i) {
        if (is_hdr(p[i])) { hidx = i; rank = (uint32_t)(p[i] - kHeaderBase); continue; }
        if (i + 1 >= ts_.len[t] || is_hdr(p[i + 1]) || p[i] == unk || p[i + 1] == unk) continue;
        auto it = m.emplace(pack_pair(p[i], p[i + 1]), std::make_pair(uint64_t(0), ~uint64_t(0))).first;
        it->second.first += weight(rank);
        it->second.second = std::min<uint64_t>(it->second.second, ((uint64_t)rank << 32) | (i - hidx - 1));
      }
    }
    for (const auto& kv : m)
      out->push_back({pair_first(kv.first), (int32_t)(uint32_t)kv.first, kv.second.first, kv.second.second});
  }

  void count_pairs(int32_t unk, std::vector<PairCount>* out) override {
    out->clear();
    bool small = true;
    for (size_t t = 0; t < ts_.num_tiles() && small; ++t)
      for (uint32_t i = 0; i < ts_.len[t]; ++i) {
        const int32_t v = ts_.tok[ts_.off[t] + i];
        if (!is_hdr(v) && v != unk && (uint32_t)v >= 256) { small = false; break; }
      }
    if (!small) {
      if (cb_) fatal("emulated multi-rank count supports ids < 256 only");
      count_pairs_any(unk, out);
      return;
    }
    const size_t D = 257 * 257;  // ids < 256 plus slot 0 (first count only)
    std::vector<uint64_t> cnt(D, 0), ft(D, ~0ull);
    for (size_t t = 0; t < ts_.num_tiles(); ++t) {
      const int32_t* p = ts_.tok.data() + ts_.off[t];
      uint32_t hidx = 0, rank = 0;
      for (uint32_t i = 0; i < ts_.len[t]; ++i) {
        if (is_hdr(p[i])) { hidx = i; rank = (uint32_t)(p[i] - kHeaderBase); continue; }
        if (i + 1 >= ts_.len[t] || is_hdr(p[i + 1]) || p[i] == unk || p[i + 1] == unk) continue;
        if ((uint32_t)p[i] >= 256 || (uint32_t)p[i + 1] >= 256) fatal("emulated count supports ids < 256 only");
        const size_t k = (size_t)p[i] * 257 + (size_t)p[i + 1];
        cnt[k] += weight(rank);
        ft[k] = std::min<uint64_t>(ft[k], ((uint64_t)rank << 32) | (i - hidx - 1));
      }
    }
    if (cb_) cb_(ctx_, cnt.data(), ft.data(), D);
    for (size_t k = 0; k < D; ++k)
      if (ft[k] != ~0ull) out->push_back({(int32_t)(k / 257), (int32_t)(k % 257), cnt[k], ft[k]});
    if (const char* rp = std::getenv("HH_RECORD")) {  // selector replay input (tests/native/selector_replay.cpp)
      rec_ = std::fopen(rp, "wb");
      if (!rec_) fatal("HH_RECORD: cannot open the file");
      const uint64_t n = out->size();
      std::fwrite(&n, 8, 1, rec_);
      std::fwrite(out->data(), sizeof(PairCount), n, rec_);
    }
  }
  FILE* rec_ = nullptr;

  void emit(uint32_t key, uint64_t w, uint64_t ft) {
    if (raw_) {  // direct mode: unreduced records, duplicates combined by the host
      raw_->push_back({key, 0, w, ft});
      return;
    }
    dsum_[key] += w;
    if (ft < dft_[key]) dft_[key] = ft;
  }
  uint32_t slot(int32_t id) const { return (uint32_t)id < cap_ ? (uint32_t)id + 1 : 0; }

  void merge_chain(const int32_t* ab, int n, int32_t X0) override {
    for (int i = 0; i < n; ++i) merge_one(ab[2 * i], ab[2 * i + 1], X0 + i);
  }

  void merge_one(int32_t a, int32_t b, int32_t X) {
    if ((uint32_t)X >= cap_) fatal("emulated slot capacity exceeded");
    std::vector<int32_t> out;
    std::vector<uint32_t> cand, matched;
    const bool use_list = index_.candidates(a, b, &cand);
    const size_t nvisit = use_list ? cand.size() : ts_.num_tiles();
    // like the device's direct mode: candidate-list merges ship per-occurrence records
    std::vector<DeltaRecord> raw;
    raw_ = (use_list && direct_) ? &raw : nullptr;
    for (size_t it = 0; it < nvisit; ++it) {
      const size_t t = use_list ? cand[it] : it;
      int32_t* p = ts_.tok.data() + ts_.off[t];
      const uint32_t len = ts_.len[t];
      size_t hits = 0;
      out.clear();
      uint32_t hidx = 0, rank = 0;
      bool prev_x = false;
      uint32_t i = 0;
      while (i < len) {
        const int32_t tk = p[i];
        if (is_hdr(tk)) {
          hidx = i;
          rank = (uint32_t)(tk - kHeaderBase);
          out.push_back(tk);
          prev_x = false;
          ++i;
          continue;
        }
        if (tk == a && i + 1 < len && p[i + 1] == b) {
          const uint64_t w = weight(rank);
          const uint64_t ftb = ((uint64_t)rank << 32) | ((uint64_t)(i - hidx - 1) << 2);
          if (i - 1 > hidx) {
            const int32_t left = prev_x ? X : p[i - 1];
            emit(slot(left) * 4 + kOldLeft, w, ftb | kOldLeft);
            emit(slot(left) * 4 + kNewLeft, w, ftb | kNewLeft);
          }
          if (i + 2 < len && !is_hdr(p[i + 2])) {
            emit(slot(p[i + 2]) * 4 + kOldRight, w, ftb | kOldRight);
            emit(slot(p[i + 2]) * 4 + kNewRight, w, ftb | kNewRight);
          }
          out.push_back(X);
          prev_x = true;
          ++hits;
          i += 2;
        } else {
          out.push_back(tk);
          prev_x = false;
          ++i;
        }
      }
      std::memcpy(p, out.data(), out.size() * sizeof(int32_t));
      ts_.len[t] = (uint32_t)out.size();
      if (hits) matched.push_back((uint32_t)t);
    }
    visited_ += nvisit;
    hist_.push_back((uint32_t)nvisit);
    mhist_.push_back((uint32_t)matched.size());
    Pending pd;
    pd.a = a;
    pd.b = b;
    pd.X = X;
    pd.matched = std::move(matched);
    if (raw_) pd.recs = std::move(raw);
    else drain(&pd.recs);
    raw_ = nullptr;
    queue_.push_back(std::move(pd));
  }

  // touched slots -> records, clearing the tables
  void drain(std::vector<DeltaRecord>* out) {
    out->clear();
    for (size_t k = 0; k < dsum_.size(); ++k) {
      if (dft_[k] == ~0ull) continue;
      out->push_back({(uint32_t)k, 0, dsum_[k], dft_[k]});
      dsum_[k] = 0;
      dft_[k] = ~0ull;
    }
  }

  void rollback(int32_t X) override {
    while (!queue_.empty() && queue_.back().X >= X) {  // newest first
      const Pending& pd = queue_.back();
      std::vector<int32_t> out;
      for (uint32_t t : pd.matched) {  // the exact inverse of the merge: X -> a b
        int32_t* p = ts_.tok.data() + ts_.off[t];
        out.clear();
        for (uint32_t i = 0; i < ts_.len[t]; ++i) {
          if (p[i] == pd.X) {
            out.push_back(pd.a);
            out.push_back(pd.b);
          } else {
            out.push_back(p[i]);
          }
        }
        std::memcpy(p, out.data(), out.size() * sizeof(int32_t));
        ts_.len[t] = (uint32_t)out.size();
      }
      queue_.pop_back();
      ++rollbacks_;
    }
    if (!queue_.empty() && queue_.front().X >= X) fatal("emulated rollback out of order");
  }
  uint64_t rollbacks_ = 0;
  uint64_t visited() const { return visited_; }
  std::vector<uint32_t> hist_;

  size_t collect(int32_t X, const DeltaRecord** recs) override {
    if (queue_.empty() || queue_.front().X != X) fatal("emulated collect of a merge that is not outstanding");
    Pending pd = std::move(queue_.front());
    queue_.erase(queue_.begin());
    if (gather_) {  // multi-rank: every rank's records, concatenated (the host combines them)
      size_t nb = 0;
      const void* all = gather_(ctx_, pd.recs.data(), pd.recs.size() * sizeof(DeltaRecord), &nb);
      if (nb % sizeof(DeltaRecord)) fatal("emulated exchange returned a partial record");
      pd.recs.resize(nb / sizeof(DeltaRecord));
      if (nb) std::memcpy(pd.recs.data(), all, nb);
    }
    if (X & 1) {  // odd merges take k_resident's bitmap form of the same tile set
      std::vector<uint32_t> words((index_.num_tiles() + 31) / 32, 0);
      std::vector<uint32_t> m(pd.matched);
      std::sort(m.begin(), m.end());
      m.erase(std::unique(m.begin(), m.end()), m.end());
      for (uint32_t t : m) words[t >> 5] |= 1u << (t & 31);
      index_.set_tiles_bits(X, words.data(), m.size());
    } else {
      index_.set_tiles(X, pd.matched.data(), pd.matched.size());
    }
    if (rec_) {
      const int32_t hdr[4] = {pd.a, pd.b, X, (int32_t)pd.recs.size()};
      std::fwrite(hdr, 4, 4, rec_);
      std::fwrite(pd.recs.data(), sizeof(DeltaRecord), pd.recs.size(), rec_);
      std::fflush(rec_);
    }
    recs_ = std::move(pd.recs);
    // with a host phase set, the records come newest-first: the device's order is arbitrary
    // (workgroups, spills), so the host side must not depend on it
    if (phase_ > 0) std::reverse(recs_.begin(), recs_.end());
    if (phase_left_ > 0) --phase_left_;
    changes_out_ = fin_ && !gather_;
    if (changes_out_) {  // K4 as the device's finalize_changes gives it, restated the reference's way
      to_changes(pd.a, pd.b, X);
      *recs = reinterpret_cast<const DeltaRecord*>(chg_.data());
      return chg_.size();
    }
    *recs = recs_.data();
    return recs_.size();
  }
  bool records_are_changes() const override { return changes_out_; }
  // The reference's FreqChangeMap (bpe.cpp:9-50) fed the records' events in scan order (first
  // touch ascending): 1024 buckets by key % 1024, head insertion, deltas summed per key; read out
  // bucket by bucket, chain head first, the merged pair skipped (bpe.cpp:297-313).
  void to_changes(int32_t a, int32_t b, int32_t X) {
    std::vector<const DeltaRecord*> ev(recs_.size());
    for (size_t i = 0; i < recs_.size(); ++i) ev[i] = &recs_[i];
    std::sort(ev.begin(), ev.end(), [](const DeltaRecord* x, const DeltaRecord* y) { return x->ft < y->ft; });
    std::vector<std::vector<Selector::Change>> bucket(1024);
    for (const DeltaRecord* r : ev) {
      const uint32_t cat = r->key & 3u, slot = r->key >> 2;
      const int32_t id = slot == 0 ? unk_ : (int32_t)(slot - 1);
      const int32_t f = cat < 2u ? id : (cat == 2u ? b : X);
      const int32_t g = cat == 0u ? a : (cat == 1u ? X : id);
      const uint64_t hk = ((uint64_t)(int64_t)f << 32) | (uint64_t)(int64_t)g;
      const int64_t d = (cat & 1u) ? (int64_t)r->sum : -(int64_t)r->sum;
      std::vector<Selector::Change>& ch = bucket[hk % 1024];
      bool found = false;
      for (Selector::Change& c : ch)
        if (c.hk == hk) {
          c.delta += d;
          found = true;
          break;
        }
      if (!found) ch.insert(ch.begin(), Selector::Change{hk, d, r->ft});  // head insertion
    }
    chg_.clear();
    const uint64_t kab = ((uint64_t)(int64_t)a << 32) | (uint64_t)(int64_t)b;
    for (const auto& ch : bucket)
      for (const Selector::Change& c : ch)
        if (c.hk != kab) chg_.push_back(c);
  }
  bool fin_ = std::getenv("HH_FINALIZE") ? std::atoi(std::getenv("HH_FINALIZE")) != 0 : false;
  bool changes_out_ = false;
  std::vector<Selector::Change> chg_;

  // The oldest outstanding merge's records before it is collected (the emulated kernels ran at
  // launch time, so they are always ready): the Engine's apply helper reads them on its thread.
  bool peek(int32_t X, const DeltaRecord** recs, size_t* n) override {
    if (!peek_on_ || gather_ || queue_.empty() || queue_.front().X != X) return false;
    *recs = queue_.front().recs.data();
    *n = queue_.front().recs.size();
    return true;
  }
  bool peek_on_ = std::getenv("HH_PEEK") ? std::atoi(std::getenv("HH_PEEK")) != 0 : true;

  // The device's resident phase, emulated: the first `k` merges of each tiebreak=device train()
  // are selected on the host (Engine::train_device) before device_select takes over.
  void set_device_phase(int k) { phase_ = phase_left_ = k < 0 ? 0 : k; }
  bool device_select_now() const override { return phase_left_ == 0; }
  int max_guesses() const override { return max_guesses_; }
  int max_guesses_ = 3;   // hh_set_max_guesses: the launch path's 1

  void token_freq(size_t T, std::vector<uint64_t>* freq) override {
    freq->assign(T, 0);
    for (size_t t = 0; t < ts_.num_tiles(); ++t) {
      const int32_t* p = ts_.tok.data() + ts_.off[t];
      uint32_t rank = 0;
      for (uint32_t i = 0; i < ts_.len[t]; ++i) {
        if (is_hdr(p[i])) { rank = (uint32_t)(p[i] - kHeaderBase); continue; }
        if ((uint32_t)p[i] < T) (*freq)[p[i]] += weight(rank);
      }
    }
    if (cb_) {
      std::vector<uint64_t> dummy(T, ~0ull);
      cb_(ctx_, freq->data(), dummy.data(), T);
    }
  }

  // tiebreak=device, restated on the CPU: the same pair table semantics as k_word_loop<true>
  // (count desc, key asc; each merge's records fold into the counts, the merged pair drops to 0).
  int device_select(const std::vector<PairCount>& pairs, int32_t X0, int n, uint64_t min_freq,
                    std::vector<SelectedMerge>* out) override {
    phase_left_ = phase_;  // the next train() starts with its host phase again
    std::unordered_map<uint64_t, uint64_t> cnt;
    for (const PairCount& p : pairs) cnt[pack_pair(p.a, p.b)] += p.count;
    const int32_t unk = unk_;
    out->clear();
    for (int m = 0; m < n; ++m) {
      uint64_t bc = 0, bk = ~0ull;
      for (const auto& kv : cnt)
        if (kv.second >= min_freq && (kv.second > bc || (kv.second == bc && kv.first < bk))) {
          bc = kv.second;
          bk = kv.first;
        }
      if (bc == 0) break;
      const int32_t a = pair_first(bk), b = (int32_t)(uint32_t)bk, X = X0 + m;
      merge_one(a, b, X);
      const DeltaRecord* recs = nullptr;
      const bool fin = fin_;
      fin_ = false;  // the device selector folds the raw records into its table
      const size_t nr = collect(X, &recs);
      fin_ = fin;
      for (size_t i = 0; i < nr; ++i) {
        const uint32_t sl = recs[i].key >> 2, cat = recs[i].key & 3u;
        const int32_t id = sl == 0 ? unk : (int32_t)(sl - 1);
        if (id == unk) continue;
        const int32_t f = cat < 2 ? id : (cat == 2 ? b : X), g = cat == 0 ? a : (cat == 1 ? X : id);
        if (f == a && g == b) continue;
        uint64_t& v = cnt[pack_pair(f, g)];
        v += (cat & 1u) ? recs[i].sum : (uint64_t)(-(int64_t)recs[i].sum);
      }
      cnt[bk] = 0;
      out->push_back({a, b, bc});
    }
    return (int)out->size();
  }
  void set_unk(int32_t u) { unk_ = u; }

  const TiledStream& stream() const { return ts_; }

 private:
  const WordTable& wt_;
  Layout layout_;
  uint32_t cap_;
  int32_t unk_ = 0;
  int phase_ = 0, phase_left_ = 0;
  TiledStream ts_;
  TileIndex index_;
  uint64_t visited_ = 0;
  std::vector<uint64_t> dsum_, dft_;
  std::vector<DeltaRecord>* raw_ = nullptr;
 public:
  std::vector<uint32_t> mhist_;  // matched tiles per launch
 private:
  bool direct_ = std::getenv("HH_DIRECT") ? std::atoi(std::getenv("HH_DIRECT")) != 0 : true;
  std::vector<DeltaRecord> recs_;
  struct Pending {
    int32_t a = 0, b = 0, X = 0;
    std::vector<uint32_t> matched;
    std::vector<DeltaRecord> recs;
  };
  std::vector<Pending> queue_;  // merges launched but not collected, oldest first
  bool spec_ = true;
  ExchangeCb cb_ = nullptr;
  GatherCb gather_ = nullptr;
  void* ctx_ = nullptr;
};

struct Harness {
  WordTable wt;
  std::unique_ptr<EmuBackend> be;
  Engine engine;
  FILE* trace = nullptr;
  uint64_t vocab = 0;
  int32_t unk = 0;
  float cov = 0.995f;
};

// Delta slots for every id a call sequence can create: later trainings continue the ids.
uint32_t slot_cap(uint64_t vocab, int32_t unk) {
  uint32_t cap = 1024;
  while (cap < 4 * (vocab + 256) || (unk >= 0 && cap < (uint64_t)unk + 1)) cap *= 2;
  return cap;
}

}  // namespace

extern "C" {

void* hh_open(const char* path, uint64_t vocab, int32_t unk, float cov, uint64_t mpf, int layout, int rank, int world) {
  Harness* h = new Harness();
  if (cov <= 0.0f || cov >= 1.0f) cov = 0.995f;
  if (mpf == 0) mpf = kDefaultMinPairFreq;
  LoadOptions opt;
  opt.unk_id = unk;
  opt.coverage = cov;
  opt.want_stream = layout == 1;
  opt.threads = 3;  // any thread count must give the same table
  std::string err;
  if (load_corpus(path, opt, &h->wt, &err) != 0) {
    delete h;
    return nullptr;
  }
  const Layout lay = layout == 1 ? Layout::kStream : Layout::kTypes;
  size_t b = 0, e = 0;
  shard_range(h->wt, lay, rank, world, &b, &e);
  h->be.reset(new EmuBackend(h->wt, lay, b, e, slot_cap(vocab, unk)));
  h->be->set_unk(unk);
  h->engine.configure(vocab, unk, mpf);
  h->engine.set_log(0);
  h->vocab = vocab;
  h->unk = unk;
  h->cov = cov;
  return h;
}

// Call sequences (bpe.cpp's entry points in any order) over the emulated device: a trainer with
// no corpus, then hh_load / hh_init / hh_count / hh_merge_batch / hh_train / hh_save.
void* hh_create(uint64_t vocab, int32_t unk, float cov, uint64_t mpf) {
  Harness* h = new Harness();
  if (cov <= 0.0f || cov >= 1.0f) cov = 0.995f;
  if (mpf == 0) mpf = kDefaultMinPairFreq;
  h->engine.configure(vocab, unk, mpf);
  h->engine.set_log(0);
  h->vocab = vocab;
  h->unk = unk;
  h->cov = cov;
  return h;
}

// bpe_load_corpus as trainer.cpp runs it: a new word table and device copy, engine.reload().
int hh_load(void* p, const char* path) {
  Harness* h = (Harness*)p;
  LoadOptions opt;
  opt.unk_id = h->unk;
  opt.coverage = h->cov;
  opt.threads = 2;
  std::string err;
  WordTable wt;
  if (load_corpus(path, opt, &wt, &err) != 0) return -1;
  h->be.reset();
  h->wt = std::move(wt);
  h->be.reset(new EmuBackend(h->wt, Layout::kTypes, 0, h->wt.num_words(), slot_cap(h->vocab, h->unk)));
  h->be->set_unk(h->unk);
  h->engine.reload();
  return 0;
}

void hh_set_early_guess(void* p, int on) { ((Harness*)p)->engine.set_early_guess(on != 0); }
void hh_set_verify_exact(void* p, int on) { ((Harness*)p)->engine.set_verify_exact(on != 0); }
uint64_t hh_exact_checks(void* p) { return ((Harness*)p)->engine.exact_checks(); }
uint64_t hh_exact_failures(void* p) { return ((Harness*)p)->engine.exact_failures(); }
void hh_set_max_guesses(void* p, int n) {
  Harness* h = (Harness*)p;
  if (h->be) h->be->max_guesses_ = n;
}
// Posts n guesses straight through Backend::post_guess (pairs (a_i, b_i), ids X0 + i), then
// undoes them; returns the guesses that were in flight.  Past max_guesses the post is fatal.
int hh_post_guesses(void* p, const int32_t* ab, int n, int32_t X0) {
  Harness* h = (Harness*)p;
  if (!h->be) return -1;
  h->be->reserve_ids(X0 + n);
  for (int i = 0; i < n; ++i) h->be->post_guess(ab[2 * i], ab[2 * i + 1], X0 + i);
  const int in_flight = h->be->guesses_in_flight();
  h->be->undo_guesses(X0);
  return in_flight;
}
void hh_set_tiebreak_device(void* p, int on) { ((Harness*)p)->engine.set_tiebreak_device(on != 0); }
void hh_set_device_phase(void* p, int k) {
  Harness* h = (Harness*)p;
  if (h->be) h->be->set_device_phase(k);
}
uint64_t hh_host_phase_merges(void* p) { return ((Harness*)p)->engine.host_phase_merges(); }
uint64_t hh_helper_used(void* p) { return ((Harness*)p)->engine.helper_used(); }
void hh_set_apply_helper(void* p, int on) { ((Harness*)p)->engine.set_apply_helper(on != 0); }
void hh_set_verify(void* p, int every) { ((Harness*)p)->engine.set_verify(every); }
uint64_t hh_verify_failures(void* p) { return ((Harness*)p)->engine.verify_failures(); }

void hh_count(void* p) {
  Harness* h = (Harness*)p;
  if (h->be) h->engine.count_bigrams(*h->be);
}

void hh_set_trace(void* p, const char* path) {
  Harness* h = (Harness*)p;
  if (h->trace) std::fclose(h->trace);
  h->trace = path ? std::fopen(path, "w") : nullptr;
  h->engine.set_trace(h->trace);
}

void hh_trace_line(void* p, const char* line) {
  Harness* h = (Harness*)p;
  if (h->trace) {
    std::fputs(line, h->trace);
    std::fflush(h->trace);
  }
}

// Sharded load (corpus.h LoadOptions::shard_*): this rank counts its byte range, the ranks'
// word lists are merged through `gather`; the merge loop then runs replicated over the full table.
void* hh_open_sharded(const char* path, uint64_t vocab, int32_t unk, float cov, uint64_t mpf, int rank, int world,
                      GatherCb gather, void* ctx) {
  Harness* h = new Harness();
  if (cov <= 0.0f || cov >= 1.0f) cov = 0.995f;
  if (mpf == 0) mpf = kDefaultMinPairFreq;
  LoadOptions opt;
  opt.unk_id = unk;
  opt.coverage = cov;
  opt.threads = 2;
  opt.shard_rank = rank;
  opt.shard_world = world;
  opt.gather = gather;
  opt.gather_ctx = ctx;
  std::string err;
  if (load_corpus(path, opt, &h->wt, &err) != 0) {
    delete h;
    return nullptr;
  }
  h->be.reset(new EmuBackend(h->wt, Layout::kTypes, 0, h->wt.num_words(), slot_cap(vocab, unk)));
  h->be->set_unk(unk);
  h->engine.configure(vocab, unk, mpf);
  h->engine.set_log(0);
  return h;
}

void hh_close(void* p) {
  Harness* h = (Harness*)p;
  if (h->trace) std::fclose(h->trace);
  delete h;
}

void hh_set_exchange(void* p, ExchangeCb cb, GatherCb gather, void* ctx) {
  ((Harness*)p)->be->set_exchange(cb, gather, ctx);
}

// trace_path: a new trace file, or "" to keep the current one (hh_set_trace).
int hh_train(void* p, const char* trace_path) {
  Harness* h = (Harness*)p;
  if (!trace_path || *trace_path) hh_set_trace(p, trace_path);
  const int n = h->engine.train(*h->be);
  if (h->trace) std::fflush(h->trace);
  return n;
}

int hh_merge_batch(void* p, int batch) {
  Harness* h = (Harness*)p;
  return h->be ? h->engine.merge_batch(*h->be, batch) : 0;
}
void hh_init(void* p) {
  Harness* h = (Harness*)p;
  h->engine.reset_selection();
  if (h->be) h->engine.count_bigrams(*h->be);
}

void hh_save(void* p, const char* model, const char* vocab, int write) {
  Harness* h = (Harness*)p;
  std::vector<uint64_t> freq;
  if (h->be) h->be->token_freq(kBaseVocab + h->engine.num_merges(), &freq);
  if (write) h->engine.write_outputs(freq, model, vocab);
}

uint64_t hh_num_words(void* p) { return ((Harness*)p)->wt.num_words(); }
uint64_t hh_num_symbols(void* p) { return ((Harness*)p)->wt.num_symbols(); }
uint64_t hh_num_tiles(void* p) { return ((Harness*)p)->be->stream().num_tiles(); }
uint64_t hh_live_tokens(void* p) {
  uint64_t s = 0;
  for (uint32_t l : ((Harness*)p)->be->stream().len) s += l;
  return s;
}
uint64_t hh_tiles_visited(void* p) { return ((Harness*)p)->be->visited(); }
uint64_t hh_match_hist(void* p, uint32_t* out, uint64_t cap) {
  const auto& h = ((Harness*)p)->be->mhist_;
  for (size_t i = 0; i < h.size() && i < cap; ++i) out[i] = h[i];
  return h.size();
}
uint64_t hh_visit_hist(void* p, uint32_t* out, uint64_t cap) {
  const auto& h = ((Harness*)p)->be->hist_;
  for (size_t i = 0; i < h.size() && i < cap; ++i) out[i] = h[i];
  return h.size();
}
void hh_counters(void* p, uint64_t* out) {
  const auto& c = ((Harness*)p)->engine.selector().counters();
  out[0] = c.pops; out[1] = c.stale; out[2] = c.pushes; out[3] = c.records; out[4] = c.changes;
  out[5] = ((Harness*)p)->engine.selector().num_pairs();
}
// Chain prediction acceptance: hist[j] = selections whose predicted chain matched exactly the
// next j merges (j = 0..k).
void hh_set_chain(void* p, int n) { ((Harness*)p)->engine.set_chain(n, 2048); }
void hh_chain_probe(void* p, int k, int window) { ((Harness*)p)->engine.set_chain_probe((size_t)k, (size_t)window); }
void hh_chain_hist(void* p, uint64_t* hist, int k) {
  Harness* h = (Harness*)p;
  const auto& log = h->engine.chain_log();
  const size_t M = h->engine.num_merges();
  for (int j = 0; j <= k; ++j) hist[j] = 0;
  for (size_t i = 0; i < log.size() && i < M; ++i) {
    int m = 0;
    for (size_t j = 0; 2 * j < log[i].size() && i + 1 + j < M; ++j) {
      if (log[i][2 * j] != h->engine.merge_first(i + 1 + j) || log[i][2 * j + 1] != h->engine.merge_second(i + 1 + j)) break;
      ++m;
    }
    hist[m]++;
  }
}
void hh_spec(void* p, int on, uint64_t* out) {
  Harness* h = (Harness*)p;
  if (on >= 0) {
    h->engine.set_speculation(on != 0);
    h->be->set_speculation(on != 0);
  }
  out[0] = h->engine.spec_hits();
  out[1] = h->engine.spec_misses();
}
void hh_times(void* p, double* out) {
  const EngineTimes& t = ((Harness*)p)->engine.times();
  out[0] = t.select_s; out[1] = t.launch_s; out[2] = t.wait_s; out[3] = t.apply_s; out[4] = t.train_s;
}
uint64_t hh_heap_size(void* p) { return ((Harness*)p)->engine.selector().heap_size(); }
uint64_t hh_distinct_bytes(void* p) { return ((Harness*)p)->wt.distinct_bytes; }
uint64_t hh_kept_bytes(void* p) { return ((Harness*)p)->wt.kept_bytes; }

// Word i of the reference-ordered table: copies its bytes (up to cap) and returns its length;
// *count receives its occurrence count.
uint64_t hh_word(void* p, uint64_t i, uint8_t* buf, uint64_t cap, uint64_t* count) {
  const WordTable& wt = ((Harness*)p)->wt;
  const uint64_t o = wt.offset[i], l = wt.offset[i + 1] - o;
  std::memcpy(buf, wt.bytes.data() + o, std::min(l, cap));
  *count = wt.count[i];
  return l;
}

}  // extern "C"

// The harness has no device: the loader's GPU word count (hip/load_device.hip) is absent here,
// so load_corpus always takes the host count.
namespace shred {
bool gpu_count_words(int, const uint8_t*, size_t, std::vector<WordRec>*, std::string* why, bool) {
  if (why) *why = "host harness: no device";
  return false;
}
bool gpu_count_file(int, int, uint64_t, size_t, std::vector<WordRec>*, std::vector<uint8_t>*, bool* nul,
                    std::string* why) {
  *nul = false;
  if (why) *why = "host harness: no device";
  return false;
}
}  // namespace shred
