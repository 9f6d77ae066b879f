// C ABI of the MI355X BPE trainer: include/shredword_bpe.h.
//
// Entry points mirror the reference one for one (shredword/csrc/bpe/bpe.cpp): create_trainer
// :67-85, bpe_trainer_destroy :87-96, bpe_init :98-108, bpe_load_corpus :110-185,
// bpe_count_bigrams :187-230, bpe_merge_batch :232-323, bpe_train :345-386, bpe_save :388-432.
// The O(S) scans run on the GPU (Device); heap replay and pair info stay on the host (Engine /
// Selector) because they decide merge order exactly.  There is no CPU fallback: without a usable
// GPU, train / merge_batch return -1 and save reports an error.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/shredword_bpe.h"
#include "common.h"
#include "corpus.h"
#include "device.h"
#include "dist.h"
#include "engine.h"
#include "tiles.h"

using namespace shred;

struct Trainer {
  BPEConfig config{};
  WordTable wt;
  bool loaded = false;
  bool device_stale = true;
  std::unique_ptr<Device> dev;
  Engine engine;
  Layout layout = Layout::kTypes;
  FILE* trace = nullptr;
  bool timing = false;
  int device = -1;
  bool local_exchange = false;   // test: the multi-GPU exchange over a single-rank communicator
  int dist_mode = -1;            // multi-GPU: 1 per-merge records exchange, 0 sharded load + replicated
                                 // loop, -1 auto (exchange for the stream layout, replicate for types)
  bool dist_exchange() const { return dist_mode == 1 || (dist_mode < 0 && layout == Layout::kStream); }
  uint32_t exchange_bucket = 0;  // records per rank and exchange bucket (0: default)
  int resident = -1;             // LDS-resident merge loop: -1 default (on), 0 off, 1 on
  int index = -1;                // indexed merge loop: -1 default (on), 0 off, 1 on
  int hybrid = -1;               // resident first, indexed after: -1 default (on), 0 off, 1 on
  int64_t switch_occ = -1;       // hybrid switch: occurrences of a resident merge below which (-1 default)
  int spec_depth = 0;            // resident guesses in flight (0: env SHREDWORD_SPEC_DEPTH or default)
  int64_t finalize = -1;         // indexed loop: K4 on the device up to this many records (-1 default, 0 off)
  bool gpu_load = true;          // count the corpus words on the device (types layout)
  double load_s = 0;
  // shred_set_load_gather: a sharded load over the caller's all-gather (no RCCL)
  LoadGather ext_gather = nullptr;
  void* ext_ctx = nullptr;
  int ext_rank = 0, ext_world = 1;
};

namespace {

int env_int(const char* k, int dflt) {
  const char* v = std::getenv(k);
  return (v && *v) ? std::atoi(v) : dflt;
}

int set_option(Trainer* t, const std::string& key, const std::string& val) {
  if (key == "layout") {
    if (val == "types") t->layout = Layout::kTypes;
    else if (val == "stream") t->layout = Layout::kStream;
    else return -1;
    t->device_stale = true;
  } else if (key == "log") {
    t->engine.set_log(std::atoi(val.c_str()));
  } else if (key == "trace") {
    if (t->trace) std::fclose(t->trace);
    t->trace = val.empty() ? nullptr : std::fopen(val.c_str(), "w");
    t->engine.set_trace(t->trace);
    if (!val.empty() && !t->trace) return -1;
  } else if (key == "trace_note") {  // a caller's line in the trace file (tests of call sequences)
    if (!t->trace) return -1;
    std::fprintf(t->trace, "%s\n", val.c_str());
    std::fflush(t->trace);
  } else if (key == "timing") {
    t->timing = std::atoi(val.c_str()) != 0;
    if (t->dev) t->dev->set_timing(t->timing);
  } else if (key == "clear_stats") {
    t->engine.times() = EngineTimes();
    if (t->dev) t->dev->clear_times();
  } else if (key == "merge_groups") {
    if (!t->dev) return -1;  // tuning of an existing device (after load_corpus)
    t->dev->set_merge_groups(std::atoi(val.c_str()));
  } else if (key == "chain") {
    t->engine.set_chain(std::atoi(val.c_str()), 2048);
  } else if (key == "speculate") {
    t->engine.set_speculation(std::atoi(val.c_str()) != 0);
  } else if (key == "early_guess") {
    t->engine.set_early_guess(std::atoi(val.c_str()) != 0);
  } else if (key == "early_max_records") {
    t->engine.set_early_max_records(std::strtoull(val.c_str(), nullptr, 10));
  } else if (key == "apply_helper") {
    t->engine.set_apply_helper(std::atoi(val.c_str()) != 0);
  } else if (key == "exchange" || key == "exchange_bucket") {
    if (t->dev) return -1;  // fixed when the device is created (load_corpus)
    if (key == "exchange") {
      if (val == "local") t->local_exchange = true;
      else if (val == "off" || val == "0") t->local_exchange = false;
      else return -1;
    } else {
      const int b = std::atoi(val.c_str());
      if (b < 1) return -1;
      t->exchange_bucket = (uint32_t)b;
    }
  } else if (key == "gpu_load") {
    t->gpu_load = std::atoi(val.c_str()) != 0;
  } else if (key == "resident") {
    t->resident = std::atoi(val.c_str()) != 0 ? 1 : 0;
    if (t->dev) t->dev->set_resident(t->resident != 0);
  } else if (key == "index") {
    t->index = std::atoi(val.c_str()) != 0 ? 1 : 0;
    if (t->dev) t->dev->set_index(t->index != 0);
  } else if (key == "hybrid") {
    t->hybrid = std::atoi(val.c_str()) != 0 ? 1 : 0;
    if (t->dev) t->dev->set_hybrid(t->hybrid != 0);
  } else if (key == "switch_occ") {
    const long long n = std::atoll(val.c_str());
    if (n < 0) return -1;
    t->switch_occ = n;
    if (t->dev) t->dev->set_switch_occurrences((uint64_t)n);
  } else if (key == "finalize") {  // K4 on the device (ordered changes) for merges of <= n records
    const long long n = std::atoll(val.c_str());
    if (n < 0) return -1;
    t->finalize = n;
    if (t->dev) t->dev->set_finalize((uint32_t)n);
  } else if (key == "spec_depth") {
    const int d = std::atoi(val.c_str());
    if (d < 1 || d > Device::kResSlots - 1) return -1;
    t->spec_depth = d;
    if (t->dev) t->dev->set_spec_depth(d);
  } else if (key == "device") {
    t->device = std::atoi(val.c_str());
  } else if (key == "dist") {
    if (val == "replicate") t->dist_mode = 0;
    else if (val == "exchange") t->dist_mode = 1;
    else if (val == "auto") t->dist_mode = -1;
    else return -1;
    t->device_stale = true;
  } else if (key == "tiebreak") {  // merge selection: the reference's heap (exact) or the device's argmax
    if (val == "exact") t->engine.set_tiebreak_device(false);
    else if (val == "device") t->engine.set_tiebreak_device(true);
    else return -1;
  } else if (key == "verify_argmax") {
    const int n = std::atoi(val.c_str());
    if (n < 0) return -1;
    t->engine.set_verify(n);
  } else {
    return -1;
  }
  return 0;
}


// Creates the device and uploads this rank's share of the word table if needed.
bool ensure_device(Trainer* t, const char* caller) {
  if (!t->dev) {
    std::string why;
    if (!Device::available(&why)) {
      std::fprintf(stderr, "[ERROR]\t %s: no usable MI355X/HIP device (%s); this trainer has no CPU path\n", caller,
                   why.c_str());
      std::fflush(stderr);
      return false;
    }
    int ord = t->device;
    if (ord < 0) ord = dist_active() ? dist_state().device : env_int("LOCAL_RANK", 0);
    const int n = shred_device_count();
    if (n > 0) ord = ord % n;
    t->dev.reset(new Device(ord));
    t->dev->set_timing(t->timing);
    t->dev->set_unk(t->config.unk_id);
    if (t->resident >= 0) t->dev->set_resident(t->resident != 0);
    if (t->index >= 0) t->dev->set_index(t->index != 0);
    if (t->hybrid >= 0) t->dev->set_hybrid(t->hybrid != 0);
    if (t->switch_occ >= 0) t->dev->set_switch_occurrences((uint64_t)t->switch_occ);
    if (t->finalize >= 0) t->dev->set_finalize((uint32_t)t->finalize);
    t->dev->set_spec_depth(t->spec_depth ? t->spec_depth : env_int("SHREDWORD_SPEC_DEPTH", 1));
    if ((dist_active() && t->dist_exchange()) || t->local_exchange) {
      Device::Exchange x;
      if (dist_active()) {
        x.rank = dist_state().rank;
        x.world = dist_state().world;
        x.comm = dist_state().comm;
      } else {
        x.comm = dist_local_comm(ord);
      }
      x.allgather = dist_allgather_device;
      const int b = t->exchange_bucket ? (int)t->exchange_bucket : env_int("SHREDWORD_EXCHANGE_BUCKET", 0);
      if (b > 0) x.bucket_records = (uint32_t)b;
      t->dev->set_exchange(x);
    }
  }
  if (t->device_stale) {
    if (t->layout == Layout::kStream && t->wt.occurrence_rank.size() != t->wt.total_occurrences) {
      std::fprintf(stderr, "[ERROR]\t %s: layout=stream must be selected before load_corpus\n", caller);
      return false;
    }
    size_t begin = 0, end = 0;
    const bool xshard = dist_active() && t->dist_exchange();  // replicate: every rank holds the whole table
    const int rank = xshard ? dist_state().rank : 0, world = xshard ? dist_state().world : 1;
    shard_range(t->wt, t->layout, rank, world, &begin, &end);
    const double tp = now_seconds();
    TiledStream ts;
    pack_tiles(t->wt, t->layout, begin, end, &ts);
    int32_t max_id = 0;
    for (int c = 0; c < 256; ++c)
      if (t->wt.keep[c]) max_id = c;
    const double tu = now_seconds();
    t->dev->upload(ts, t->layout, t->wt.count, max_id);
    t->device_stale = false;
    if (std::getenv("SHREDWORD_LOAD_REPORT"))
      std::fprintf(stderr, "[LOAD] phase pack_tiles %.1f ms, device upload %.1f ms (tiles + word runs + index + "
                   "resident plan)\n", 1e3 * (tu - tp), 1e3 * (now_seconds() - tu));
  }
  return true;
}

}  // namespace

extern "C" {

Trainer* create_trainer(const BPEConfig* config) {
  if (!config) fatal("Config pointer is NULL");
  if (config->unk_id < kMinUnkId) fatal("unk_id below -2^30 is reserved for word headers");
  Trainer* t = new Trainer();
  t->config = *config;
  if (t->config.character_coverage <= 0.0 || t->config.character_coverage >= 1.0) t->config.character_coverage = 0.995f;
  if (t->config.min_pair_freq == 0) t->config.min_pair_freq = kDefaultMinPairFreq;
  t->engine.configure(t->config.target_vocab_size, t->config.unk_id, t->config.min_pair_freq);
  t->engine.set_log(env_int("SHREDWORD_LOG", 1));
  t->timing = env_int("SHREDWORD_TIMING", 0) != 0;
  t->gpu_load = env_int("SHREDWORD_GPU_LOAD", 1) != 0;
  t->device = env_int("SHREDWORD_DEVICE", -1);
  if (const char* v = std::getenv("SHREDWORD_LAYOUT")) set_option(t, "layout", v);
  if (const char* v = std::getenv("SHREDWORD_TRACE")) set_option(t, "trace", v);
  t->engine.set_speculation(env_int("SHREDWORD_SPECULATE", 1) != 0);
  t->engine.set_correction(env_int("SHREDWORD_CORRECT", 1) != 0);
  t->engine.set_early_guess(env_int("SHREDWORD_EARLY_GUESS", 0) != 0);
  t->engine.set_apply_helper(env_int("SHREDWORD_APPLY_HELPER", 0) != 0);
  if (const char* e = std::getenv("SHREDWORD_EARLY_MAX_RECORDS")) t->engine.set_early_max_records(std::strtoull(e, nullptr, 10));
  if (const char* e = std::getenv("SHREDWORD_PRED_WINDOW")) t->engine.set_pred_window(std::strtoull(e, nullptr, 10));
  if (const char* v = std::getenv("SHREDWORD_CHAIN")) set_option(t, "chain", v);
  t->engine.set_verify(env_int("SHREDWORD_VERIFY_ARGMAX", 0));
  if (const char* v = std::getenv("SHREDWORD_DIST")) set_option(t, "dist", v);
  if (const char* v = std::getenv("SHREDWORD_RESIDENT")) set_option(t, "resident", v);
  if (const char* v = std::getenv("SHREDWORD_TIEBREAK")) set_option(t, "tiebreak", v);
  if (t->engine.log() >= 1) std::printf("[INFO]\t BPE trainer initialized. Heap initialized successfully.\n");
  return t;
}

void bpe_trainer_destroy(Trainer* t) {
  if (!t) fatal("No Trainer pointer found to destroy!");
  if (t->trace) std::fclose(t->trace);
  delete t;
}

int bpe_load_corpus(Trainer* t, const char* path) {
  if (!t || !path) {
    std::fprintf(stderr, "[ERROR]\t NULL trainer or input path pointers\n");
    return -1;
  }
  const double t0 = now_seconds();
  LoadOptions opt;
  opt.unk_id = t->config.unk_id;
  opt.coverage = t->config.character_coverage;
  opt.want_stream = t->layout == Layout::kStream;
  if (t->gpu_load && !opt.want_stream && shred_device_count() > 0) {  // the ordinal ensure_device will use
    int ord = t->device;
    if (ord < 0) ord = dist_active() ? dist_state().device : env_int("LOCAL_RANK", 0);
    opt.gpu_device = ord % shred_device_count();
    opt.gpu_min_bytes = (size_t)env_int("SHREDWORD_GPU_LOAD_MIN", 1 << 20);
  }
  if (dist_active() && !t->dist_exchange() && !opt.want_stream) {  // sharded load, replicated merge loop
    opt.shard_rank = dist_state().rank;
    opt.shard_world = dist_state().world;
    opt.gather = dist_allgather_bytes;
  } else if (t->ext_gather && t->ext_world > 1 && !opt.want_stream) {  // the same over the caller's gather
    opt.shard_rank = t->ext_rank;
    opt.shard_world = t->ext_world;
    opt.gather = t->ext_gather;
    opt.gather_ctx = t->ext_ctx;
  }
  if (t->ext_gather && t->ext_world > 1 && opt.want_stream) {
    std::fprintf(stderr, "[ERROR]\t a sharded load (shred_set_load_gather) needs the types layout, not layout=stream\n");
    return -1;
  }
  std::string err;
  WordTable wt;
  if (load_corpus(path, opt, &wt, &err) != 0) {
    std::fprintf(stderr, "[ERROR]\t %s\n", err.c_str());
    return -1;
  }
  const double t_table = now_seconds();
  t->wt = std::move(wt);  // last load wins (bpe.cpp:176-178)
  t->loaded = true;
  t->device_stale = true;
  t->engine.reload();     // a fresh pair map; the merges and the heap stay (bpe.cpp:183)
  if (t->engine.log() >= 1)
    std::printf("[DEBUG]\t Character histogram built with %zu unique characters.\n", t->wt.distinct_bytes);
  // Put the word table in HBM now when a GPU is present, so train() starts HBM-resident.
  std::string why;
  if (Device::available(&why) && !ensure_device(t, "bpe_load_corpus")) return -1;
  t->load_s = now_seconds() - t0;
  if (std::getenv("SHREDWORD_LOAD_REPORT"))
    std::fprintf(stderr, "[LOAD] phase word_table %.1f ms (file -> distinct words, order, coverage, symbols), "
                 "device_table %.1f ms (tiles, upload, resident plan, word runs + index), total %.1f ms\n",
                 1e3 * (t_table - t0), 1e3 * (t->load_s - (t_table - t0)), 1e3 * t->load_s);
  return 0;
}

void bpe_init(Trainer* t) {
  if (!t) fatal("NULL trainer pointer");
  t->engine.reset_selection();
  bpe_count_bigrams(t);
}

// Before any load the reference's corpus is empty (zero-initialised Trainer): a count adds
// nothing, a batch finds the heap empty, a train performs no merge.  No device is needed then.
namespace {
struct NoCorpus : Backend {
  void count_pairs(int32_t, std::vector<PairCount>* out) override { out->clear(); }
  void merge_chain(const int32_t*, int, int32_t) override { fatal("merge without a corpus"); }
  size_t collect(int32_t, const DeltaRecord**) override { return 0; }
  void token_freq(size_t T, std::vector<uint64_t>* freq) override { freq->assign(T, 0); }
};
}  // namespace

void bpe_count_bigrams(Trainer* t) {
  if (!t) fatal("NULL trainer pointer");
  if (!t->loaded) {
    NoCorpus none;
    t->engine.count_bigrams(none);
    return;
  }
  if (!ensure_device(t, "bpe_count_bigrams")) return;
  t->engine.count_bigrams(*t->dev);
}

int bpe_merge_batch(Trainer* t, int batch_size) {
  if (!t) {
    std::fprintf(stderr, "[ERROR]\t Trainer pointer is NULL!\n");
    return -1;
  }
  if (!t->loaded) return 0;  // the heap of a trainer that never loaded is empty
  if (!ensure_device(t, "bpe_merge_batch")) return -1;
  return t->engine.merge_batch(*t->dev, batch_size);
}

int bpe_train(Trainer* t) {
  if (!t) {
    std::fprintf(stderr, "[ERROR]\t Trainer pointer is NULL!\n");
    return -1;
  }
  if (!t->loaded) {
    NoCorpus none;
    return t->engine.train(none);
  }
  if (!ensure_device(t, "bpe_train")) return -1;
  return t->engine.train(*t->dev);
}

void bpe_save(const Trainer* tc, const char* model_path, const char* vocab_path) {
  if (!tc) fatal("Trainer pointer is NULL!");
  Trainer* t = const_cast<Trainer*>(tc);
  std::vector<uint64_t> freq;
  if (t->loaded) {
    if (!ensure_device(t, "bpe_save")) return;
    t->dev->token_freq(kBaseVocab + t->engine.num_merges(), &freq);
  }
  if (dist_active() && dist_state().rank != 0) return;  // rank 0 writes the files
  t->engine.write_outputs(freq, model_path, vocab_path);
}

// ---- extensions -----------------------------------------------------------------------------
int shred_set_option(Trainer* t, const char* key, const char* value) {
  if (!t || !key || !value) return -1;
  return set_option(t, key, value);
}

int shred_set_load_gather(Trainer* t, int rank, int world, shred_gather_fn gather, void* ctx) {
  if (!t) return -1;
  if (world > 1 && (rank < 0 || rank >= world)) return -1;
  t->ext_gather = world > 1 ? gather : nullptr;
  t->ext_ctx = ctx;
  t->ext_rank = world > 1 ? rank : 0;
  t->ext_world = world > 1 ? world : 1;
  return 0;
}

int shred_reset(Trainer* t) {
  if (!t) return -1;
  if (t->dev) t->dev->reset_tokens();
  t->engine.forget_merges();
  return 0;
}

double shred_probe_merge(Trainer* t, int32_t a, int32_t b, int iters) {
  if (!t || iters <= 0 || !ensure_device(t, "shred_probe_merge")) return -1.0;
  const int32_t X = kBaseVocab + (int32_t)t->engine.num_merges();
  const bool resident = t->dev->resident();  // probes time the launch path
  t->dev->set_resident(false);
  double total = 0;
  for (int i = 0; i < iters; ++i) {
    const double t0 = now_seconds();
    t->dev->merge_scan(a, b, X);
    const DeltaRecord* recs = nullptr;
    const size_t n = t->dev->collect(X, &recs);
    total += now_seconds() - t0;
    if (n != 0) {
      t->dev->set_resident(resident);
      return -1.0;  // the pair occurs: the probe would have changed the corpus
    }
  }
  t->dev->set_resident(resident);
  return 1e6 * total / iters;
}

int shred_probe_rollback(Trainer* t, int32_t a, int32_t b) {
  if (!t || !ensure_device(t, "shred_probe_rollback")) return -1;
  const int32_t X = kBaseVocab + (int32_t)t->engine.num_merges();
  const bool resident = t->dev->resident();  // the undo path belongs to the launch path
  t->dev->set_resident(false);
  t->dev->merge_scan(a, b, X);
  t->dev->rollback(X);
  t->dev->set_resident(resident);
  return 0;
}

int64_t shred_debug_tokens(Trainer* t, int32_t* out, size_t cap) {
  if (!t || !ensure_device(t, "shred_debug_tokens")) return -1;
  std::vector<int32_t> v;
  t->dev->download_tokens(&v);
  if (out) std::memcpy(out, v.data(), std::min(cap, v.size()) * sizeof(int32_t));
  return (int64_t)v.size();
}

int64_t shred_index_trace(Trainer* t, uint32_t* out, size_t cap) {
  if (!t || !t->dev) return -1;
  const WordLoop* wl = t->dev->word_loop();
  if (!wl) return 0;
  const std::vector<uint32_t>& v = wl->trace();
  if (out) std::memcpy(out, v.data(), std::min(cap, v.size()) * sizeof(uint32_t));
  return (int64_t)v.size();
}

int shred_get_stats(const Trainer* tc, ShredStats* s) {
  if (!tc || !s) return -1;
  Trainer* t = const_cast<Trainer*>(tc);
  std::memset(s, 0, sizeof(*s));
  const EngineTimes& et = t->engine.times();
  s->load_seconds = t->load_s;
  s->init_seconds = et.init_s;
  s->train_seconds = et.train_s;
  s->host_select_seconds = et.select_s;
  s->host_launch_seconds = et.launch_s;
  s->host_wait_seconds = et.wait_s;
  s->host_apply_seconds = et.apply_s;
  s->host_apply_combine_seconds = et.combine_s;
  s->host_apply_correct_seconds = et.correct_s;
  s->host_apply_finish_seconds = et.finish_s;
  s->host_apply_early_seconds = et.early_s;
  s->host_apply_offer_seconds = et.offer_s;
  if (t->dev) {
    const KernelTimes& k = t->dev->times();
    s->merge_kernel_ms = k.merge_ms;
    s->count_kernel_ms = k.count_ms;
    s->merge_kernel_bytes = k.merge_bytes;
    s->count_kernel_bytes = k.count_bytes;
    s->merge_launches = k.merge_launches;
    s->count_launches = k.count_launches;
    s->hist_kernel_ms = k.hist_ms;
    s->hist_kernel_bytes = k.hist_bytes;
    s->hist_launches = k.hist_launches;
    s->device_bytes = t->dev->device_bytes();
    s->num_tiles = t->dev->num_tiles();
    s->live_tokens = t->dev->live_tokens();
    s->resident_launches = t->dev->resident_launches();
    s->resident_ms = t->dev->resident_ms();
    s->resident_latency_us = t->dev->resident_latency_us();
    s->resident_aborts = t->dev->resident_aborts();
    s->resident_merges = k.res_merges;
    s->resident_bytes = k.res_bytes;
    s->resident_k3_bytes = k.res_k3_bytes;
    s->resident_kernel_ms = k.res_ms;
    if (const WordLoop* wl = t->dev->word_loop()) {
      const WordLoopStats& w = wl->stats();
      s->index_on = t->dev->index_eligible() ? 1 : 0;
      s->index_merges = w.merges;
      s->index_undos = w.undos;
      s->index_launches = w.launches;
      s->index_candidates = w.candidates;
      s->index_changed = w.changed;
      s->index_occurrences = w.occurrences;
      s->index_ms = w.kernel_ms;
      s->index_dev_us = w.dev_us;
      s->index_wait_us = w.wait_us;
      s->index_dev_lookup_us = w.dev_lookup_us;
      s->index_dev_scan_us = w.dev_scan_us;
      s->index_scanned = w.scanned;
      s->index_build_us = w.build_us;
      s->index_no_sub = w.no_sub;
      s->index_staged = w.staged;
      s->index_run_ints_read = w.run_ints_read;
      s->index_run_ints_written = w.run_ints_written;
      s->index_records = w.records;
      s->index_raw_records = w.raw_records;
      s->index_finalized = w.finalized;
      s->index_dev_out_us = w.dev_out_us;
      s->index_dev_fin_us = w.dev_fin_us;
      s->index_fin_records = w.fin_records;
      s->index_spill_merges = w.spill_merges;
      s->index_spill_keys = w.spill_keys;
      s->index_switch_merge = t->dev->switch_merge();
      s->index_switch_ms = t->dev->switch_ms();
      const SelectStats& q = wl->select_stats();
      s->sel_merges = q.merges;
      s->sel_launches = q.launches;
      s->sel_rebuilds = q.rebuilds;
      s->sel_kernel_ms = q.kernel_ms;
      s->sel_rebuild_ms = q.rebuild_ms;
      s->sel_select_us = q.select_us;
      s->sel_merge_us = q.merge_us;
      s->sel_table_us = q.table_us;
      s->sel_table_pairs = q.table_pairs;
      s->sel_table_slots = q.table_slots;
      s->sel_table_grows = q.grows;
    }
  }
  {
    s->load_on_gpu = t->wt.counted_on_gpu ? 1 : 0;
  }
  s->num_words = t->wt.num_words();
  s->num_symbols = t->wt.num_symbols();
  s->num_occurrences = t->wt.total_occurrences;
  s->num_merges = t->engine.num_merges();
  s->sel_host_merges = t->engine.host_phase_merges();
  s->heap_size = t->engine.selector().heap_size();
  const Selector::Counters& c = t->engine.selector().counters();
  s->heap_pops = c.pops;
  s->heap_stale_pops = c.stale;
  s->heap_pushes = c.pushes;
  s->delta_records = c.records;
  s->apply_cycles_combine = c.cyc_combine;
  s->apply_cycles_order = c.cyc_order;
  s->apply_cycles_walk = c.cyc_walk;
  s->apply_cycles_push = c.cyc_push;
  s->helper_adopted = t->engine.helper_used();
  if (t->dev) s->tiles_visited = t->dev->visited_tiles();
  if (t->dev) s->exchange_overflows = t->dev->exchange_overflows();
  s->spec_hits = t->engine.spec_hits();
  s->spec_misses = t->engine.spec_misses();
  s->verify_checks = t->engine.verify_checks();
  s->verify_failures = t->engine.verify_failures();
  s->layout = (int32_t)t->layout;
  s->world_size = dist_active() ? dist_state().world : 1;
  return 0;
}

int shred_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int shred_hbm_probe(int device, size_t bytes, int reps, double* read_gbps, double* copy_gbps) {
  return Device::hbm_probe(device, bytes, reps, read_gbps, copy_gbps);
}

void* shred_occupy(int device, int free_cus, double max_seconds) { return Device::occupy(device, free_cus, max_seconds); }
void shred_release(void* handle) { Device::release(handle); }

int shred_dist_unique_id(void* out, size_t cap) { return dist_unique_id(out, cap); }
int shred_dist_init(int rank, int world, const void* id, size_t len, int device) {
  return dist_init(rank, world, id, len, device);
}
int shred_dist_finalize(void) { return dist_finalize(); }
int shred_dist_ranks(void) { return dist_comm_ranks(); }

}  // extern "C"
