// C ABI of the MI355X BPE trainer: include/shredword_bpe.h.
//
// Control flow mirrors the reference entry points (shredword/csrc/bpe/bpe.cpp) one for one:
// create_trainer :67-85, bpe_trainer_destroy :87-96, bpe_init :98-108, bpe_load_corpus :110-185,
// bpe_count_bigrams :187-230, bpe_merge_batch :232-323, bpe_train :345-386, bpe_save :388-432.
// The merge loop's O(S) scans run on the GPU (Device); heap replay and pair info stay on the host
// (Selector) because they decide merge order exactly.  There is no CPU fallback: without a usable
// GPU, train/merge return -1 and save reports an error.
#include <hip/hip_runtime.h>
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/shredword_bpe.h"
#include "common.h"
#include "corpus.h"
#include "device.h"
#include "dist.h"
#include "selector.h"

using namespace shred;

struct Trainer {
  BPEConfig config{};
  WordTable wt;
  bool loaded = false;
  bool device_stale = true;
  std::unique_ptr<Device> dev;
  Selector sel;
  std::vector<int32_t> merge_a, merge_b;
  size_t num_merges = 0;
  // options
  Layout layout = Layout::kTypes;
  int log = 1;
  std::string trace_path;
  FILE* trace = nullptr;
  bool timing = false;
  int device = -1;
  // stats
  double load_s = 0, init_s = 0, train_s = 0;
  double select_s = 0, launch_s = 0, wait_s = 0, apply_s = 0;
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
    t->log = std::atoi(val.c_str());
  } else if (key == "trace") {
    if (t->trace) std::fclose(t->trace);
    t->trace = nullptr;
    t->trace_path = val;
    if (!val.empty()) {
      t->trace = std::fopen(val.c_str(), "w");
      if (!t->trace) return -1;
    }
  } else if (key == "timing") {
    t->timing = std::atoi(val.c_str()) != 0;
    if (t->dev) t->dev->set_timing(t->timing);
  } else if (key == "clear_stats") {
    t->select_s = t->launch_s = t->wait_s = t->apply_s = 0;
    t->init_s = t->train_s = 0;
    if (t->dev) t->dev->clear_times();
  } else if (key == "device") {
    t->device = std::atoi(val.c_str());
  } else {
    return -1;
  }
  return 0;
}

void exchange_allreduce(void*, uint64_t* dsum, uint64_t* dft, size_t n, void* stream) {
  dist_allreduce_device(dsum, n, false, stream);
  dist_allreduce_device(dft, n, true, stream);
}

// Creates the device and uploads this rank's share of the corpus if needed.
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
    if (dist_active()) t->dev->set_exchange(exchange_allreduce, nullptr);
  }
  if (t->device_stale) {
    if (t->layout == Layout::kStream && t->wt.occurrence_rank.size() != t->wt.total_occurrences)
      fatal("layout=stream needs the corpus loaded with the stream layout selected (set it before load_corpus)");
    size_t begin = 0, end = SIZE_MAX;
    if (dist_active()) {
      const bool stream = t->layout == Layout::kStream;
      const size_t n = stream ? t->wt.occurrence_rank.size() : t->wt.num_words();
      std::vector<uint64_t> prefix(n + 1, 0);
      for (size_t e = 0; e < n; ++e) {
        const uint32_t r = stream ? t->wt.occurrence_rank[e] : (uint32_t)e;
        prefix[e + 1] = prefix[e] + (t->wt.offset[r + 1] - t->wt.offset[r]) + 1;
      }
      dist_split(prefix, dist_state().rank, dist_state().world, &begin, &end);
    }
    t->dev->upload(t->wt, t->layout, begin, end);
    t->device_stale = false;
  }
  return true;
}

void count_into_selector(Trainer* t) {
  std::vector<PairCount> pairs;
  t->dev->count_pairs(t->config.unk_id, &pairs);
  dist_merge_pairs(&pairs);
  t->sel.add_counts(std::move(pairs));
}

// One merge (bpe.cpp:259-318): returns false when the heap has no valid candidate left.
bool merge_one(Trainer* t) {
  int32_t a, b;
  uint64_t freq;
  const double t0 = now_seconds();
  const bool ok = t->sel.select(&a, &b, &freq);
  const double t1 = now_seconds();
  t->select_s += t1 - t0;
  if (!ok) return false;
  const int32_t X = kBaseVocab + (int32_t)t->num_merges;
  if (t->log >= 2)
    std::printf("[MERGE]\t Merging (%d,%d) freq=%llu -> new_id=%d (merge %zu)\n", a, b, (unsigned long long)freq, X,
                t->num_merges + 1);
  if (t->trace) std::fprintf(t->trace, "M %d %d %llu %d\n", a, b, (unsigned long long)freq, X);
  t->merge_a.push_back(a);
  t->merge_b.push_back(b);
  t->dev->merge_scan(a, b, X);
  const double t2 = now_seconds();
  const DeltaRecord* recs = nullptr;
  const size_t n = t->dev->collect(X, &recs);
  const double t3 = now_seconds();
  t->sel.apply(a, b, X, recs, n);
  const double t4 = now_seconds();
  t->launch_s += t2 - t1;
  t->wait_s += t3 - t2;
  t->apply_s += t4 - t3;
  t->num_merges++;
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
  t->sel.reset(t->config.unk_id, t->config.min_pair_freq);
  t->log = env_int("SHREDWORD_LOG", 1);
  t->timing = env_int("SHREDWORD_TIMING", 0) != 0;
  t->device = env_int("SHREDWORD_DEVICE", -1);
  if (const char* v = std::getenv("SHREDWORD_LAYOUT")) set_option(t, "layout", v);
  if (const char* v = std::getenv("SHREDWORD_TRACE")) set_option(t, "trace", v);
  if (t->log >= 1) std::printf("[INFO]\t BPE trainer initialized. Heap initialized successfully.\n");
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
  std::string err;
  WordTable wt;
  if (load_corpus(path, opt, &wt, &err) != 0) {
    std::fprintf(stderr, "[ERROR]\t %s\n", err.c_str());
    return -1;
  }
  t->wt = std::move(wt);  // last load wins (bpe.cpp:176-178)
  t->loaded = true;
  t->device_stale = true;
  t->sel.reset(t->config.unk_id, t->config.min_pair_freq);
  if (t->log >= 1)
    std::printf("[DEBUG]\t Character histogram built with %zu unique characters.\n", t->wt.distinct_bytes);
  // Put the word table in HBM now when a GPU is present, so train() starts HBM-resident.
  std::string why;
  if (Device::available(&why)) ensure_device(t, "bpe_load_corpus");
  t->load_s = now_seconds() - t0;
  return 0;
}

void bpe_init(Trainer* t) {
  if (!t) fatal("NULL trainer pointer");
  t->sel.reset(t->config.unk_id, t->config.min_pair_freq);
  bpe_count_bigrams(t);
}

void bpe_count_bigrams(Trainer* t) {
  if (!t) fatal("NULL trainer pointer");
  if (!ensure_device(t, "bpe_count_bigrams")) return;
  if (t->log >= 1) std::printf("[INFO]\t Counting bigrams from %zu words...\n", t->wt.num_words());
  count_into_selector(t);
  if (t->log >= 1)
    std::printf("[INFO]\t Added %zu pairs to heap (freq >= %llu)\n", t->sel.heap_size(),
                (unsigned long long)t->config.min_pair_freq);
}

int bpe_merge_batch(Trainer* t, int batch_size) {
  if (!t) {
    std::fprintf(stderr, "[ERROR]\t Trainer pointer is NULL!\n");
    return -1;
  }
  if (!ensure_device(t, "bpe_merge_batch")) return -1;
  if (t->sel.heap_empty()) {
    if (t->log >= 2) std::printf("[INFO]\t Heap is empty, no more merges possible\n");
    return 0;
  }
  int done = 0;
  while (done < batch_size && !t->sel.heap_empty()) {
    if (!merge_one(t)) break;
    ++done;
  }
  return done;
}

int bpe_train(Trainer* t) {
  if (!t) {
    std::fprintf(stderr, "[ERROR]\t Trainer pointer is NULL!\n");
    return -1;
  }
  const double t0 = now_seconds();
  if (t->log >= 1)
    std::printf("[INFO]\t Starting BPE training (target vocab size: %zu)\n", t->config.target_vocab_size);
  if (!ensure_device(t, "bpe_train")) return -1;
  t->sel.reset(t->config.unk_id, t->config.min_pair_freq);
  count_into_selector(t);
  t->init_s = now_seconds() - t0;
  int total = 0;
  const int target = (int)t->config.target_vocab_size - kBaseVocab;  // bpe.cpp:353
  while (total < target) {
    if (t->sel.heap_empty()) {
      if (t->log >= 1) std::printf("[INFO]\t Heap exhausted, stopping training\n");
      break;
    }
    const uint64_t tf = t->sel.heap_top_freq();
    int batch = tf > 50000 ? 10 : tf > 20000 ? 5 : tf > 10000 ? 3 : tf > 5000 ? 2 : 1;  // bpe.cpp:363-368
    if (batch > target - total) batch = target - total;
    if (t->trace) std::fprintf(t->trace, "B %d %d %zu %llu\n", batch, total, t->sel.heap_size(), (unsigned long long)tf);
    if (t->log >= 2)
      std::printf("[INFO]\t Processing batch of %d merges (completed: %d/%d, heap size: %zu, top freq: %llu)\n", batch,
                  total, target, t->sel.heap_size(), (unsigned long long)tf);
    int merged = 0;
    while (merged < batch && !t->sel.heap_empty()) {
      if (!merge_one(t)) break;
      ++merged;
    }
    if (merged <= 0) {
      if (t->log >= 1) std::printf("[WARNING]\t No merges performed, stopping\n");
      break;
    }
    total += merged;
  }
  if (t->trace) std::fflush(t->trace);
  t->train_s = now_seconds() - t0;
  if (t->log >= 1) std::printf("[INFO]\t Training completed. Performed %d merges\n", total);
  return total;
}

void bpe_save(const Trainer* tc, const char* model_path, const char* vocab_path) {
  if (!tc) fatal("Trainer pointer is NULL!");
  Trainer* t = const_cast<Trainer*>(tc);
  const size_t M = t->num_merges, T = kBaseVocab + M;
  std::vector<std::string> tok(T);
  for (size_t i = 1; i < (size_t)kBaseVocab; ++i) tok[i] = std::string(1, (char)i);  // tok[0] = "" (C string)
  for (size_t m = 0; m < M; ++m) tok[kBaseVocab + m] = tok[t->merge_a[m]] + tok[t->merge_b[m]];
  std::vector<uint64_t> freq(T, 0);
  if (t->loaded) {
    if (!ensure_device(t, "bpe_save")) return;
    t->dev->token_freq(T, &freq);
    dist_allreduce_host(freq.data(), T, false);
  }
  if (dist_active() && dist_state().rank != 0) return;  // rank 0 writes the files
  if (FILE* vf = std::fopen(vocab_path, "w")) {
    for (size_t i = 0; i < T; ++i) {
      std::fwrite(tok[i].data(), 1, tok[i].size(), vf);
      std::fprintf(vf, " %llu\n", (unsigned long long)freq[i]);
    }
    std::fclose(vf);
  } else {
    std::fprintf(stderr, "[ERROR]\t Couldn't open file: %s\n", vocab_path);
  }
  if (FILE* mf = std::fopen(model_path, "wb")) {
    std::vector<int32_t> rec(3 * M);
    for (size_t m = 0; m < M; ++m) {
      rec[3 * m] = t->merge_a[m];
      rec[3 * m + 1] = t->merge_b[m];
      rec[3 * m + 2] = (int32_t)(kBaseVocab + m);
    }
    if (M) std::fwrite(rec.data(), sizeof(int32_t), rec.size(), mf);
    std::fclose(mf);
  } else {
    std::fprintf(stderr, "[ERROR]\t Couldn't open file: %s\n", model_path);
  }
  if (t->log >= 1)
    std::printf("[INFO]\tSaved %zu-token vocab to %s and %zu merges to %s\n", T, vocab_path, M, model_path);
}

// ---- extensions -----------------------------------------------------------------------------
int shred_set_option(Trainer* t, const char* key, const char* value) {
  if (!t || !key || !value) return -1;
  return set_option(t, key, value);
}

int shred_reset(Trainer* t) {
  if (!t) return -1;
  if (t->dev) t->dev->reset_tokens();
  t->num_merges = 0;
  t->merge_a.clear();
  t->merge_b.clear();
  t->sel.reset(t->config.unk_id, t->config.min_pair_freq);
  return 0;
}

int shred_get_stats(const Trainer* t, ShredStats* s) {
  if (!t || !s) return -1;
  std::memset(s, 0, sizeof(*s));
  s->load_seconds = t->load_s;
  s->init_seconds = t->init_s;
  s->train_seconds = t->train_s;
  s->host_select_seconds = t->select_s;
  s->host_launch_seconds = t->launch_s;
  s->host_wait_seconds = t->wait_s;
  s->host_apply_seconds = t->apply_s;
  if (t->dev) {
    const KernelTimes& k = t->dev->times();
    s->merge_kernel_ms = k.merge_ms;
    s->count_kernel_ms = k.count_ms;
    s->merge_kernel_bytes = k.merge_bytes;
    s->count_kernel_bytes = k.count_bytes;
    s->merge_launches = k.merge_launches;
    s->count_launches = k.count_launches;
    s->device_bytes = t->dev->device_bytes();
    s->num_tiles = t->dev->num_tiles();
    s->live_tokens = t->dev->live_tokens();
  }
  s->num_words = t->wt.num_words();
  s->num_symbols = t->wt.num_symbols();
  s->num_occurrences = t->wt.total_occurrences;
  s->num_merges = t->num_merges;
  s->heap_size = t->sel.heap_size();
  s->layout = (int32_t)t->layout;
  s->world_size = dist_active() ? dist_state().world : 1;
  return 0;
}

int shred_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int shred_dist_unique_id(void* out, size_t cap) { return dist_unique_id(out, cap); }
int shred_dist_init(int rank, int world, const void* id, size_t len, int device) {
  return dist_init(rank, world, id, len, device);
}
int shred_dist_finalize(void) { return dist_finalize(); }

}  // extern "C"
