/* ref_driver — runs the zero-initialised REFERENCE BPE trainer (oracle/_ref/libtrainer_ref.so)
 * through its own C ABI (reference shredword/csrc/bpe/bpe.h:62-72) and nothing else.
 * TEST INFRASTRUCTURE ONLY: used to generate golden fixtures and to calibrate the CPU port.
 *
 *   ref_driver CORPUS VOCAB UNK COVERAGE MIN_PAIR_FREQ OUT_MODEL OUT_VOCAB
 *   ref_driver --script VOCAB UNK COVERAGE MIN_PAIR_FREQ OP...
 *
 * The first form is load -> train -> save.  The second drives one trainer through a sequence of
 * C-ABI calls, so the stateful behaviour of the reference is pinned as well (missing
 * 2): OP is one of
 *   load=PATH            bpe_load_corpus   (bpe.cpp:110-185: replaces the corpus and the pair map,
 *                                           keeps num_merges, merge_ops and the heap)
 *   init                 bpe_init          (bpe.cpp:98-108)
 *   count                bpe_count_bigrams (bpe.cpp:187-230, adds to the current pair map and heap)
 *   batch=K              bpe_merge_batch   (bpe.cpp:232-323)
 *   train                bpe_train         (bpe.cpp:345-386: bpe_init + the batch loop)
 *   save=MODEL,VOCAB     bpe_save          (bpe.cpp:388-432)
 * and after every OP the line "[SCRIPT]\t <op> <return value>" goes to stdout, between the
 * reference's own [MERGE]/[INFO] lines (bpe.cpp:260, :369).
 *
 * The reference prints its [MERGE]/[INFO] trace on stdout; redirect it.  Timing of
 * load/train/save goes to stderr as "TIMING load=<s> train=<s> save=<s> merges=<n>". */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

typedef struct {               /* layout of BPEConfig, reference bpe.h:43-48 */
  size_t target_vocab_size;
  int32_t unk_id;
  float character_coverage;
  uint64_t min_pair_freq;
} RefBPEConfig;

void* create_trainer(const RefBPEConfig* config);
void bpe_trainer_destroy(void* trainer);
int bpe_load_corpus(void* trainer, const char* input_path);
void bpe_init(void* trainer);
void bpe_count_bigrams(void* trainer);
int bpe_merge_batch(void* trainer, int batch_size);
int bpe_train(void* trainer);
void bpe_save(const void* trainer, const char* model_path, const char* vocab_path);

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static RefBPEConfig parse_config(char** v) {
  RefBPEConfig cfg;
  cfg.target_vocab_size = (size_t)strtoull(v[0], NULL, 10);
  cfg.unk_id = (int32_t)strtol(v[1], NULL, 10);
  cfg.character_coverage = strtof(v[2], NULL);
  cfg.min_pair_freq = strtoull(v[3], NULL, 10);
  return cfg;
}

static void script_mark(const char* op, long ret) {
  printf("[SCRIPT]\t %s %ld\n", op, ret);
  fflush(stdout);
}

static int run_script(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s --script VOCAB UNK COVERAGE MIN_PAIR_FREQ OP...\n", argv[0]);
    return 2;
  }
  RefBPEConfig cfg = parse_config(argv + 2);
  void* t = create_trainer(&cfg);
  fflush(stdout);
  for (int i = 6; i < argc; ++i) {
    char* op = argv[i];
    if (!strncmp(op, "load=", 5)) {
      script_mark("load", bpe_load_corpus(t, op + 5));
    } else if (!strcmp(op, "init")) {
      bpe_init(t);
      script_mark("init", 0);
    } else if (!strcmp(op, "count")) {
      bpe_count_bigrams(t);
      script_mark("count", 0);
    } else if (!strncmp(op, "batch=", 6)) {
      script_mark("batch", bpe_merge_batch(t, atoi(op + 6)));
    } else if (!strcmp(op, "train")) {
      script_mark("train", bpe_train(t));
    } else if (!strncmp(op, "save=", 5)) {
      char* paths = strdup(op + 5);
      char* comma = strchr(paths, ',');
      if (!comma) { fprintf(stderr, "save=MODEL,VOCAB\n"); return 2; }
      *comma = 0;
      bpe_save(t, paths, comma + 1);
      script_mark("save", 0);
      free(paths);
    } else {
      fprintf(stderr, "unknown op %s\n", op);
      return 2;
    }
  }
  fflush(stdout);
  _exit(0);
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "--script")) return run_script(argc, argv);
  if (argc != 8) {
    fprintf(stderr, "usage: %s CORPUS VOCAB UNK COVERAGE MIN_PAIR_FREQ OUT_MODEL OUT_VOCAB\n", argv[0]);
    return 2;
  }
  RefBPEConfig cfg = parse_config(argv + 2);
  void* t = create_trainer(&cfg);
  double t0 = now();
  if (bpe_load_corpus(t, argv[1]) != 0) { fprintf(stderr, "load failed\n"); return 1; }
  double t1 = now();
  int merges = bpe_train(t);
  double t2 = now();
  fflush(stdout);
  fprintf(stderr, "TIMING load=%.6f train=%.6f merges=%d\n", t1 - t0, t2 - t1, merges);
  bpe_save(t, argv[6], argv[7]);
  double t3 = now();
  fflush(stdout);
  fprintf(stderr, "TIMING save=%.6f\n", t3 - t2);
  /* With unk_id=-1 the reference writes freq[-1] (bpe.cpp:413) and may crash on free; the
   * files are complete by then, so leave without tearing anything down. */
  _exit(0);
}
