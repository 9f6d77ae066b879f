/* ref_driver — runs the zero-initialised REFERENCE BPE trainer (oracle/_ref/libtrainer_ref.so)
 * through its own C ABI (reference shredword/csrc/bpe/bpe.h:62-72) and nothing else.
 * TEST INFRASTRUCTURE ONLY: used to generate golden fixtures and to calibrate the CPU port.
 *
 *   ref_driver CORPUS VOCAB UNK COVERAGE MIN_PAIR_FREQ OUT_MODEL OUT_VOCAB
 *
 * The reference prints its [MERGE]/[INFO] trace on stdout (bpe.cpp:260, :369); redirect it.
 * Timing of load/train/save goes to stderr as "TIMING load=<s> train=<s> save=<s> merges=<n>". */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
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
int bpe_train(void* trainer);
void bpe_save(const void* trainer, const char* model_path, const char* vocab_path);

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char** argv) {
  if (argc != 8) {
    fprintf(stderr, "usage: %s CORPUS VOCAB UNK COVERAGE MIN_PAIR_FREQ OUT_MODEL OUT_VOCAB\n", argv[0]);
    return 2;
  }
  RefBPEConfig cfg;
  cfg.target_vocab_size = (size_t)strtoull(argv[2], NULL, 10);
  cfg.unk_id = (int32_t)strtol(argv[3], NULL, 10);
  cfg.character_coverage = strtof(argv[4], NULL);
  cfg.min_pair_freq = strtoull(argv[5], NULL, 10);
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
