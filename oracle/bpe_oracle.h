/* bpe_oracle.h — CPU restatement of the reference BPE path (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.  The
 * product (shredword-trainer_amd/) never links or calls it.
 *
 * Parity status: PINNED.  The restatement is checked byte-for-byte against golden .model/.vocab
 * files and [MERGE]/heap-size traces produced in the survey container by the reference's own
 * sources compiled with zero-initialised malloc (oracle/Makefile target `ref`,
 * tests/golden/make_golden.py).
 */
#ifndef BPE_ORACLE_H
#define BPE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OrConfig {           /* same meaning as reference BPEConfig, bpe.h:43-48 */
  size_t target_vocab_size;
  int32_t unk_id;
  float character_coverage;
  uint64_t min_pair_freq;
} OrConfig;

typedef struct OrTrainer OrTrainer;

OrTrainer* or_create(const OrConfig* cfg);
void or_destroy(OrTrainer* t);
/* 0 ok, -1 on open failure (reference bpe.cpp:110-185). */
int or_load(OrTrainer* t, const char* path);
/* Runs the merge loop (reference bpe.cpp:345-386).  Stops early after max_merges (<0: none) or
 * once max_seconds (<=0: none) of train time have elapsed.  Returns merges performed. */
int or_train(OrTrainer* t, long max_merges, double max_seconds);
void or_save(const OrTrainer* t, const char* model_path, const char* vocab_path);
/* The reference's other entry points, for call sequences through one trainer:
 * bpe_init (bpe.cpp:98-108), bpe_count_bigrams (:187-230, adds to the current pair map and heap),
 * bpe_merge_batch (:232-323, returns merges done).  or_load keeps the merges and the heap and
 * starts a fresh pair map, as bpe_load_corpus does (:176-183). */
void or_init(OrTrainer* t);
void or_count(OrTrainer* t);
int or_merge_batch(OrTrainer* t, int batch);
size_t or_num_merges(const OrTrainer* t);
/* The selection rule of the product's opt-in tiebreak=device mode (NOT the reference's): from
 * merge `after` on (0: from the first), each merge takes the pair of largest count, ties to the
 * smallest key ((u32)first << 32 | (u32)second), among pairs without unk whose count is >=
 * min_pair_freq; the heap rule decides the merges before.  The merge itself and every count
 * stay the reference's.  mode 0 = the reference rule throughout. */
void or_set_tiebreak(OrTrainer* t, int mode, long after);
/* Trace file: "M a b freq new_id" per merge (bpe.cpp:260) and
 * "B batch done heap_size top_freq" per batch (bpe.cpp:369).  NULL disables. */
void or_set_trace(OrTrainer* t, const char* path);
void or_set_progress(OrTrainer* t, long every);  /* > 0: PROGRESS lines on stderr every `every` merges */
/* n > 1: each merge's recount and merge scan split over n threads (word ranges); same output. */
void or_set_threads(OrTrainer* t, int n);
/* The last or_load's bytes read and number of distinct byte values. */
uint64_t or_load_bytes(const OrTrainer* t);
int or_load_unique_bytes(const OrTrainer* t);

/* Introspection for unit tests. */
size_t or_num_words(const OrTrainer* t);
size_t or_num_symbols(const OrTrainer* t);
double or_last_train_seconds(const OrTrainer* t);
/* Initial pair table in heap-push order (bpe.cpp:187-230): writes up to cap entries of
 * (first, second, freq) into out (3 int64 per entry); returns the number of pairs with freq>0. */
size_t or_initial_pairs(OrTrainer* t, int64_t* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
