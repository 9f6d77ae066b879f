/* shredword_bpe.h — C ABI of the MI355X BPE trainer (libtrainer.so).
 *
 * Drop-in for the reference's BPE C ABI (shredword/csrc/bpe/bpe.h:62-72) as bound by its ctypes
 * layer (shredword/cbase.py:50-57): same symbol names, argument meaning, return conventions and
 * BPEConfig layout (bpe.h:43-48; 24 bytes, offsets 0/8/12/16).  The 13 Unigram symbols that
 * cbase.py:59-71 binds at import are exported as stubs that fail (Unigram is out of scope,
 * SURVEY.md §2 #7).  Symbols prefixed shred_ are extensions; a reference user never needs them.
 *
 * Plain pointers and sizes only.  The Trainer handle is opaque; it is not thread-safe (like the
 * reference's), and no call holds or needs the Python GIL.
 */
#ifndef SHREDWORD_BPE_H
#define SHREDWORD_BPE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* reference bpe.h:43-48 */
typedef struct BPEConfig {
  size_t target_vocab_size;
  int32_t unk_id;            /* must be >= -2^30 (values below are reserved for word headers) */
  float character_coverage;  /* outside (0,1) -> 0.995 (bpe.cpp:78) */
  uint64_t min_pair_freq;    /* 0 -> 2000 (bpe.cpp:79) */
} BPEConfig;

typedef struct Trainer Trainer;

/* ---- reference BPE ABI (bpe.h:63-71) ---------------------------------------------------- */
/* replaces bpe.cpp:67-85.  NULL config -> message + exit(EXIT_FAILURE), as the reference. */
Trainer* create_trainer(const BPEConfig* config);
/* replaces bpe.cpp:87-96.  NULL -> message + exit(EXIT_FAILURE). */
void bpe_trainer_destroy(Trainer* trainer);
/* replaces bpe.cpp:110-185.  0 on success, -1 on NULL args or open failure.  Last call wins.
 * The distinct-word table is built on the host and uploaded to HBM when a GPU is present. */
int bpe_load_corpus(Trainer* trainer, const char* input_path);
/* replaces bpe.cpp:98-108: resets pair info and heap, then bpe_count_bigrams. */
void bpe_init(Trainer* trainer);
/* replaces bpe.cpp:187-230: device pair histogram (K1) + reference-ordered heap build. */
void bpe_count_bigrams(Trainer* trainer);
/* replaces bpe.cpp:232-323: up to batch_size merges (device K2-K4 + host heap replay).
 * Returns merges done (0 when the heap is empty), -1 on NULL or when no GPU is usable. */
int bpe_merge_batch(Trainer* trainer, int batch_size);
/* replaces bpe.cpp:345-386.  Returns merges performed, -1 on NULL or when no GPU is usable. */
int bpe_train(Trainer* trainer);
/* replaces bpe.cpp:388-432: writes .vocab (text) and .model (int32 a, b, new_id per merge). */
void bpe_save(const Trainer* trainer, const char* model_path, const char* vocab_path);

/* ---- Unigram symbols bound by cbase.py:59-71 (stubs: return failure / NULL) ------------- */
void* trainerCreate(int vocab_size, float character_coverage, int max_piece_length, int seed_size);
void trainerDestroy(void* trainer);
int addTextToTrainer(void* trainer, const char* text);  /* returns false */
int preprocessTexts(void* trainer);
int extractInitialSubwords(void* trainer);
float computeLoss(void* trainer, char** texts, int n);
double computeTokenLoss(void* trainer, const char* token, char** texts, int n);
int pruneVocabStep(void* trainer, char** texts, int n, double ratio);
int updateTokenScores(void* trainer, char** texts, int n);
int trainUnigram(void* trainer, char** texts, int n, int iterations);
int getVocab(void* trainer, char*** tokens, double** scores, int* n);
int saveVocab(void* trainer, const char* path);
int loadVocab(void* trainer, const char* path);

/* ---- extensions ------------------------------------------------------------------------ */
/* Options (also read from the environment at create_trainer as SHREDWORD_<KEY>):
 *   layout = types | stream     device word table: distinct words weighted by count (default)
 *                               or every occurrence in corpus order with weight 1
 *   log    = 0 | 1 | 2          quiet / summary (default) / reference-style per-merge lines
 *   trace  = <path>             "M a b freq new_id" / "B batch done heap top" trace file
 *   timing = 0 | 1              per-kernel HIP-event timing (shred_get_stats)
 *   device = <ordinal>          HIP device (default: LOCAL_RANK or 0)
 *   merge_groups = <n>          k_merge grid cap (tuning; after load_corpus)
 *   speculate = 0 | 1           speculation (default 1; results are identical either way): the
 *                               merge guessed to come next (from the heap) runs on the device
 *                               while the host consumes the current one; a wrong guess is rolled
 *                               back exactly on the device
 *   chain = <n>                 instead of one guess beside each merge, run the selected merge and
 *                               up to n-1 guessed successors in one launch (default 1 = off, at
 *                               most 8)
 *   exchange = local | off      test: run the multi-GPU records exchange over a single-rank RCCL
 *                               communicator (before load_corpus)
 *   resident = 0 | 1            LDS-resident merge loop (default 1): when the distinct-word
 *                               table fits the chip's LDS, the merge loop runs as one persistent
 *                               launch holding the table in LDS (results are identical either way)
 *   spec_depth = 1 | 2 | 3      resident loop: guessed merges in flight behind the current merge
 *                               (default 1, or env SHREDWORD_SPEC_DEPTH; a wrong guess undoes every
 *                               guess after it; results are identical at any depth)
 *   gpu_load = 0 | 1            count the corpus words on the device at load_corpus (default 1;
 *                               types layout, files without NUL bytes; same table either way)
 *   exchange_bucket = <n>       multi-GPU: records per rank in the fixed all-gather bucket
 *                               (default 1024; larger record sets take a second round)
 *   dist = auto | replicate | exchange
 *                               multi-GPU mode (before load_corpus; default auto = exchange for
 *                               the stream layout, replicate for types): replicate shards the
 *                               load (each rank counts its byte range, word lists all-gathered and
 *                               merged) and runs the merge loop on every rank over the full word
 *                               table with no per-merge collective; exchange shards the word table
 *                               and all-gathers each merge's neighbour records (RCCL over xGMI).
 *                               Output bytes are identical in every mode and world size.
 *   tiebreak = exact|device     merge selection of train(): exact (default) replays the reference's
 *                               heap (bit-exact files); device (opt-in, NOT bit-exact) selects every
 *                               merge on the GPU inside the indexed loop, with no host round trip per
 *                               merge: the pair of largest count, ties to the smaller (first, second)
 *                               key (env SHREDWORD_TIEBREAK; types layout, one GPU)
 *   index = 0 | 1, hybrid = 0 | 1, switch_occ = <n>
 *                               the indexed merge loop (k_word_loop) takes over from k_resident once
 *                               a window of merges changed fewer than switch_occ entries (defaults
 *                               1, 1, 4000; results are identical on every path)
 *   early_guess = 0 | 1, early_max_records = <n>
 *                               post the guess for merge X+2 once X is applied (default 0)
 *   apply_helper = 0 | 1        a second host thread prepares the guessed merge's changes (default 0)
 *   finalize = <n>              K4 on the device: merges with <= n delta records leave k_word_loop as
 *                               changes combined per pair key in the reference's application order
 *                               (default 0 = off; identical results)
 *   trace_note = <text>         appends a line to the trace file
 *   verify_argmax = <n>         debug (K5 check): every n merges (0 = off, the default; env
 *                               SHREDWORD_VERIFY_ARGMAX) the device recounts the corpus's pairs
 *                               and reduces them (k_pair_max): the host heap's selected frequency
 *                               must be the largest pair count and the pair's own count
 *                               (stats: verify_checks, verify_failures; results are unchanged)
 * Returns 0, or -1 for an unknown key/value. */
int shred_set_option(Trainer* trainer, const char* key, const char* value);
/* Restores the loaded corpus to its unmerged state and forgets merges (benchmark repeats). */
int shred_reset(Trainer* trainer);
/* The sharded load (dist=replicate) over a caller-supplied all-gather instead of RCCL (host-side
 * collectives, e.g. torch.distributed gloo): later load_corpus calls count only byte range `rank`
 * of `world` on this trainer's device, and `gather(ctx, send, nbytes, &out_bytes)` must return
 * every rank's buffer concatenated in rank order (valid until its next call), or NULL when the
 * gather failed: load_corpus then fails (-1) instead of building a table from a partial gather.
 * world <= 1 or a NULL gather turns it off.  The stream layout has no sharded load: load_corpus
 * returns -1 when a gather is set with layout=stream.  Returns 0, or -1 for a bad rank. */
typedef const void* (*shred_gather_fn)(void* ctx, const void* send, size_t nbytes, size_t* out_bytes);
int shred_set_load_gather(Trainer* trainer, int rank, int world, shred_gather_fn gather, void* ctx);
/* Diagnostic: runs `iters` device merges of a pair (a, b) that must not occur in the corpus
 * (so nothing changes), timing launch -> records on the host.  Returns mean microseconds per
 * merge, or -1 when the pair occurs / no device. */
double shred_probe_merge(Trainer* trainer, int32_t a, int32_t b, int iters);
/* Diagnostic: launches the merge (a, b) -> next id and immediately rolls it back (the undo path
 * of speculation); the corpus must be unchanged afterwards.  Returns 0, or -1 without a device. */
int shred_probe_rollback(Trainer* trainer, int32_t a, int32_t b);
/* Diagnostic: copies the live token stream (per corpus entry: header INT32_MIN + rank, then its
 * tokens) into out[0 .. cap); returns the full length (call with cap 0 to size), -1 on error. */
int64_t shred_debug_tokens(Trainer* trainer, int32_t* out, size_t cap);

/* Diagnostic: the indexed loop's per-merge trace of the merges collected since timing was last
 * switched on or the stats cleared (set_option timing / clear_stats): 15 uint32 per merge — X,
 * listed words, scanned words, changed words, occurrences, device ns command -> flag, of which
 * lookup ns and scan ns, then wave 0's stamps (ns after the command: pool entries loaded, first
 * run loaded, first word merged, unused), the device ns since the previous merge's flag spent
 * waiting for commands and undoing guesses, and the host ns from post to flag.  Copies
 * min(cap, n) values into out; returns n (-1 on error). */
int64_t shred_index_trace(Trainer* trainer, uint32_t* out, size_t cap);

typedef struct ShredStats {
  double load_seconds, init_seconds, train_seconds;
  double host_select_seconds, host_launch_seconds, host_wait_seconds, host_apply_seconds;
  double merge_kernel_ms, count_kernel_ms;
  double merge_kernel_bytes, count_kernel_bytes;
  uint64_t merge_launches, count_launches;
  uint64_t num_words, num_symbols, num_occurrences, num_merges, heap_size, live_tokens;
  uint64_t device_bytes, num_tiles;
  int32_t layout, world_size;
  uint64_t heap_pops, heap_stale_pops, heap_pushes, delta_records, tiles_visited;
  uint64_t apply_cycles_combine, apply_cycles_order, apply_cycles_walk;
  uint64_t spec_hits, spec_misses;
  uint64_t exchange_overflows; /* multi-GPU: merges whose records needed a second all-gather */
  /* stream layout K1 bulk (k_pair_hist, counts of every occurrence past the first of each type) */
  double hist_kernel_ms, hist_kernel_bytes;
  uint64_t hist_launches;
  /* LDS-resident merge loop: k_resident launches and their summed durations (HIP events) */
  uint64_t resident_launches;
  double resident_ms;
  double resident_latency_us;  /* mean per-merge dispatch -> host flag time (device clock) */
  uint64_t load_on_gpu;        /* 1: the last load_corpus counted its words on the device */
  /* indexed merge loop (k_word_loop, the default for the types layout on one GPU) */
  uint64_t index_on;           /* 1: merges run through the pair -> words index */
  uint64_t index_merges, index_undos, index_launches;
  uint64_t index_candidates;   /* Σ listed words scanned by collected merges */
  uint64_t index_changed;      /* Σ words a collected merge changed */
  uint64_t index_occurrences;  /* Σ occurrences merged */
  double index_ms;             /* Σ k_word_loop launch durations (HIP events) */
  double index_dev_us;         /* Σ per-merge device time, command seen -> flag (device clock) */
  double index_wait_us;        /* Σ per-merge host time, post -> flag seen */
  double index_dev_lookup_us;  /* of index_dev_us: command seen -> word list known */
  double index_dev_scan_us;    /* of index_dev_us: word list known -> every listed word merged */
  uint64_t index_scanned;      /* of index_candidates: words whose runs were read */
  double index_build_us;       /* Σ device time building the merges' pair groups (after their flags) */
  uint64_t index_no_sub;       /* merges whose pair groups were not built (words-of list + filter) */
  uint64_t index_staged;       /* Σ pair-group entries written */
  int64_t index_switch_merge;  /* hybrid: the first merge id of the indexed loop in the last train() (-1: none) */
  double index_switch_ms;      /* hybrid: Σ host time of the resident -> indexed switches */
  uint64_t resident_aborts;    /* k_resident launches that found their grid not co-resident (then off) */
  uint64_t verify_checks;      /* verify_argmax: selections checked against a device recount */
  uint64_t verify_failures;    /* of verify_checks: frequency != device max or != the pair's count */
  /* algorithmic bytes of the two merge loops, collected while timing is on */
  uint64_t resident_merges;    /* merges collected from k_resident */
  double resident_bytes;       /* Σ 4 B x live tokens over those merges (K2: the scan a merge stands for) */
  double resident_kernel_ms;   /* Σ durations of the k_resident launches that merged (HIP events) */
  uint64_t index_run_ints_read;     /* k_word_loop: Σ ints of the scanned words' runs (length + tokens) */
  uint64_t index_run_ints_written;  /* k_word_loop: Σ ints of the changed runs written back */
  uint64_t index_records;           /* k_word_loop: Σ 24-B delta records written to host memory */
  double resident_k3_bytes;    /* k_resident: Σ 8 B x tokens of the tiles a merge rewrote (K3: read + write) */
  /* tiebreak=device (k_word_loop<true>: the device selects its merges) */
  uint64_t sel_merges;         /* merges selected on the device */
  uint64_t sel_launches;       /* launches of the self-selecting loop */
  uint64_t sel_rebuilds;       /* frontier rebuilds (whole chip, between launches) */
  double sel_kernel_ms;        /* Σ launch durations (HIP events) */
  double sel_rebuild_ms;       /* Σ host wall time of the rebuilds */
  double sel_select_us;        /* device: Σ time selecting (frontier scan + argmax) */
  double sel_merge_us;         /* device: Σ time merging and updating the pair table */
  uint64_t sel_table_pairs;    /* pairs in the device pair table at the end */
  uint64_t sel_table_slots;    /* its capacity */
  uint64_t sel_host_merges;    /* tiebreak=device: early merges selected on the host by the same rule
                                  (exact counts) while the whole-chip resident loop runs them */
  uint64_t sel_table_grows;    /* tiebreak=device: pair tables grown 4x between launches */
  /* K4 on the device (k_word_loop finalize_changes, round 5) */
  uint64_t index_raw_records;  /* k_word_loop: Σ delta records before the device's combine */
  uint64_t index_finalized;    /* k_word_loop: merges whose records left as ordered changes */
  double index_dev_out_us;     /* k_word_loop: Σ device time handing the records out (raw or finalized) */
  double index_dev_fin_us;     /*   of which: the finalized merges */
  uint64_t index_fin_records;  /*   their raw records */
  double sel_table_us;         /* tiebreak=device: of sel_merge_us, the pair-table + frontier update */
  uint64_t index_spill_merges; /* k_word_loop: merges whose delta keys overflowed the LDS hash into HBM */
  uint64_t index_spill_keys;   /*   Σ their spilled keys */
  /* host_apply_seconds split (round 6): the records' combine + order on the main thread (merges
   * whose combine ran on the helper thread: helper_adopted), the late correction, the pair-info
   * walk + heap pushes (apply_cycles_walk / apply_cycles_push TSC cycles of it), the early guess,
   * the helper hand-over */
  double host_apply_combine_seconds, host_apply_correct_seconds, host_apply_finish_seconds;
  double host_apply_early_seconds, host_apply_offer_seconds;
  uint64_t helper_adopted, apply_cycles_push;
} ShredStats;
int shred_get_stats(const Trainer* trainer, ShredStats* out);

/* Number of usable HIP devices (0 without a GPU); never initialises more than the runtime. */
int shred_device_count(void);

/* Measurement: achievable HBM bandwidth of `device`, a streaming read and a
 * streaming copy of `bytes`, `reps` timed launches each; GB/s of bytes moved (copy counts read +
 * write).  Returns 0, or -1 without a device / on allocation failure. */
int shred_hbm_probe(int device, size_t bytes, int reps, double* read_gbps, double* copy_gbps);

/* Diagnostic (tests of the resident loop's co-residency check): fills every wave slot of all CUs
 * but `free_cus` with a spinning kernel on its own stream, until shred_release() or
 * `max_seconds`; returns once it runs (NULL on bad arguments).  */
void* shred_occupy(int device, int free_cus, double max_seconds);
void shred_release(void* handle);

/* Multi-GPU (one process per GPU, RCCL over xGMI): rank 0 calls shred_dist_unique_id, the
 * bytes are broadcast out of band (torch.distributed), then every rank calls shred_dist_init
 * before create_trainer.  Trainers then shard the word table and all-reduce the per-merge
 * delta tables.  Returns 0 on success. */
int shred_dist_unique_id(void* out, size_t cap);
int shred_dist_init(int rank, int world_size, const void* unique_id, size_t len, int device);
int shred_dist_finalize(void);
/* Ranks of the communicator shred_dist_init made (ncclCommCount); 0 when there is none. */
int shred_dist_ranks(void);

#ifdef __cplusplus
}
#endif
#endif
