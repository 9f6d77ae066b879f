"""ctypes binding of libtrainer.so (mirrors the reference's shredword/cbase.py).

Library discovery follows the reference (cbase.py:4-26): the first file named ``trainer*`` or
``libtrainer*`` with a shared-library suffix in this package, ``lib/`` below it, or ``../build``;
``SHREDWORD_LIB`` overrides.  The library is loaded with RTLD_GLOBAL (cbase.py:29) and the 8 BPE
plus 13 Unigram symbols are bound at import (cbase.py:50-71), so a library missing any of them
fails here with AttributeError, as with the reference.  The Trainer handle is opaque.
"""
import ctypes
import os
import sysconfig
from ctypes import (POINTER, Structure, c_bool, c_char_p, c_double, c_float, c_int, c_int32, c_int64,
                    c_size_t, c_uint32, c_uint64, c_void_p)


def _get_lib_path():
    env = os.environ.get("SHREDWORD_LIB")
    if env:
        return os.path.abspath(env)
    pkg_dir = os.path.dirname(os.path.abspath(__file__))
    names = ("libtrainer", "trainer")
    exts = [e for e in (".so", ".pyd", ".dll", ".dylib", sysconfig.get_config_var("EXT_SUFFIX")) if e]
    search = [pkg_dir, os.path.join(pkg_dir, "lib"), os.path.join(pkg_dir, "..", "build")]
    for d in search:
        if not os.path.isdir(d):
            continue
        for root, _dirs, files in os.walk(d):
            for f in sorted(files):
                if f.startswith(names) and any(f.endswith(e) for e in exts):
                    return os.path.abspath(os.path.join(root, f))
    available = []
    for d in search:
        if os.path.isdir(d):
            available.extend(os.listdir(d))
    raise FileNotFoundError(f"Could not find trainer library in {search}. Available files: {available}")


_lib_path = _get_lib_path()
lib = ctypes.CDLL(_lib_path, mode=getattr(ctypes, "RTLD_GLOBAL", 0))

MIN_HEAP_SIZE, MAX_OCCS_PER_MERGE, INITIAL_VOCAB_SIZE, INITIAL_STR_SIZE = 4096, 50000, 256, 4096


class BPEConfig(Structure):
    """reference bpe.h:43-48 / cbase.py:47 (24 bytes, offsets 0/8/12/16)."""
    _fields_ = [("target_vocab_size", c_size_t), ("unk_id", c_int32),
                ("character_coverage", c_float), ("min_pair_freq", c_uint64)]


class ShredStats(Structure):
    _fields_ = [("load_seconds", c_double), ("init_seconds", c_double), ("train_seconds", c_double),
                ("host_select_seconds", c_double), ("host_launch_seconds", c_double),
                ("host_wait_seconds", c_double), ("host_apply_seconds", c_double),
                ("merge_kernel_ms", c_double), ("count_kernel_ms", c_double),
                ("merge_kernel_bytes", c_double), ("count_kernel_bytes", c_double),
                ("merge_launches", c_uint64), ("count_launches", c_uint64),
                ("num_words", c_uint64), ("num_symbols", c_uint64), ("num_occurrences", c_uint64),
                ("num_merges", c_uint64), ("heap_size", c_uint64), ("live_tokens", c_uint64),
                ("device_bytes", c_uint64), ("num_tiles", c_uint64),
                ("layout", c_int32), ("world_size", c_int32),
                ("heap_pops", c_uint64), ("heap_stale_pops", c_uint64), ("heap_pushes", c_uint64),
                ("delta_records", c_uint64), ("tiles_visited", c_uint64),
                ("apply_cycles_combine", c_uint64), ("apply_cycles_order", c_uint64),
                ("apply_cycles_walk", c_uint64),
                ("spec_hits", c_uint64), ("spec_misses", c_uint64),
                ("exchange_overflows", c_uint64),
                ("hist_kernel_ms", c_double), ("hist_kernel_bytes", c_double), ("hist_launches", c_uint64),
                ("resident_launches", c_uint64), ("resident_ms", c_double), ("resident_latency_us", c_double),
                ("load_on_gpu", c_uint64),
                ("index_on", c_uint64), ("index_merges", c_uint64), ("index_undos", c_uint64),
                ("index_launches", c_uint64), ("index_candidates", c_uint64), ("index_changed", c_uint64),
                ("index_occurrences", c_uint64), ("index_ms", c_double), ("index_dev_us", c_double),
                ("index_wait_us", c_double),
                ("index_dev_lookup_us", c_double), ("index_dev_scan_us", c_double),
                ("index_scanned", c_uint64), ("index_build_us", c_double), ("index_no_sub", c_uint64),
                ("index_staged", c_uint64), ("index_switch_merge", c_int64), ("index_switch_ms", c_double),
                ("resident_aborts", c_uint64), ("verify_checks", c_uint64), ("verify_failures", c_uint64),
                ("resident_merges", c_uint64), ("resident_bytes", c_double), ("resident_kernel_ms", c_double),
                ("index_run_ints_read", c_uint64), ("index_run_ints_written", c_uint64),
                ("index_records", c_uint64), ("resident_k3_bytes", c_double),
                ("sel_merges", c_uint64), ("sel_launches", c_uint64), ("sel_rebuilds", c_uint64),
                ("sel_kernel_ms", c_double), ("sel_rebuild_ms", c_double), ("sel_select_us", c_double),
                ("sel_merge_us", c_double), ("sel_table_pairs", c_uint64), ("sel_table_slots", c_uint64),
                ("sel_host_merges", c_uint64), ("sel_table_grows", c_uint64),
                ("index_raw_records", c_uint64), ("index_finalized", c_uint64),
                ("index_dev_out_us", c_double), ("index_dev_fin_us", c_double), ("index_fin_records", c_uint64),
                ("sel_table_us", c_double), ("index_spill_merges", c_uint64), ("index_spill_keys", c_uint64),
                ("host_apply_combine_seconds", c_double), ("host_apply_correct_seconds", c_double),
                ("host_apply_finish_seconds", c_double), ("host_apply_early_seconds", c_double),
                ("host_apply_offer_seconds", c_double), ("helper_adopted", c_uint64),
                ("apply_cycles_push", c_uint64)]


Trainer = c_void_p

lib.create_trainer.argtypes, lib.create_trainer.restype = [POINTER(BPEConfig)], Trainer
lib.bpe_trainer_destroy.argtypes, lib.bpe_trainer_destroy.restype = [Trainer], None
lib.bpe_init.argtypes, lib.bpe_init.restype = [Trainer], None
lib.bpe_count_bigrams.argtypes, lib.bpe_count_bigrams.restype = [Trainer], None
lib.bpe_load_corpus.argtypes, lib.bpe_load_corpus.restype = [Trainer, c_char_p], c_int
lib.bpe_merge_batch.argtypes, lib.bpe_merge_batch.restype = [Trainer, c_int], c_int
lib.bpe_train.argtypes, lib.bpe_train.restype = [Trainer], c_int
lib.bpe_save.argtypes, lib.bpe_save.restype = [Trainer, c_char_p, c_char_p], None

lib.trainerCreate.argtypes, lib.trainerCreate.restype = [c_int, c_float, c_int, c_int], c_void_p
lib.trainerDestroy.argtypes, lib.trainerDestroy.restype = [c_void_p], None
lib.addTextToTrainer.argtypes, lib.addTextToTrainer.restype = [c_void_p, c_char_p], c_bool
lib.preprocessTexts.argtypes, lib.preprocessTexts.restype = [c_void_p], c_bool
lib.extractInitialSubwords.argtypes, lib.extractInitialSubwords.restype = [c_void_p], c_bool
lib.computeLoss.argtypes, lib.computeLoss.restype = [c_void_p, POINTER(c_char_p), c_int], c_float
lib.computeTokenLoss.argtypes, lib.computeTokenLoss.restype = [c_void_p, c_char_p, POINTER(c_char_p), c_int], c_double
lib.pruneVocabStep.argtypes, lib.pruneVocabStep.restype = [c_void_p, POINTER(c_char_p), c_int, c_double], c_bool
lib.updateTokenScores.argtypes, lib.updateTokenScores.restype = [c_void_p, POINTER(c_char_p), c_int], c_bool
lib.trainUnigram.argtypes, lib.trainUnigram.restype = [c_void_p, POINTER(c_char_p), c_int, c_int], c_bool
lib.getVocab.argtypes, lib.getVocab.restype = [c_void_p, POINTER(POINTER(c_char_p)), POINTER(POINTER(c_double)), POINTER(c_int)], c_bool
lib.saveVocab.argtypes, lib.saveVocab.restype = [c_void_p, c_char_p], c_bool
lib.loadVocab.argtypes, lib.loadVocab.restype = [c_void_p, c_char_p], c_bool

# extensions (include/shredword_bpe.h)
lib.shred_set_option.argtypes, lib.shred_set_option.restype = [Trainer, c_char_p, c_char_p], c_int
lib.shred_reset.argtypes, lib.shred_reset.restype = [Trainer], c_int
# shred_gather_fn: (ctx, send, nbytes, size_t* out_bytes) -> every rank's bytes, concatenated
GATHER_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                             ctypes.POINTER(ctypes.c_size_t))
lib.shred_set_load_gather.argtypes = [Trainer, c_int, c_int, GATHER_FN, ctypes.c_void_p]
lib.shred_set_load_gather.restype = c_int
lib.shred_probe_merge.argtypes, lib.shred_probe_merge.restype = [Trainer, c_int32, c_int32, c_int], c_double
if hasattr(lib, "shred_probe_rollback"):  # diagnostics (absent from older builds)
    lib.shred_probe_rollback.argtypes, lib.shred_probe_rollback.restype = [Trainer, c_int32, c_int32], c_int
    lib.shred_debug_tokens.argtypes, lib.shred_debug_tokens.restype = [Trainer, POINTER(c_int32), c_size_t], c_int64
    lib.shred_index_trace.argtypes, lib.shred_index_trace.restype = [Trainer, POINTER(c_uint32), c_size_t], c_int64
lib.shred_get_stats.argtypes, lib.shred_get_stats.restype = [Trainer, POINTER(ShredStats)], c_int
lib.shred_device_count.argtypes, lib.shred_device_count.restype = [], c_int
lib.shred_hbm_probe.argtypes = [c_int, c_size_t, c_int, POINTER(c_double), POINTER(c_double)]
lib.shred_hbm_probe.restype = c_int
lib.shred_occupy.argtypes, lib.shred_occupy.restype = [c_int, c_int, c_double], c_void_p
lib.shred_release.argtypes, lib.shred_release.restype = [c_void_p], None
lib.shred_dist_unique_id.argtypes, lib.shred_dist_unique_id.restype = [c_void_p, c_size_t], c_int
lib.shred_dist_init.argtypes, lib.shred_dist_init.restype = [c_int, c_int, c_void_p, c_size_t, c_int], c_int
lib.shred_dist_finalize.argtypes, lib.shred_dist_finalize.restype = [], c_int
lib.shred_dist_ranks.argtypes, lib.shred_dist_ranks.restype = [], c_int

# encoder (include/shredword_encode.h)
Encoder = c_void_p
lib.shred_encoder_create.argtypes = [POINTER(c_int32), c_size_t, POINTER(c_int32), c_int]
lib.shred_encoder_create.restype = Encoder
lib.shred_encoder_load.argtypes, lib.shred_encoder_load.restype = [c_char_p, c_char_p, c_int32, c_int], Encoder
lib.shred_encoder_destroy.argtypes, lib.shred_encoder_destroy.restype = [Encoder], None
lib.shred_encoder_info.argtypes = [Encoder, POINTER(c_size_t), POINTER(c_int32)]
lib.shred_encoder_info.restype = c_int
lib.shred_encode.argtypes = [Encoder, c_void_p, c_size_t, c_void_p, c_size_t]
lib.shred_encode.restype = c_int64
lib.shred_encode_device.argtypes = [Encoder, c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, POINTER(c_double)]
lib.shred_encode_device.restype = c_int64
lib.shred_decode.argtypes = [Encoder, c_void_p, c_size_t, c_void_p, c_size_t]
lib.shred_decode.restype = c_int64
