"""ctypes wrapper of the test-only CPU harness (tests/native): product host code + kernel emulation."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "native", "_build", "libhostharness.so")

EXCHANGE_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                               ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t)
# records all-gather: (ctx, send, nbytes, out_bytes*) -> concatenated bytes (callback-owned)
GATHER_CB = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                             ctypes.POINTER(ctypes.c_size_t))


def load():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "native")], check=True)
    lib = ctypes.CDLL(LIB)
    lib.hh_open.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_float, ctypes.c_uint64,
                            ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.hh_open.restype = ctypes.c_void_p
    lib.hh_open_sharded.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_float, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_int, GATHER_CB, ctypes.c_void_p]
    lib.hh_open_sharded.restype = ctypes.c_void_p
    lib.hh_close.argtypes = [ctypes.c_void_p]
    lib.hh_set_exchange.argtypes = [ctypes.c_void_p, EXCHANGE_CB, GATHER_CB, ctypes.c_void_p]
    lib.hh_train.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    lib.hh_train.restype = ctypes.c_int
    lib.hh_merge_batch.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hh_merge_batch.restype = ctypes.c_int
    lib.hh_init.argtypes = [ctypes.c_void_p]
    lib.hh_create.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.c_float, ctypes.c_uint64]
    lib.hh_create.restype = ctypes.c_void_p
    lib.hh_load.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    lib.hh_load.restype = ctypes.c_int
    lib.hh_count.argtypes = [ctypes.c_void_p]
    lib.hh_set_tiebreak_device.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hh_set_device_phase.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hh_host_phase_merges.argtypes = [ctypes.c_void_p]
    lib.hh_host_phase_merges.restype = ctypes.c_uint64
    lib.hh_helper_used.argtypes = [ctypes.c_void_p]
    lib.hh_helper_used.restype = ctypes.c_uint64
    lib.hh_set_apply_helper.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hh_set_verify.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hh_verify_failures.argtypes = [ctypes.c_void_p]
    lib.hh_verify_failures.restype = ctypes.c_uint64
    lib.hh_set_early_guess.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hh_set_verify_exact.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for fn in ("hh_exact_checks", "hh_exact_failures"):
        getattr(lib, fn).argtypes = [ctypes.c_void_p]
        getattr(lib, fn).restype = ctypes.c_uint64
    lib.hh_set_max_guesses.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hh_post_guesses.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.c_int32]
    lib.hh_post_guesses.restype = ctypes.c_int
    lib.hh_set_trace.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    lib.hh_trace_line.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    lib.hh_save.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    for fn in ("hh_num_words", "hh_num_symbols", "hh_num_tiles", "hh_live_tokens", "hh_heap_size",
               "hh_distinct_bytes", "hh_kept_bytes", "hh_tiles_visited"):
        getattr(lib, fn).argtypes = [ctypes.c_void_p]
        getattr(lib, fn).restype = ctypes.c_uint64
    lib.hh_visit_hist.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint64]
    lib.hh_visit_hist.restype = ctypes.c_uint64
    lib.hh_match_hist.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint64]
    lib.hh_match_hist.restype = ctypes.c_uint64
    lib.hh_set_chain.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.hh_chain_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.hh_chain_hist.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    lib.hh_spec.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    lib.hh_word.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                            ctypes.POINTER(ctypes.c_uint64)]
    lib.hh_word.restype = ctypes.c_uint64
    return lib


def open_case(lib, corpus, cfg, layout="types", rank=0, world=1):
    h = lib.hh_open(corpus.encode(), cfg["vocab_size"], cfg["unk_id"], cfg["character_coverage"],
                    cfg["min_pair_freq"], 1 if layout == "stream" else 0, rank, world)
    if not h:
        raise IOError(corpus)
    return h


def table_fingerprint(lib, h):
    """md5 over the word table in rank order: every spelling with its count (and the byte cut)."""
    import hashlib
    m = hashlib.md5()
    buf = ctypes.create_string_buffer(1 << 16)
    cnt = ctypes.c_uint64()
    for i in range(lib.hh_num_words(h)):
        n = lib.hh_word(h, i, buf, len(buf), ctypes.byref(cnt))
        m.update(buf.raw[:n] + b"\0" + str(cnt.value).encode() + b"\n")
    m.update(f"{lib.hh_num_symbols(h)} {lib.hh_distinct_bytes(h)} {lib.hh_kept_bytes(h)}".encode())
    return m.hexdigest()
