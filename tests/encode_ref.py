"""Test helpers for the encoder: the oracle encoder (oracle/encode_oracle.c, the
checker — never the thing measured), and readers of the reference's .model / .vocab formats
(shredword/csrc/bpe/bpe.cpp:388-432) restated here for the tests."""
import ctypes
import os
import subprocess

import numpy as np

from conftest import ORACLE

_LIB = None


def oracle_lib():
    global _LIB
    if _LIB is None:
        subprocess.run(["make", "-s", "-C", ORACLE, "port"], check=True)
        _LIB = ctypes.CDLL(os.path.join(ORACLE, "_build", "libbpe_oracle.so"))
        _LIB.or_encode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        _LIB.or_encode.restype = ctypes.c_int64
    return _LIB


def oracle_encode(merges, byte_map, text: bytes) -> np.ndarray:
    m = np.ascontiguousarray(np.asarray(merges, dtype=np.int32).reshape(-1, 3))
    bm = None if byte_map is None else np.ascontiguousarray(byte_map, dtype=np.int32)
    buf = np.frombuffer(text, dtype=np.uint8) if len(text) else np.zeros(1, np.uint8)
    out = np.empty(max(1, len(text)), dtype=np.int32)
    r = oracle_lib().or_encode(m.ctypes.data, m.shape[0], None if bm is None else bm.ctypes.data, buf.ctypes.data,
                               len(text), out.ctypes.data, out.size)
    if r < 0:
        raise ValueError(f"oracle encode failed ({r})")
    return out[:r].copy()


def model_merges(model_bytes: bytes) -> np.ndarray:
    """.model: int32 triples (first, second, 256 + m), bpe.cpp:419-427."""
    return np.frombuffer(model_bytes, dtype=np.int32).reshape(-1, 3).copy()


def token_bytes(merges) -> list:
    toks = [bytes([b]) for b in range(256)]
    for a, b, _ in np.asarray(merges).reshape(-1, 3):
        toks.append(toks[a] + toks[b])
    return toks


def vocab_freqs(vocab_bytes: bytes, toks) -> np.ndarray:
    """.vocab record i = token i as a C string (NUL bytes vanish) + ' ' + freq + '\\n' (bpe.cpp:417)."""
    pos, out = 0, np.zeros(len(toks), dtype=np.uint64)
    for i, t in enumerate(toks):
        t = t.replace(b"\0", b"")
        assert vocab_bytes[pos:pos + len(t) + 1] == t + b" ", f"vocab record {i} does not match the model"
        pos += len(t) + 1
        end = vocab_bytes.index(b"\n", pos)
        out[i] = int(vocab_bytes[pos:end])
        pos = end + 1
    assert pos == len(vocab_bytes)
    return out


def derived_byte_map(merges, freqs, unk_id) -> np.ndarray:
    """Bytes with .vocab frequency 0 that no merge uses were dropped by the coverage rule."""
    used = set(int(x) for x in np.asarray(merges).reshape(-1, 3)[:, :2].ravel() if x < 256)
    bm = np.arange(256, dtype=np.int32)
    for b in range(256):
        if freqs[b] == 0 and b not in used:
            bm[b] = unk_id
    return bm


def id_counts(ids, n_tokens) -> np.ndarray:
    ids = np.asarray(ids)
    return np.bincount(ids[(ids >= 0) & (ids < n_tokens)], minlength=n_tokens).astype(np.uint64)
