"""GPU tests of the encoder through the C ABI (include/shredword_encode.h):

* bit-exact id sequences against the oracle encoder (oracle/encode_oracle.c) on every golden
  corpus with the reference's own .model, and id counts equal to the reference's .vocab column;
* the encoder fed a model the GPU trainer just wrote (train -> save -> encode the training
  corpus -> counts == .vocab), at 32 MB;
* the word cache (default) and the direct kernel on the same inputs; a cache overflow (more
  distinct words than slots) reruns exactly on the direct path;
* edge cases: empty text, delimiters only, no trailing delimiter, word lengths around the LDS
  strip (31/32/33) and the limit (1024 ok, 1025 rejected), random bytes incl. NUL and 0x80-0xFF,
  unaligned device text, a too-small output, the coverage byte map, decode round trips.
"""
import ctypes
import os

import numpy as np
import pytest

import corpora
from conftest import golden_cases
from encode_ref import derived_byte_map, id_counts, model_merges, oracle_encode, token_bytes, vocab_freqs

pytestmark = pytest.mark.gpu

CASES = [c for c in golden_cases() if not c.startswith("cli_")]


def _enc_from(merges, byte_map=None):
    from shredword.encoder import BPEEncoder
    return BPEEncoder.from_merges(merges, byte_map)


@pytest.mark.parametrize("name", CASES)
def test_golden_encode_matches_oracle(name, case_corpus, tmp_path):
    from shredword.encoder import BPEEncoder
    case, path = case_corpus(name)
    text = open(path, "rb").read()
    merges = model_merges(case["model_bytes"])
    toks = token_bytes(merges)
    freqs = vocab_freqs(case["vocab_bytes"], toks)
    unk = case["config"]["unk_id"]
    (tmp_path / "g.model").write_bytes(case["model_bytes"])
    (tmp_path / "g.vocab").write_bytes(case["vocab_bytes"])
    enc = BPEEncoder(str(tmp_path / "g.model"), str(tmp_path / "g.vocab"), unk_id=unk)
    bm = derived_byte_map(merges, freqs, unk)
    assert np.array_equal(enc.byte_map, bm)
    assert enc.num_merges == len(merges)
    with enc:
        try:
            want = oracle_encode(merges, bm, text)
        except ValueError:  # a word longer than the encoder's limit: both reject it
            with pytest.raises(ValueError):
                enc.encode(text)
            return
        got = enc.encode(text)
        assert got.dtype == np.int32 and np.array_equal(got, want)
        if b"\0" not in text:
            assert np.array_equal(id_counts(got, len(toks)), freqs)


def test_train_save_encode_roundtrip(tmp_path):
    """The GPU trainer's own outputs: encoding its training corpus reproduces its .vocab counts."""
    from shredword.encoder import BPEEncoder
    from shredword.trainer import BPETrainer
    corpus = tmp_path / "c.txt"
    corpora.gen_synthetic(str(corpus), 32_000_000, 11, "utf8")
    t = BPETrainer(vocab_size=4000, min_pair_freq=20)
    t.set_option("log", 0)
    t.load_corpus(str(corpus))
    t.train()
    t.save(str(tmp_path / "t.model"), str(tmp_path / "t.vocab"))
    t.destroy()
    enc = BPEEncoder(str(tmp_path / "t.model"), str(tmp_path / "t.vocab"), unk_id=0)
    text = corpus.read_bytes()
    ids = enc.encode(text)
    merges = model_merges((tmp_path / "t.model").read_bytes())
    toks = token_bytes(merges)
    freqs = vocab_freqs((tmp_path / "t.vocab").read_bytes(), toks)
    assert np.array_equal(id_counts(ids, len(toks)), freqs)
    # the device path on an HBM-resident tensor gives the same ids
    import torch
    d = torch.from_numpy(np.frombuffer(text, dtype=np.uint8).copy()).cuda()
    dids, ms = enc.encode_device(d)
    assert ms > 0 and np.array_equal(dids.cpu().numpy(), ids)
    enc.destroy()


def _random_merges(rng, alphabet, M):
    """A trainer-like merge list over `alphabet`: operands drawn from ids that exist."""
    ids = list(alphabet)
    out = []
    seen = set()
    while len(out) < M:
        a, b = int(rng.choice(ids)), int(rng.choice(ids))
        if (a, b) in seen:
            continue
        seen.add((a, b))
        out.append([a, b, 256 + len(out)])
        ids.append(256 + len(out) - 1)
    return np.array(out, dtype=np.int32)


@pytest.mark.parametrize("cache", ["1", "0"])
def test_edge_cases_against_oracle(cache, monkeypatch):
    """Both paths: the word cache (default) and the direct per-occurrence kernel."""
    monkeypatch.setenv("SHREDWORD_ENCODE_CACHE", cache)
    rng = np.random.default_rng(5)
    alpha = [97, 98, 99, 100]
    merges = _random_merges(rng, alpha, 300)
    enc = _enc_from(merges)
    words = [bytes(rng.choice(alpha, size=L).astype(np.uint8)) for L in
             (1, 2, 3, 31, 32, 33, 34, 63, 64, 65, 100, 500, 1023, 1024)]
    cases = [b"", b" ", b" \t\r\n" * 100, b"a", b"ab", b"abcd", words[3], b" ".join(words),
             b"\n".join(words) + b"\n", b"\t".join(words[::-1]),
             b"a" * 1024, b"ab" * 512, b" " * 31 + b"abc",
             bytes(rng.integers(0, 256, size=100_000, dtype=np.uint8).tolist()).replace(b"\n", b"\n" * 1)]
    # many words in one span and spans that straddle block boundaries (4096 B per workgroup)
    cases.append(b"a b " * 5000)
    cases.append(b"".join(bytes(rng.choice(alpha, size=int(rng.integers(1, 40))).astype(np.uint8)) + b" "
                          for _ in range(20000)))
    for text in cases:
        want = oracle_encode(merges, None, text)
        got = enc.encode(text)
        assert np.array_equal(got, want), (len(text), text[:40])
        if b"\0" not in text:
            assert enc.decode(got) == b"".join(text.split(b" ")).replace(b"\t", b"").replace(b"\r", b"").replace(b"\n", b"")
    with pytest.raises(ValueError):
        enc.encode(b"x " + b"a" * 1025 + b" y")
    # a too-small output buffer is refused, not overrun
    from shredword.cbase import lib
    buf = np.frombuffer(b"ab cd ab", dtype=np.uint8)
    out = np.full(8, -7, dtype=np.int32)
    full = lib.shred_encode(enc.enc, buf.ctypes.data, buf.size, out.ctypes.data, out.size)
    assert full > 0
    out[:] = -7
    assert lib.shred_encode(enc.enc, buf.ctypes.data, buf.size, out.ctypes.data, full - 1) == -2
    assert (out == -7).all()
    enc.destroy()


@pytest.mark.parametrize("cache", ["1", "0"])
def test_unaligned_device_text_and_byte_map(cache, monkeypatch):
    monkeypatch.setenv("SHREDWORD_ENCODE_CACHE", cache)
    import torch
    rng = np.random.default_rng(9)
    alpha = list(range(0x61, 0x6b))
    merges = _random_merges(rng, alpha, 1000)
    bm = np.arange(256, dtype=np.int32)
    bm[0x6a] = -1        # a dropped byte -> unk (never merges)
    bm[0x20] = 0x20
    enc = _enc_from(merges, bm)
    text = b"".join(bytes(rng.choice(alpha, size=int(rng.integers(1, 50))).astype(np.uint8)) + b" "
                    for _ in range(50000))
    want = oracle_encode(merges, bm, text)
    big = torch.from_numpy(np.frombuffer(b"x" + text, dtype=np.uint8).copy()).cuda()
    got, _ = enc.encode_device(big[1:])  # 1-byte offset: the unaligned load path
    assert np.array_equal(got.cpu().numpy(), want)
    assert (want == -1).any()
    got2, _ = enc.encode_device(big[:1])  # one word, one byte
    assert got2.cpu().tolist() == [ord("x")]
    enc.destroy()


def test_invalid_models_are_rejected(tmp_path):
    from shredword.encoder import BPEEncoder
    with pytest.raises(RuntimeError):
        BPEEncoder.from_merges([[97, 98, 300]])          # new id must be 256 + m
    with pytest.raises(RuntimeError):
        BPEEncoder.from_merges([[97, 256, 256]])         # operand not yet defined
    (tmp_path / "bad.model").write_bytes(b"\1\2\3")
    with pytest.raises(RuntimeError):
        BPEEncoder(str(tmp_path / "bad.model"))
    (tmp_path / "m.model").write_bytes(np.array([[97, 98, 256]], np.int32).tobytes())
    (tmp_path / "v.vocab").write_bytes(b"wrong 1\n")
    with pytest.raises(RuntimeError):
        BPEEncoder(str(tmp_path / "m.model"), str(tmp_path / "v.vocab"))
    e = BPEEncoder(str(tmp_path / "m.model"))              # identity byte map without a .vocab
    assert e.encode(b"abab ba").tolist() == [256, 256, 98, 97]
    e.destroy()


def test_word_cache_overflow_falls_back_exactly():
    """1.5 M distinct words overflow the 1 M-slot word cache: the call reruns on the direct path."""
    rng = np.random.default_rng(3)
    alpha = list(range(0x30, 0x3a))
    merges = _random_merges(rng, alpha, 300)
    words = rng.permutation(1_500_000)
    text = ("\n".join(f"{w:07d}" for w in words) + "\n").encode()
    enc = _enc_from(merges)
    want = oracle_encode(merges, None, text)
    assert np.array_equal(enc.encode(text), want)
    enc.destroy()


def test_repeated_pairs_past_16_bit_ids():
    """A merge list with repeated pairs: 2 distinct pairs but ranks up to 65301 (ids past
    0xFFFF), so the 16-bit LDS packing must be off (it is decided from the largest rank)."""
    M = 65302
    merges = np.empty((M, 3), dtype=np.int32)
    merges[:, 0], merges[:, 1] = 97, 98
    merges[:, 2] = 256 + np.arange(M)
    merges[-1, :2] = (256, 99)  # rank 65301 -> id 65557
    enc = _enc_from(merges)
    for cache in ("1", "0"):
        os.environ["SHREDWORD_ENCODE_CACHE"] = cache
        try:
            text = b"abc ab abcabc ca " * 1000
            assert np.array_equal(enc.encode(text), oracle_encode(merges, None, text))
            assert enc.encode(b"abc").tolist() == [65557]
        finally:
            del os.environ["SHREDWORD_ENCODE_CACHE"]
    enc.destroy()


def test_word_arena_overflow_falls_back_exactly():
    """Distinct long words whose ids + bytes exceed the arena (one int per text byte): the
    word-cache call reruns exactly on the direct path."""
    rng = np.random.default_rng(4)
    alpha = [97, 98, 99, 100]
    merges = _random_merges(rng, alpha, 200)
    text = b" ".join(bytes(rng.choice(alpha, size=1000).astype(np.uint8)) for _ in range(2000)) + b" "
    enc = _enc_from(merges)
    assert np.array_equal(enc.encode(text), oracle_encode(merges, None, text))
    enc.destroy()


def test_host_text_in_pieces(monkeypatch):
    """encode() of host text in small pieces cut at delimiters gives the ids of one call, and a
    word past the limit at a piece boundary is still rejected."""
    rng = np.random.default_rng(8)
    alpha = [97, 98, 99]
    merges = _random_merges(rng, alpha, 400)
    enc = _enc_from(merges)
    text = b"".join(bytes(rng.choice(alpha, size=int(rng.integers(1, 60))).astype(np.uint8)) +
                    bytes([int(rng.choice([9, 10, 13, 32]))]) for _ in range(40000))
    want = enc.encode(text)
    assert np.array_equal(want, oracle_encode(merges, None, text))
    monkeypatch.setenv("SHREDWORD_ENCODE_PIECE", "5000")
    assert np.array_equal(enc.encode(text), want)
    with pytest.raises(ValueError):
        enc.encode(b"ab " * 3000 + b"a" * 1100 + b" ab")
    enc.destroy()


def test_device_mismatch_is_refused():
    import torch
    enc = _enc_from(np.array([[97, 98, 256]], np.int32))
    with pytest.raises(ValueError):
        enc.encode_device(torch.zeros(4, dtype=torch.uint8))  # host tensor
    t = torch.tensor(list(b"ab ab"), dtype=torch.uint8, device="cuda:0")
    with pytest.raises(ValueError):
        enc.encode_device(t, out=torch.empty(8, dtype=torch.int64, device="cuda:0"))
    assert enc.encode_device(t)[0].cpu().tolist() == [256, 256]
    enc.destroy()
