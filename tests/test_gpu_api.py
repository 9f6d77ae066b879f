"""GPU tests of the drop-in API beyond the goldens.

* the reference's own pytest suite (test/test_bpe.py:35-65) on the MI355X trainer;
* run-to-run determinism (reset + retrain, and a fresh trainer) — device atomics are order-free;
* bpe_init + bpe_merge_batch through the C ABI;
* a medium corpus against the CPU oracle (bit-exact) in both layouts;
* speculation: k_unmerge restores the stream exactly; speculation on/off in lock step;
* the C2 workload at full size (1 GB) through size-independent invariants: byte conservation
  (Σ freq(token) x len(token) = Σ word bytes x count) and non-increasing merge frequencies.
"""
import os
import subprocess

import numpy as np
import pytest

import corpora
from conftest import ORACLE

pytestmark = pytest.mark.gpu


def _trainer(**kw):
    from shredword.trainer import BPETrainer
    t = BPETrainer(**kw)
    t.set_option("log", 0)
    return t


@pytest.fixture(scope="module")
def small_corpus(tmp_path_factory):
    p = tmp_path_factory.mktemp("small") / "corpus.txt"
    corpora.write_small_corpus(str(p))
    return str(p)


def test_reference_train_and_save(small_corpus, tmp_path):
    """reference test/test_bpe.py:35-54"""
    model, vocab = tmp_path / "bpe.model", tmp_path / "bpe.vocab"
    t = _trainer(vocab_size=300, min_pair_freq=2)
    t.load_corpus(small_corpus)
    merges = t.train()
    assert merges > 0
    t.save(str(model), str(vocab))
    t.destroy()
    assert model.exists() and vocab.exists()
    assert model.stat().st_size == 12 * merges
    # one line per token; token 10's spelling is itself a newline
    assert vocab.read_bytes().count(b"\n") == 256 + merges + 1


def test_reference_zero_merge_expected(small_corpus):
    """reference test/test_bpe.py:56-65"""
    t = _trainer(vocab_size=50, min_pair_freq=1000)
    t.load_corpus(small_corpus)
    assert t.train() == 0
    t.destroy()


def _train_bytes(t, tmp_path, tag):
    n = t.train()
    m, v = tmp_path / f"{tag}.model", tmp_path / f"{tag}.vocab"
    t.save(str(m), str(v))
    return n, m.read_bytes(), v.read_bytes()


def test_deterministic_rerun(tmp_path):
    corpus = str(tmp_path / "c.txt")
    corpora.gen_synthetic(corpus, 4_000_000, 21, "utf8")
    t = _trainer(vocab_size=3000, min_pair_freq=2)
    t.load_corpus(corpus)
    first = _train_bytes(t, tmp_path, "a")
    t.reset()
    second = _train_bytes(t, tmp_path, "b")
    t.destroy()
    t2 = _trainer(vocab_size=3000, min_pair_freq=2)
    t2.load_corpus(corpus)
    third = _train_bytes(t2, tmp_path, "c")
    t2.destroy()
    assert first == second == third


def test_init_and_merge_batch_abi(small_corpus, tmp_path):
    from shredword.cbase import lib
    ref = _trainer(vocab_size=300, min_pair_freq=2)
    ref.load_corpus(small_corpus)
    n_ref, model_ref, vocab_ref = _train_bytes(ref, tmp_path, "ref")
    ref.destroy()
    t = _trainer(vocab_size=300, min_pair_freq=2)
    t.load_corpus(small_corpus)
    lib.bpe_init(t.trainer)
    done = 0
    while done < n_ref:
        k = lib.bpe_merge_batch(t.trainer, min(5, n_ref - done))
        assert k > 0
        done += k
    m, v = tmp_path / "mb.model", tmp_path / "mb.vocab"
    t.save(str(m), str(v))
    t.destroy()
    assert m.read_bytes() == model_ref and v.read_bytes() == vocab_ref


@pytest.mark.parametrize("layout", ["types", "stream"])
def test_medium_corpus_matches_oracle(layout, tmp_path):
    corpus = str(tmp_path / "m.txt")
    corpora.gen_synthetic(corpus, 12_000_000, 31, "mixed")
    subprocess.run(["make", "-s", "-C", ORACLE, "port"], check=True)
    om, ov = str(tmp_path / "o.model"), str(tmp_path / "o.vocab")
    subprocess.run([os.path.join(ORACLE, "_build", "bpe_oracle"), corpus, "6000", "0", "0.9995", "20", om, ov],
                   check=True, stderr=subprocess.DEVNULL)
    t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
    t.set_option("layout", layout)
    t.load_corpus(corpus)
    n, model, vocab = _train_bytes(t, tmp_path, "g")
    t.destroy()
    assert model == open(om, "rb").read()
    assert vocab == open(ov, "rb").read()
    assert n > 1000


@pytest.fixture(scope="module")
def medium_corpus(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("med") / "m.txt")
    corpora.gen_synthetic(path, 12_000_000, 31, "mixed")
    return path


@pytest.fixture(scope="module")
def medium_oracle(medium_corpus, tmp_path_factory):
    d = tmp_path_factory.mktemp("medo")
    subprocess.run(["make", "-s", "-C", ORACLE, "port"], check=True)
    om, ov = str(d / "o.model"), str(d / "o.vocab")
    subprocess.run([os.path.join(ORACLE, "_build", "bpe_oracle"), medium_corpus, "6000", "0", "0.9995", "20", om, ov],
                   check=True, stderr=subprocess.DEVNULL)
    return open(om, "rb").read(), open(ov, "rb").read()


@pytest.mark.parametrize("layout,bucket", [("types", 0), ("types", 8), ("stream", 64)])
def test_exchange_path_matches_oracle(layout, bucket, medium_corpus, medium_oracle, tmp_path):
    """The multi-GPU path on one GPU: every merge's records go through the RCCL all-gather (a
    single-rank communicator) and k_xout, small buckets force the overflow round.  torch is
    imported first, as in a real multi-GPU process (torch.distributed): the library then shares
    torch's RCCL instead of opening its own (two RCCLs in one process abort at exit)."""
    import torch  # noqa: F401
    t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
    t.set_option("layout", layout)
    t.set_option("exchange", "local")
    if bucket:
        t.set_option("exchange_bucket", bucket)
    t.load_corpus(medium_corpus)
    n, model, vocab = _train_bytes(t, tmp_path, "x")
    st = t.stats()
    t.destroy()
    assert (model, vocab) == medium_oracle
    assert n > 1000
    assert st["spec_hits"] > 0
    if bucket:
        assert st["exchange_overflows"] > 0


def test_rollback_restores_stream(medium_corpus):
    """The undo path of speculation (k_unmerge) leaves the corpus bit-identical, including
    a == b runs and pairs spanning many tiles."""
    from shredword.cbase import lib
    t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
    t.set_option("layout", "stream")
    t.load_corpus(medium_corpus)
    lib.bpe_init(t.trainer)
    assert lib.bpe_merge_batch(t.trainer, 40) == 40
    before = t.tokens()
    for pair in [(101, 32), (32, 116), (116, 104), (101, 101), (108, 108), (256, 257), (32, 32)]:
        assert lib.shred_probe_rollback(t.trainer, *pair) == 0
        after = t.tokens()
        assert after.shape == before.shape and (after == before).all(), pair
    t.destroy()


@pytest.mark.parametrize("layout,index", [("stream", 0), ("types", 0), ("types", 1)])
def test_speculation_lockstep(layout, index, medium_corpus):
    """Speculative pipelining on vs off, in bpe_merge_batch chunks: identical merges and an
    identical device token stream after every chunk (rollbacks included).  index=1: the indexed
    loop (guesses undone by UNMERGE); index=0: the launch path."""
    from shredword.cbase import lib
    ts = []
    for spec in (0, 1):
        t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
        t.set_option("layout", layout)
        t.set_option("speculate", spec)
        t.set_option("resident", 0)
        t.set_option("index", index)
        t.load_corpus(medium_corpus)
        lib.bpe_init(t.trainer)
        ts.append(t)
    done = 0
    for chunk in [64, 1, 7, 200, 33] * 40:
        na = lib.bpe_merge_batch(ts[0].trainer, chunk)
        nb = lib.bpe_merge_batch(ts[1].trainer, chunk)
        assert na == nb
        xa, xb = ts[0].tokens(), ts[1].tokens()
        assert xa.shape == xb.shape and (xa == xb).all(), f"streams differ after {done + na} merges"
        done += na
        if na < chunk:
            break
    st = ts[1].stats()
    assert st["spec_hits"] > 0 and st["spec_misses"] > 0
    for t in ts:
        t.destroy()


@pytest.mark.parametrize("tokens,depth", [("lds", 1), ("hbm", 1), ("lds", 2), ("hbm", 3)])
def test_resident_lockstep(tokens, depth, medium_corpus, tmp_path, monkeypatch):
    """The resident merge loop (k_resident) against the launch path, in bpe_merge_batch
    chunks: identical merges and device token streams after every chunk (each chunk ends the
    persistent launch and writes the tiles back).  tokens=hbm keeps the tokens in HBM (the mode
    of tables larger than the chip's LDS); depth = guessed merges in flight behind the current
    one (a wrong guess undoes every guess after it, newest first)."""
    from shredword.cbase import lib
    if tokens == "hbm":
        monkeypatch.setenv("SHREDWORD_RESIDENT_HBM", "1")
    ts = []
    for res in (0, 1):
        t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
        t.set_option("resident", res)
        t.set_option("index", 0)
        t.set_option("spec_depth", depth)
        t.load_corpus(medium_corpus)
        lib.bpe_init(t.trainer)
        ts.append(t)
    done = 0
    for chunk in [1, 300, 7, 1000, 64] * 20:
        na = lib.bpe_merge_batch(ts[0].trainer, chunk)
        nb = lib.bpe_merge_batch(ts[1].trainer, chunk)
        assert na == nb
        xa, xb = ts[0].tokens(), ts[1].tokens()
        assert xa.shape == xb.shape and (xa == xb).all(), f"streams differ after {done + na} merges"
        done += na
        if na < chunk:
            break
    assert done > 4000
    st0, st1 = ts[0].stats(), ts[1].stats()
    assert st0["resident_launches"] == 0 and st1["resident_launches"] > 10
    assert st1["spec_hits"] > 0 and st1["spec_misses"] > 0  # guesses confirmed and undone in LDS
    paths = []
    for i, t in enumerate(ts):
        m, v = str(tmp_path / f"r{i}.model"), str(tmp_path / f"r{i}.vocab")
        t.save(m, v)
        paths.append((open(m, "rb").read(), open(v, "rb").read()))
        t.destroy()
    assert paths[0] == paths[1]


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_index_lockstep(depth, medium_corpus, tmp_path):
    """The indexed loop (k_word_loop) against the launch path, in bpe_merge_batch chunks: the
    same merges and the same device token stream after every chunk (each chunk ends the
    persistent launch and writes the words back into the tiles), with `depth` guesses in flight."""
    from shredword.cbase import lib
    ts = []
    for idx in (0, 1):
        t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
        t.set_option("resident", 0)
        t.set_option("index", idx)
        t.set_option("spec_depth", depth)
        t.load_corpus(medium_corpus)
        lib.bpe_init(t.trainer)
        ts.append(t)
    done = 0
    for chunk in [1, 300, 7, 1000, 64] * 20:
        na = lib.bpe_merge_batch(ts[0].trainer, chunk)
        nb = lib.bpe_merge_batch(ts[1].trainer, chunk)
        assert na == nb
        xa, xb = ts[0].tokens(), ts[1].tokens()
        assert xa.shape == xb.shape and (xa == xb).all(), f"streams differ after {done + na} merges"
        done += na
        if na < chunk:
            break
    assert done > 4000
    st0, st1 = ts[0].stats(), ts[1].stats()
    assert st0["index_merges"] == 0 and st1["index_merges"] >= done
    assert st1["spec_hits"] > 0 and st1["index_undos"] > 0
    paths = []
    for i, t in enumerate(ts):
        m, v = str(tmp_path / f"i{i}.model"), str(tmp_path / f"i{i}.vocab")
        t.save(m, v)
        paths.append((open(m, "rb").read(), open(v, "rb").read()))
        t.destroy()
    assert paths[0] == paths[1]


@pytest.mark.parametrize("switch_occ", [300, 1 << 40])
def test_hybrid_lockstep(switch_occ, medium_corpus):
    """The hybrid path (k_resident, then the indexed loop from the first merge that changes fewer
    than switch_occ occurrences) against the launch path in bpe_merge_batch chunks: the same
    merges and device token stream after every chunk (the switch happens inside a chunk)."""
    from shredword.cbase import lib
    ts = []
    for hybrid in (0, 1):
        t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
        if hybrid:
            t.set_option("switch_occ", switch_occ)
        else:
            t.set_option("resident", 0)
            t.set_option("index", 0)
        t.load_corpus(medium_corpus)
        lib.bpe_init(t.trainer)
        ts.append(t)
    done = 0
    for chunk in [1, 300, 7, 1000, 64] * 20:
        na = lib.bpe_merge_batch(ts[0].trainer, chunk)
        nb = lib.bpe_merge_batch(ts[1].trainer, chunk)
        assert na == nb
        xa, xb = ts[0].tokens(), ts[1].tokens()
        assert xa.shape == xb.shape and (xa == xb).all(), f"streams differ after {done + na} merges"
        done += na
        if na < chunk:
            break
    st = ts[1].stats()
    assert st["resident_launches"] > 0 and st["index_merges"] > 0 and st["index_switch_merge"] >= 256
    for t in ts:
        t.destroy()


def test_index_after_tile_path_merges(medium_corpus, tmp_path):
    """Merges on the tile path (index off) followed by indexed merges (index on) on the same
    trainer: the loop re-reads the merged tiles and re-indexes them; then reset() returns to the
    uploaded table and its initial index, and a full retrain matches a fresh trainer."""
    from shredword.cbase import lib
    ref = _trainer(vocab_size=3000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
    ref.set_option("index", 0)
    ref.set_option("resident", 0)
    ref.load_corpus(medium_corpus)
    n_ref, model_ref, vocab_ref = _train_bytes(ref, tmp_path, "ref")
    ref.destroy()
    t = _trainer(vocab_size=3000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
    t.load_corpus(medium_corpus)
    lib.bpe_init(t.trainer)
    t.set_option("index", 0)
    t.set_option("resident", 0)
    assert lib.bpe_merge_batch(t.trainer, 500) == 500
    t.set_option("index", 1)
    done = 500
    while done < n_ref:
        k = lib.bpe_merge_batch(t.trainer, min(777, n_ref - done))
        assert k > 0
        done += k
    m, v = tmp_path / "mix.model", tmp_path / "mix.vocab"
    t.save(str(m), str(v))
    assert m.read_bytes() == model_ref and v.read_bytes() == vocab_ref
    assert t.stats()["index_merges"] >= n_ref - 500
    t.reset()
    n2, model2, vocab2 = _train_bytes(t, tmp_path, "again")
    t.destroy()
    assert (n2, model2, vocab2) == (n_ref, model_ref, vocab_ref)


def _parse_vocab(vocab: bytes, ops):
    """(spelling, freq) per id, walking the file with spellings derived from the merges:
    a spelling may contain any byte (token 10 is a newline), so lines cannot be split blindly."""
    spell = [bytes([i]) if i else b"" for i in range(256)]
    for a, b, _x in ops:
        spell.append(spell[a] + spell[b])
    out, pos = [], 0
    for tok in spell:
        assert vocab[pos:pos + len(tok)] == tok
        pos += len(tok)
        assert vocab[pos:pos + 1] == b" "
        end = vocab.index(b"\n", pos + 1)
        out.append((tok, int(vocab[pos + 1:end])))
        pos = end + 1
    assert pos == len(vocab)
    return out


def _fullsize(name):
    import gzip
    import json
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize", name)
    if not os.path.exists(os.path.join(d, "case.json")):
        pytest.skip(f"no full-size fixture for {name}")
    case = json.load(open(os.path.join(d, "case.json")))
    with gzip.open(os.path.join(d, "model.bin.gz"), "rb") as f:
        case["model_bytes"] = f.read()
    with gzip.open(os.path.join(d, "trace.txt.gz"), "rt") as f:
        case["trace"] = f.read()
    r = case["recipe"]
    d = os.path.join(os.environ.get("TMPDIR", "/tmp"), "shredword_bench")
    if r["bytes"] > 20_000_000_000:  # C4 80 GB / C5 100 GB: memory-backed (the box's disk is smaller)
        import shutil
        d = "/dev/shm/shredword_full"
        os.makedirs(d, exist_ok=True)
        if shutil.disk_usage(d).free < r["bytes"] + (8 << 30):
            pytest.skip(f"{name}: {r['bytes'] / 1e9:.0f} GB corpus does not fit {d}")
    corpus = os.path.join(d, f"{name}_{r['script']}_{r['bytes']}_s{r['seed']}.txt")
    if not (os.path.exists(corpus) and os.path.getsize(corpus) == r["bytes"]):
        os.makedirs(os.path.dirname(corpus), exist_ok=True)
        corpora.gen_synthetic(corpus, r["bytes"], r["seed"], r["script"])
    return case, corpus


# C4 (80 GB) and C4's parameters at 10 GB are loaded as the C4 job loads its corpus: 8 byte ranges
# counted on the device in turn and merged (the per-rank step of the sharded load,
# SHREDWORD_LOAD_SIM_SHARDS)
_FULLSIZE_ENV = {"c4_10g": {"SHREDWORD_LOAD_SIM_SHARDS": "8"}, "c4": {"SHREDWORD_LOAD_SIM_SHARDS": "8"}}


@pytest.mark.parametrize("name", ["c2", "c3", "c5_10g", "c4_10g", "c5", "c4"])
def test_full_size_matches_oracle_run(name, tmp_path, monkeypatch):
    """Full-size corpora, bit-exact: .model bytes, .vocab md5 and every merge / batch line against
    the oracle's full run committed in tests/golden/fullsize/ (the oracle is pinned to the
    reference by every golden, including the reference's own 31,744- and 63,744-merge runs).
    c2 = C2 (1 GB, vocab 8192), c3 = C3 (10 GB, vocab 32000, min_pair_freq 2), c5_10g = C5's
    parameters (vocab 64000, coverage 0.9995, mixed script) on 10 GB, c4_10g = C4's parameters
    on 10 GB through the 8-way sharded load; c5 = C5 at its full 100 GB and c4 = C4 at its full
    80 GB (8-way sharded load), against streamed oracle runs (round 5, make_fullsize.py), their
    corpora generated into /dev/shm and removed afterwards."""
    import hashlib
    import time
    from conftest import progress
    t0 = time.time()
    case, corpus = _fullsize(name)
    progress(f"[{name}] corpus ready {time.time() - t0:.0f} s")
    for k, v in _FULLSIZE_ENV.get(name, {}).items():
        monkeypatch.setenv(k, v)
    cfg = case["config"]
    try:
        t = _trainer(vocab_size=cfg["vocab_size"], unk_id=cfg["unk_id"], character_coverage=cfg["character_coverage"],
                     min_pair_freq=cfg["min_pair_freq"])
        trace = str(tmp_path / "trace.txt")
        t.set_option("trace", trace)
        t.load_corpus(corpus)
        progress(f"[{name}] loaded {time.time() - t0:.0f} s")
        n, model, vocab = _train_bytes(t, tmp_path, name)
        progress(f"[{name}] trained {time.time() - t0:.0f} s")
        st = t.stats()
        t.destroy()
    finally:
        if case["recipe"]["bytes"] > 20_000_000_000:
            os.unlink(corpus)  # 80-100 GB of the box's memory
    assert (st["num_words"], st["num_symbols"]) == (case["distinct_words"], case["symbols"])
    assert n == case["merges"]
    assert open(trace).read() == case["trace"]
    assert model == case["model_bytes"]
    assert hashlib.md5(vocab).hexdigest() == case["vocab_md5"]


def _word_bytes(corpus):
    """Bytes of the corpus that are not delimiters ([\t\r\n ]), streamed in 1 GB pieces."""
    total = 0
    with open(corpus, "rb") as f:
        while True:
            buf = f.read(1 << 30)
            if not buf:
                return total
            d = np.frombuffer(buf, dtype=np.uint8)
            total += d.size - int(np.count_nonzero((d == 32) | (d == 10) | (d == 9) | (d == 13)))


# Size-independent invariants at full size: byte conservation, operands before their merge,
# non-increasing merge frequencies >= min_pair_freq, and the K5 device recount every 500 merges
# (the host heap's pick is the largest pair count and its own count).
_INVARIANT_CASES = {
    # name: (bytes, seed, script, vocab, coverage, min_pair_freq, env, expected merges or None)
    "c2": (1_000_000_000, 2, "utf8", 8192, 0.995, 2000, {}, 7936),
    "c5_10g": (10_000_000_000, 5, "mixed", 64000, 0.9995, 2000, {}, None),
    "c4_10g": (10_000_000_000, 4, "utf8", 32000, 0.995, 2000, {"SHREDWORD_LOAD_SIM_SHARDS": "8"}, None),
}


@pytest.mark.parametrize("name", sorted(_INVARIANT_CASES))
def test_full_size_invariants(name, tmp_path, monkeypatch):
    nbytes, seed, script, vocab_size, cov, mpf, env, expect = _INVARIANT_CASES[name]
    corpus = os.path.join(os.environ.get("TMPDIR", "/tmp"), "shredword_bench", f"{name}_{script}_{nbytes}_s{seed}.txt")
    if not (os.path.exists(corpus) and os.path.getsize(corpus) == nbytes):
        os.makedirs(os.path.dirname(corpus), exist_ok=True)
        corpora.gen_synthetic(corpus, nbytes, seed, script)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    t = _trainer(vocab_size=vocab_size, unk_id=0, character_coverage=cov, min_pair_freq=mpf)
    trace = str(tmp_path / "trace.txt")
    t.set_option("trace", trace)
    t.set_option("verify_argmax", 500)
    t.load_corpus(corpus)
    n, model, vocab = _train_bytes(t, tmp_path, name)
    st = t.stats()
    t.destroy()
    if expect is not None:
        assert n == expect
    assert 0 < n <= vocab_size - 256
    assert st["verify_checks"] >= n // 500 and st["verify_failures"] == 0
    T = 256 + n
    ops = np.frombuffer(model, dtype="<i4").reshape(-1, 3)
    assert (ops[:, 2] == np.arange(256, T)).all()
    assert (ops[:, :2] < ops[:, 2:3]).all()  # operands exist before their merge
    toks = _parse_vocab(vocab, ops)
    assert len(toks) == T
    # Byte conservation: every byte of every word occurrence ends in exactly one final token.
    # unk_id = 0 has the empty spelling and counts one byte per unk symbol (byte 0 never occurs).
    assert sum(len(tok) * f for tok, f in toks[1:]) + toks[0][1] == _word_bytes(corpus)
    freqs = [int(ln.split()[3]) for ln in open(trace) if ln.startswith("M ")]
    assert len(freqs) == n
    assert all(x >= y for x, y in zip(freqs, freqs[1:])), "merge frequencies must not increase"
    assert freqs[-1] >= mpf


@pytest.mark.parametrize("wide", ["0", "1", "2"], ids=["narrow", "wide", "xwide"])
@pytest.mark.parametrize("kind", ["medium", "adversarial_no_nul", "utf8"])
def test_gpu_word_count_matches_host(kind, wide, medium_corpus, tmp_path, monkeypatch):
    """load_corpus counting words on the device (load_device.hip) against the host count: the
    same word table, so the same training bytes -- with both k_word_count workgroup shapes
    (256 threads / 1536 LDS slots, 512 / 3072; SHREDWORD_LOAD_WIDE).  The adversarial corpus (CR/TAB
    runs, 10 kB lines, a 10,333-byte word, no final newline) is taken without its NUL bytes,
    which keep the host's fgets/strlen path.  Shapes: 256 threads / 1536 slots, 512 / 3072, and
    768 / 3072 (xwide, round 5)."""
    monkeypatch.setenv("SHREDWORD_GPU_LOAD_MIN", "1")
    monkeypatch.setenv("SHREDWORD_LOAD_WIDE", wide)
    if kind == "medium":
        corpus = medium_corpus
    elif kind == "utf8":
        corpus = str(tmp_path / "u.txt")
        corpora.gen_synthetic(corpus, 3_000_000, 77, "utf8")
    else:
        corpus = str(tmp_path / "adv.txt")
        with open(corpus, "wb") as f:
            f.write(corpora.adversarial_bytes(5).replace(b"\0", b""))
    outs = []
    for gpu in (0, 1):
        t = _trainer(vocab_size=3000, unk_id=0, character_coverage=0.9995, min_pair_freq=2)
        t.set_option("gpu_load", gpu)
        t.load_corpus(corpus)
        n, model, vocab = _train_bytes(t, tmp_path, f"w{gpu}")
        st = t.stats()
        t.destroy()
        assert st["load_on_gpu"] == gpu
        outs.append((n, model, vocab, st["num_words"], st["num_symbols"], st["num_occurrences"]))
    assert outs[0] == outs[1]



def test_gpu_word_count_grows_a_full_table(medium_corpus, tmp_path, monkeypatch):
    """The device word table started far below the corpus's distinct words
    (SHREDWORD_LOAD_TABLE_SLOTS=1024): the count stops at the 3/4 fill (bounded probes, every
    workgroup leaves at its next tile), grows the table 4x and reruns until it fits -- the same
    word table as the host count, in bounded time (a full table once cost minutes of probing)."""
    import time
    monkeypatch.setenv("SHREDWORD_GPU_LOAD_MIN", "1")
    outs = []
    for slots in ("1024", None):
        if slots:
            monkeypatch.setenv("SHREDWORD_LOAD_TABLE_SLOTS", slots)
        else:
            monkeypatch.delenv("SHREDWORD_LOAD_TABLE_SLOTS", raising=False)
        t = _trainer(vocab_size=2000, unk_id=0, character_coverage=0.9995, min_pair_freq=2)
        t.set_option("gpu_load", 1 if slots else 0)
        t0 = time.time()
        t.load_corpus(medium_corpus)
        dt = time.time() - t0
        n, model, vocab = _train_bytes(t, tmp_path, f"g{slots}")
        st = t.stats()
        t.destroy()
        if slots:
            assert st["load_on_gpu"] == 1 and st["num_words"] > 4 * 1024 and dt < 30
        outs.append((n, model, vocab, st["num_words"], st["num_occurrences"]))
    assert outs[0] == outs[1]


def test_gpu_word_count_detects_key_collisions(medium_corpus, tmp_path, monkeypatch):
    """Word keys narrowed to 12 bits (SHREDWORD_LOAD_KEY_BITS): thousands of distinct words share
    keys, the byte compare inside k_word_count flags it on every seed, and the load falls back to
    the host count -- the same word table as the 64-bit device count."""
    monkeypatch.setenv("SHREDWORD_GPU_LOAD_MIN", "1")
    outs = []
    for bits in ("12", "64"):
        monkeypatch.setenv("SHREDWORD_LOAD_KEY_BITS", bits)
        t = _trainer(vocab_size=2000, unk_id=0, character_coverage=0.9995, min_pair_freq=2)
        t.load_corpus(medium_corpus)
        n, model, vocab = _train_bytes(t, tmp_path, f"k{bits}")
        st = t.stats()
        t.destroy()
        assert st["load_on_gpu"] == (bits == "64")
        outs.append((n, model, vocab, st["num_words"], st["num_occurrences"]))
    assert outs[0] == outs[1]


@pytest.mark.parametrize("shards", [2, 5])
def test_sharded_load_ranges_on_gpu(shards, medium_corpus, tmp_path, monkeypatch):
    """The sharded load's per-rank step on the GPU (SHREDWORD_LOAD_SIM_SHARDS: the k byte ranges
    counted by k_word_count in turn, in one process) merged into the table: the same bytes as the
    whole-file device count."""
    monkeypatch.setenv("SHREDWORD_GPU_LOAD_MIN", "1")
    outs = []
    for sim in ("0", str(shards)):
        monkeypatch.setenv("SHREDWORD_LOAD_SIM_SHARDS", sim)
        t = _trainer(vocab_size=3000, unk_id=0, character_coverage=0.9995, min_pair_freq=2)
        t.load_corpus(medium_corpus)
        n, model, vocab = _train_bytes(t, tmp_path, f"s{sim}")
        st = t.stats()
        t.destroy()
        assert st["load_on_gpu"] == 1
        outs.append((n, model, vocab, st["num_words"], st["num_symbols"], st["num_occurrences"]))
    assert outs[0] == outs[1]


def test_resident_abort_falls_back(medium_corpus, medium_oracle, tmp_path, monkeypatch):
    """k_resident's co-residency check: with a zero bound the leader never sees every workgroup
    (an abort on every launch); the merges it was given run again on the indexed loop, and the
    files are still the oracle's."""
    monkeypatch.setenv("SHREDWORD_RESIDENT_ARRIVE_POLLS", "0")
    t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
    t.load_corpus(medium_corpus)
    n, model, vocab = _train_bytes(t, tmp_path, "ab")
    st = t.stats()
    assert (model, vocab) == medium_oracle
    assert n > 1000
    assert st["resident_aborts"] >= 1 and st["index_merges"] > 0
    # a second load on the same trainer frees and reallocates the buffers the aborted launch's
    # late workgroups read: its retired streams drain first (Device::drain_retired)
    # (reset: a reload keeps the merge count, as the reference's num_merges, bpe.cpp:176-185)
    t.load_corpus(medium_corpus)
    t.reset()
    n2, model2, vocab2 = _train_bytes(t, tmp_path, "ab2")
    t.destroy()
    assert (n2, model2, vocab2) == (n, model, vocab)


def test_word_loop_idle_timeout_resumes(medium_corpus, medium_oracle, tmp_path, monkeypatch):
    """k_word_loop ends itself after SHREDWORD_WL_IDLE_POLLS polls without a command.  With a
    bound of one poll it ends between almost every pair of merges, racing the host's posts: the
    host resumes a new launch at the first command the old one did not take (status[1]), and the
    files are still the oracle's."""
    monkeypatch.setenv("SHREDWORD_WL_IDLE_POLLS", "1")
    t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
    t.load_corpus(medium_corpus)
    n, model, vocab = _train_bytes(t, tmp_path, "to")
    st = t.stats()
    t.destroy()
    assert (model, vocab) == medium_oracle
    assert st["index_merges"] > 0 and st["index_launches"] >= 2


def test_resident_partial_residency(medium_corpus, medium_oracle, tmp_path):
    """Another process fills every wave slot of all CUs but 16 while train() runs: k_resident's grid
    cannot be co-resident, its leader aborts within its bound instead of hanging, and the run
    completes bit-exact through the fallback (reported in stats).  (A second process: kernels of
    one process may share a hardware queue and then never run side by side.)"""
    import sys
    holder = subprocess.Popen(
        [sys.executable, "-c",
         "import sys; sys.path.insert(0, %r)\n"
         "from shredword.cbase import lib\n"
         "h = lib.shred_occupy(0, 16, 60.0)\n"
         "print('ready' if h else 'failed', flush=True)\n"
         "sys.stdin.read()\n"
         "lib.shred_release(h)\n" % os.path.join(os.path.dirname(ORACLE), "shredword-trainer_amd")],
        stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        assert holder.stdout.readline().strip() == "ready"
        t = _trainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
        t.load_corpus(medium_corpus)
        n, model, vocab = _train_bytes(t, tmp_path, "pr")
        st = t.stats()
    finally:
        holder.stdin.close()
        holder.wait(timeout=120)
    t.destroy()
    assert (model, vocab) == medium_oracle
    assert n > 1000
    assert st["resident_aborts"] >= 1


_PLAIN_CTYPES = r'''
import ctypes, os, sys, tempfile
from ctypes import c_size_t, c_int32, c_float, c_uint64, c_char_p, c_int, c_void_p, Structure, POINTER
lib = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)   # as the reference's cbase.py:28-30
class BPEConfig(Structure):
    _fields_ = [("target_vocab_size", c_size_t), ("unk_id", c_int32), ("character_coverage", c_float),
                ("min_pair_freq", c_uint64)]
lib.create_trainer.argtypes, lib.create_trainer.restype = [POINTER(BPEConfig)], c_void_p
lib.bpe_load_corpus.argtypes, lib.bpe_load_corpus.restype = [c_void_p, c_char_p], c_int
lib.bpe_train.argtypes, lib.bpe_train.restype = [c_void_p], c_int
lib.bpe_save.argtypes, lib.bpe_save.restype = [c_void_p, c_char_p, c_char_p], None
lib.bpe_trainer_destroy.argtypes, lib.bpe_trainer_destroy.restype = [c_void_p], None
d = tempfile.mkdtemp()
p = os.path.join(d, "c.txt")
open(p, "w").write("ab abc aab bca the then them other " * 3000)
cfg = BPEConfig(300, 0, 0.995, 2)
t = lib.create_trainer(ctypes.byref(cfg))
assert lib.bpe_load_corpus(t, p.encode()) == 0
n = lib.bpe_train(t)
lib.bpe_save(t, os.path.join(d, "m").encode(), os.path.join(d, "v").encode())
lib.bpe_trainer_destroy(t)
assert n > 0
if sys.argv[2] == "torch":
    import torch
    x = torch.arange(1000, device="cuda").sum().item()
    assert x == 499500
print("ok", n, flush=True)
'''


@pytest.mark.parametrize("then", ["torch", "none"])
def test_plain_ctypes_then_torch_exits_cleanly(then, tmp_path):
    """The reference's binding (plain ctypes.CDLL of the library, no torch imported first), a
    train, then `import torch` and a CUDA op in the same process: one HIP runtime, exit code 0."""
    import sys
    from conftest import PKG
    script = tmp_path / "plain.py"
    script.write_text(_PLAIN_CTYPES)
    lib_path = os.path.join(PKG, "shredword", "libtrainer.so")
    proc = subprocess.run([sys.executable, str(script), lib_path, then], capture_output=True, text=True, timeout=240,
                          env=dict(os.environ, SHREDWORD_LOG="0"))
    assert proc.returncode == 0, (proc.returncode, proc.stderr[-2000:])
    assert proc.stdout.strip().startswith("ok")


@pytest.mark.parametrize("readers,chunk_mb,seg_mb,long_word", [(8, 32, 2048, False), (3, 1, 1, False),
                                                                (2, 1, 1, True), (4, 1, 0, False)])
def test_file_streamed_to_hbm_matches_host(readers, chunk_mb, seg_mb, long_word, tmp_path, monkeypatch):
    """load_corpus reads the file straight into HBM (gpu_count_file: reader threads, pread into
    pinned buffers, one DMA per chunk; the spellings come back from the device), counting 1 MiB
    segments while later chunks still upload (seg_mb 0: no overlap): the same table and training
    bytes as the host count -- also with a 2.5 MB word that runs past a segment's landed bytes
    (the count is then repeated after the upload)."""
    monkeypatch.setenv("SHREDWORD_GPU_LOAD_MIN", "1")
    monkeypatch.setenv("SHREDWORD_LOAD_READERS", str(readers))
    monkeypatch.setenv("SHREDWORD_LOAD_CHUNK_MB", str(chunk_mb))
    if seg_mb:
        monkeypatch.setenv("SHREDWORD_LOAD_SEGMENT_MB", str(seg_mb))
    else:
        monkeypatch.setenv("SHREDWORD_LOAD_OVERLAP", "0")
    corpus = str(tmp_path / "u.txt")
    corpora.gen_synthetic(corpus, 5_500_000, 78, "mixed")
    if long_word:
        data = open(corpus, "rb").read()
        at = data.index(b"\n", 900_000) + 1
        open(corpus, "wb").write(data[:at] + b"ab" * 1_250_000 + b"\n" + data[at:])
    outs = []
    for gpu in (0, 1):
        t = _trainer(vocab_size=2000, unk_id=0, character_coverage=0.9995, min_pair_freq=2)
        t.set_option("gpu_load", gpu)
        t.load_corpus(corpus)
        outs.append(_train_bytes(t, tmp_path, f"s{gpu}"))
        assert t.stats()["load_on_gpu"] == gpu
        t.destroy()
    assert outs[0] == outs[1]


def test_nul_byte_file_takes_the_host_path(tmp_path, monkeypatch):
    """A NUL byte deep inside a file (the reference's fgets/strlen drop the rest of that line):
    the device count notices it and the host path counts; files equal the host-only load's."""
    monkeypatch.setenv("SHREDWORD_GPU_LOAD_MIN", "1")
    corpus = str(tmp_path / "n.txt")
    corpora.gen_synthetic(corpus, 3_000_000, 79, "utf8")
    data = bytearray(open(corpus, "rb").read())
    at = data.index(b"\n", 2_000_000) + 5
    data[at] = 0
    open(corpus, "wb").write(bytes(data))
    outs = []
    for gpu in (1, 0):
        t = _trainer(vocab_size=1500, unk_id=0, min_pair_freq=2)
        t.set_option("gpu_load", gpu)
        t.load_corpus(corpus)
        assert t.stats()["load_on_gpu"] == 0
        outs.append(_train_bytes(t, tmp_path, f"n{gpu}"))
        t.destroy()
    assert outs[0] == outs[1]
