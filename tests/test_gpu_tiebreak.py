"""GPU tests of tiebreak=device: the device selects every merge
itself -- a pair table on the device, updated in place by each merge's exact deltas, and a
frontier argmax inside the persistent indexed loop (k_word_loop<true>) -- with no host round trip
per merge.  Opt-in and NOT the reference's merge order: ties go to the smaller (first, second)
key instead of the reference heap's layout (SURVEY §0 finding 2).

* The rule is deterministic, so it is checked bit for bit against its CPU restatement
  (bpe_oracle --tiebreak-device 0: the oracle's exact pair counts, the same tie rule).
* K5 at every step: with verify_argmax = k the device selects k merges at a time from a table
  rebuilt from a fresh K1 count, and the first merge of each chunk must be that recount's maximum
  (ties: the smaller key); the files must equal the unchunked run's.
* Deep run (31,744 merges): non-increasing frequencies >= min_pair_freq, operands before their
  merge, symbol conservation against the exact mode's .vocab.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ORACLE

pytestmark = pytest.mark.gpu

CASES = ["small_v300", "adv_unk0", "adv_unk3_cov09", "adv_unkm1", "ascii1m_unk7_cov09", "ascii1m_v3000_mpf2",
         "utf8_2m_v2000_mpf50", "ascii1m_unkm1_mpf2", "mixed2m_v4000", "utf8_4m_v8192_mpf5"]


def _train(case, corpus, tmp_path, tag="d", **opts):
    from shredword.trainer import BPETrainer
    cfg = case["config"]
    t = BPETrainer(vocab_size=cfg["vocab_size"], unk_id=cfg["unk_id"], character_coverage=cfg["character_coverage"],
                   min_pair_freq=cfg["min_pair_freq"])
    trace = str(tmp_path / f"{tag}.trace")
    t.set_option("log", 0)
    t.set_option("trace", trace)
    t.set_option("tiebreak", "device")
    for k, v in opts.items():
        t.set_option(k, v)
    t.load_corpus(corpus)
    n = t._train(t.trainer)
    m, v = str(tmp_path / f"{tag}.model"), str(tmp_path / f"{tag}.vocab")
    t.save(m, v)
    st = t.stats()
    t.destroy()
    return n, open(m, "rb").read(), open(v, "rb").read(), open(trace).read(), st


def _oracle_rule(case, corpus, tmp_path):
    subprocess.run(["make", "-s", "-C", ORACLE, "port"], check=True)
    cfg = case["config"]
    om, ov, ot = (str(tmp_path / f"o.{k}") for k in ("model", "vocab", "trace"))
    subprocess.run([os.path.join(ORACLE, "_build", "bpe_oracle"), corpus, str(cfg["vocab_size"]), str(cfg["unk_id"]),
                    repr(cfg["character_coverage"]), str(cfg["min_pair_freq"]), om, ov, "--trace", ot,
                    "--tiebreak-device", "0"], check=True, stderr=subprocess.DEVNULL)
    return open(om, "rb").read(), open(ov, "rb").read(), open(ot).read()


@pytest.mark.parametrize("name", CASES)
def test_tiebreak_device_matches_its_cpu_rule(name, case_corpus, tmp_path):
    case, corpus = case_corpus(name)
    n, model, vocab, trace, st = _train(case, corpus, tmp_path)
    om, ov, ot = _oracle_rule(case, corpus, tmp_path)
    assert trace == ot
    assert model == om
    assert vocab == ov
    assert st["sel_merges"] + st["sel_host_merges"] == n and (st["sel_merges"] == 0 or st["sel_launches"] >= 1)
    assert st["heap_size"] == 0  # the host heap took no part


@pytest.mark.parametrize("name", ["small_v300", "adv_unk3_cov09", "ascii1m_v3000_mpf2", "mixed2m_v4000"])
def test_tiebreak_device_k5_every_merge(name, case_corpus, tmp_path):
    """verify_argmax = 1: every merge selected from a table rebuilt from a fresh K1 recount must be
    that recount's maximum; the files equal the run with one table for the whole training."""
    case, corpus = case_corpus(name)
    n1, m1, v1, t1, st1 = _train(case, corpus, tmp_path, "one")
    every = 1 if case["config"]["vocab_size"] <= 1000 else 7
    n2, m2, v2, t2, st2 = _train(case, corpus, tmp_path, "chunked", verify_argmax=every)
    assert (n1, m1, v1, t1) == (n2, m2, v2, t2)
    assert st2["verify_failures"] == 0
    assert st2["verify_checks"] >= n2 // every


def _parse_vocab(vocab, ops):
    spell = [bytes([i]) if i else b"" for i in range(256)]
    for a, b, _x in ops:
        spell.append(spell[a] + spell[b])
    out, pos = [], 0
    for tok in spell:
        assert vocab[pos:pos + len(tok)] == tok
        pos += len(tok)
        end = vocab.index(b"\n", pos + 1)
        out.append(int(vocab[pos + 1:end]))
        pos = end + 1
    assert pos == len(vocab)
    return out


def _symbols(vocab, model):
    """Σ freq(id) x (base symbols of id): the corpus's weighted symbol count, which no merge changes."""
    ops = np.frombuffer(model, dtype="<i4").reshape(-1, 3)
    freq = _parse_vocab(vocab, ops)
    size = [1] * 256
    for a, b, _x in ops:
        size.append(size[a] + size[b])
    return sum(f * s for f, s in zip(freq, size))


def test_tiebreak_device_deep_run(case_corpus, tmp_path):
    """The 31,744-merge reference golden's corpus and config (vocab 32000, min_pair_freq 2) in
    tiebreak=device: invariants, a K5 recount every 997 merges, and the weighted symbol count of
    the exact mode's (the reference's) .vocab."""
    case, corpus = case_corpus("utf8_24m_v32000_mpf2")
    n, model, vocab, trace, st = _train(case, corpus, tmp_path, verify_argmax=997)
    assert n == case["merges"]
    assert st["verify_failures"] == 0 and st["verify_checks"] >= n // 997
    ops = np.frombuffer(model, dtype="<i4").reshape(-1, 3)
    assert (ops[:, 2] == np.arange(256, 256 + n)).all()
    assert (ops[:, :2] < ops[:, 2:3]).all()
    freqs = [int(ln.split()[3]) for ln in trace.splitlines() if ln.startswith("M ")]
    assert len(freqs) == n
    assert all(x >= y for x, y in zip(freqs, freqs[1:])), "merge frequencies must not increase"
    assert freqs[-1] >= case["config"]["min_pair_freq"]
    assert _symbols(vocab, model) == _symbols(case["vocab_bytes"], case["model_bytes"])
    assert st["sel_rebuilds"] >= 1 and st["sel_table_pairs"] < st["sel_table_slots"]


@pytest.mark.parametrize("name", ["ascii1m_v3000_mpf2", "mixed2m_v4000"])
def test_tiebreak_device_pair_table_grows(name, case_corpus, tmp_path, monkeypatch):
    """A pair table sized below what the run needs (SHREDWORD_SELECT_TABLE_SLOTS) is grown 4x
    between launches with its live pairs moved: the same files as the default size."""
    case, corpus = case_corpus(name)
    n1, m1, v1, t1, st1 = _train(case, corpus, tmp_path, "big")
    monkeypatch.setenv("SHREDWORD_SELECT_TABLE_SLOTS", "1024")
    n2, m2, v2, t2, st2 = _train(case, corpus, tmp_path, "small")
    assert (n1, m1, v1, t1) == (n2, m2, v2, t2)
    assert st2["sel_table_grows"] >= 1 and st1["sel_table_grows"] == 0


@pytest.mark.parametrize("probes", [0, 1])
@pytest.mark.parametrize("name", ["adv_unk3_cov09", "ascii1m_v3000_mpf2", "mixed2m_v4000"])
def test_tiebreak_device_spilled_deltas(name, probes, case_corpus, tmp_path, monkeypatch):
    """Delta keys pushed out of k_word_loop<true>'s LDS hash into the HBM spill tables (the
    kernel instance with probe bound 0 or 1, SHREDWORD_WL_PROBES): the table and frontier updates
    read them back after the merge's drain; the same files as the default instance."""
    case, corpus = case_corpus(name)
    n1, m1, v1, t1, _ = _train(case, corpus, tmp_path, "lds")
    monkeypatch.setenv("SHREDWORD_WL_PROBES", str(probes))
    n2, m2, v2, t2, _ = _train(case, corpus, tmp_path, "spill")
    assert (n1, m1, v1, t1) == (n2, m2, v2, t2)
