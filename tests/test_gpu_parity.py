"""GPU parity: the HIP path (through the C ABI via the Python drop-in) against the reference
goldens — every .model byte, .vocab byte, merge line (a, b, freq, new_id) and per-batch heap
size must match (bit-exact: integer work)."""
import os
import subprocess

import pytest

from conftest import PKG, golden_cases

pytestmark = pytest.mark.gpu


def _train(case, corpus, tmp_path, layout="types", resident=1, stats=None, index=1, spec_depth=None, speculate=None,
           hybrid=None, switch_occ=None, verify=None, **opts):
    from shredword.trainer import BPETrainer

    cfg = case["config"]
    trace = str(tmp_path / f"trace_{layout}.txt")
    t = BPETrainer(vocab_size=cfg["vocab_size"], unk_id=cfg["unk_id"],
                   character_coverage=cfg["character_coverage"], min_pair_freq=cfg["min_pair_freq"])
    t.set_option("log", 0)
    t.set_option("layout", layout)
    t.set_option("trace", trace)
    t.set_option("resident", resident)
    t.set_option("index", index)
    if hybrid is not None:
        t.set_option("hybrid", hybrid)
    if switch_occ is not None:
        t.set_option("switch_occ", switch_occ)
    if spec_depth is not None:
        t.set_option("spec_depth", spec_depth)
    if speculate is not None:
        t.set_option("speculate", speculate)
    if verify is not None:
        t.set_option("verify_argmax", verify)
    for k, v in opts.items():
        t.set_option(k, v)
    t.load_corpus(corpus)
    merges = t.train()
    model, vocab = str(tmp_path / "g.model"), str(tmp_path / "g.vocab")
    t.save(model, vocab)
    if stats is not None:
        stats.update(t.stats())
    t.destroy()
    return merges, open(model, "rb").read(), open(vocab, "rb").read(), open(trace).read()


def _check(case, got):
    merges, model, vocab, trace = got
    assert merges == case["merges"]
    assert trace == case["trace"]
    assert model == case["model_bytes"]
    assert vocab == case["vocab_bytes"]


API_CASES = [n for n in golden_cases() if not n.startswith("cli_")]
# the deep reference runs (31,744 and 63,744 merges): every path runs them too
DEEP = [n for n in API_CASES if "v32000" in n or "v64000" in n]


@pytest.mark.parametrize("name", API_CASES)
def test_types_layout_matches_reference(name, case_corpus, tmp_path):
    """Default path: hybrid — k_resident while a merge changes many words, then the indexed merge
    loop (k_word_loop: word lists, one persistent workgroup, speculation depth 1)."""
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st))
    if case["merges"] > 0 and not name.startswith("adv_"):  # (adv_: a word longer than a tile)
        assert st["resident_launches"] > 0 or st["index_merges"] >= case["merges"], st


@pytest.mark.parametrize("name", API_CASES)
def test_index_loop_matches_reference(name, case_corpus, tmp_path):
    """The indexed merge loop from the first merge (hybrid off)."""
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, hybrid=0))
    if case["merges"] > 0:
        assert st["index_merges"] >= case["merges"] and st["index_on"] == 1
        assert st["resident_launches"] == 0


@pytest.mark.parametrize("fin", [0, 8, 1024])
@pytest.mark.parametrize("name", API_CASES)
def test_index_loop_changes_on_device_match_reference(name, fin, case_corpus, tmp_path):
    """K4 on the device (round 5): k_word_loop hands the host each merge's changes combined per
    pair key and in the reference's application order (finalize_changes) for merges of at most
    `finalize` records, raw records otherwise.  0: every merge raw (the host combines and orders);
    8: both kinds within one run (<= 64 records: one wave, finalize_wave); 1024: the whole-workgroup
    finalize_changes past 64 records; the default (0, off) runs in every other test.  Same bytes."""
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, hybrid=0, finalize=fin))
    if fin == 0:
        assert st["index_finalized"] == 0
    elif case["merges"] > 50:
        assert 0 < st["index_finalized"] < st["index_merges"] + st["index_undos"], st


@pytest.mark.parametrize("name", API_CASES)
def test_large_merges_changes_on_device_match_reference(name, case_corpus, tmp_path, monkeypatch):
    """K4 on the device for the large merges only (SHREDWORD_WL_FIN_MIN=32, finalize=1024): merges of
    32..1024 records through the queued path leave as ordered changes, while the small-merge path
    (a lane per listed word) stays on for the rest and hands raw records.  Same bytes."""
    case, corpus = case_corpus(name)
    monkeypatch.setenv("SHREDWORD_WL_FIN_MIN", "32")
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, finalize=1024))


@pytest.mark.parametrize("probes", [0, 1])
@pytest.mark.parametrize("name", [n for n in API_CASES if n not in DEEP])
def test_index_loop_spilled_deltas_match_reference(name, probes, case_corpus, tmp_path, monkeypatch):
    """Delta keys pushed out of k_word_loop's LDS hash into the HBM spill tables: the kernel
    instance with the LDS probe bound 0 (every key spills) or 1 (most of a busy merge's) -- a
    template argument (SHREDWORD_WL_PROBES selects the instance), so the default kernel (32, which
    spills one or two keys in C3's 29,000 indexed merges) pays nothing for it.  The records phase
    reads the spilled keys back after the merge's store drain, which only spilling merges keep
    (word_loop.hip: `drain || S.nspill`).  Same bytes."""
    case, corpus = case_corpus(name)
    monkeypatch.setenv("SHREDWORD_WL_PROBES", str(probes))
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, hybrid=0))
    if probes == 0 and case["merges"] > 0:
        assert st["index_spill_keys"] > 0 and st["index_spill_merges"] > 0, st


@pytest.mark.parametrize("drain", [0, 1])
@pytest.mark.parametrize("name", ["small_v300", "adv_unk3_cov09", "ascii1m_v3000_mpf2", "mixed2m_v4000"])
def test_index_loop_store_drain_modes_match_reference(name, drain, case_corpus, tmp_path, monkeypatch):
    """k_word_loop's merge-end barriers: with SHREDWORD_WL_DRAIN=0 (the default) they wait on LDS
    only and the word-run / pool stores drain at the next command's barrier, which is sound only
    because nothing reads wtok, pool or lst before it (see WlParams::drain); =1 drains every
    wave's stores at the merge's end (the round-4 barriers).  Both give the reference's bytes
    (ADVICE r05)."""
    case, corpus = case_corpus(name)
    monkeypatch.setenv("SHREDWORD_WL_DRAIN", str(drain))
    _check(case, _train(case, corpus, tmp_path, "types", hybrid=0))


@pytest.mark.parametrize("path", ["hybrid", "index", "resident", "launch", "stream"])
@pytest.mark.parametrize("name", API_CASES)
def test_argmax_verifier(name, path, case_corpus, tmp_path):
    """K5 check (verify_argmax): at every checked merge the device recounts the corpus's pairs and
    reduces them (k_pair_max); the host heap's selected frequency is the largest count and the
    pair's own count -- on every merge path, with the guesses in flight undone first, and the
    files still the reference's.  Every merge is checked on the small goldens, every 97th on the
    deep runs."""
    case, corpus = case_corpus(name)
    every = 97 if name in DEEP else 1
    kw = {"hybrid": {}, "index": {"hybrid": 0}, "resident": {"index": 0}, "launch": {"index": 0, "resident": 0},
          "stream": {}}[path]
    st = {}
    _check(case, _train(case, corpus, tmp_path, "stream" if path == "stream" else "types", stats=st, verify=every, **kw))
    assert st["verify_failures"] == 0
    assert st["verify_checks"] == (case["merges"] + every - 1) // every


@pytest.mark.parametrize("switch_occ", [1 << 40, 300, 0])
@pytest.mark.parametrize("name", [n for n in API_CASES if not n.startswith("adv_") and "v64000" not in n])
def test_hybrid_switch_points(name, switch_occ, case_corpus, tmp_path):
    """The resident -> indexed switch after the first resident merge, at a mid-run merge, and
    never: the same bytes."""
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, switch_occ=switch_occ))
    if case["merges"] > 70 and switch_occ == 1 << 40:  # (the switch waits for a window of 64 merges)
        assert st["resident_launches"] > 0 and st["index_switch_merge"] >= 256 and st["index_merges"] > 0
    if switch_occ == 0 and case["merges"] > 0:
        assert st["index_merges"] == 0 and st["index_switch_merge"] == -1


@pytest.mark.parametrize("name", API_CASES)
def test_index_loop_no_speculation_matches_reference(name, case_corpus, tmp_path):
    """The indexed loop one merge at a time (no guesses, so no undo)."""
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, speculate=0, hybrid=0))
    assert st["index_undos"] == 0


@pytest.mark.parametrize("name", API_CASES)
def test_index_loop_deep_speculation_matches_reference(name, case_corpus, tmp_path):
    """The indexed loop with three guesses in flight behind the current merge (undone exactly
    when the replay picks otherwise)."""
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, spec_depth=3, hybrid=0))
    if case["merges"] > 200:
        assert st["index_undos"] > 0 and st["spec_hits"] > 0


@pytest.mark.parametrize("name", API_CASES)
def test_types_layout_resident_matches_reference(name, case_corpus, tmp_path):
    """The LDS-resident tile loop (k_resident) wherever the table fits; the adversarial corpora
    hold a word longer than one tile and take the launch path."""
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, index=0))
    if case["merges"] > 0 and not name.startswith("adv_"):
        assert st["resident_launches"] > 0


@pytest.mark.parametrize("name", [n for n in API_CASES if not n.startswith("adv_")])
def test_types_layout_resident_hbm_matches_reference(name, case_corpus, tmp_path, monkeypatch):
    """k_resident with the tokens kept in HBM (LDS holds weights and signatures)."""
    monkeypatch.setenv("SHREDWORD_RESIDENT_HBM", "1")
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, index=0))
    if case["merges"] > 0:
        assert st["resident_launches"] > 0


@pytest.mark.parametrize("plan", [("32", "1", "1"), ("64", "1", "3")], ids=["sig1024_wglobal", "sig2048_depth3"])
@pytest.mark.parametrize("name", [n for n in API_CASES if not n.startswith("adv_")])
def test_types_layout_resident_small_plan_matches_reference(name, plan, case_corpus, tmp_path, monkeypatch):
    """k_resident's plans for tables too big for the default LDS plan (C5 at 100 GB: 68,905 tiles
    of 4.1 M words): weights read from HBM and the per-tile signatures quartered / halved
    (SHREDWORD_RESIDENT_SIG_WORDS forces them here), with one and with three guesses in flight."""
    sig, wg, depth = plan
    monkeypatch.setenv("SHREDWORD_RESIDENT_SIG_WORDS", sig)
    monkeypatch.setenv("SHREDWORD_RESIDENT_W_GLOBAL", wg)
    monkeypatch.setenv("SHREDWORD_SPEC_DEPTH", depth)
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", stats=st, index=0))
    if case["merges"] > 0:
        assert st["resident_launches"] > 0


@pytest.mark.parametrize("name", [n for n in API_CASES if not n.startswith("adv_")])
def test_types_layout_resident_deep_speculation_matches_reference(name, case_corpus, tmp_path, monkeypatch):
    """k_resident with three guessed merges in flight behind the current one."""
    monkeypatch.setenv("SHREDWORD_SPEC_DEPTH", "3")
    case, corpus = case_corpus(name)
    _check(case, _train(case, corpus, tmp_path, "types", index=0))


@pytest.mark.parametrize("name", API_CASES)
def test_types_layout_launch_path_matches_reference(name, case_corpus, tmp_path):
    """The per-merge launch path (k_merge + speculation + k_unmerge), both loops off."""
    case, corpus = case_corpus(name)
    st = {}
    _check(case, _train(case, corpus, tmp_path, "types", resident=0, stats=st, index=0))
    assert st["resident_launches"] == 0


@pytest.mark.parametrize("name", ["c1_ascii10m_v8192", "ascii1m_v3000_mpf2", "adv_unk0", "adv_unkm1",
                                  "ascii1m_unk7_cov09", "small_v300"])
def test_stream_layout_matches_reference(name, case_corpus, tmp_path):
    case, corpus = case_corpus(name)
    _check(case, _train(case, corpus, tmp_path, "stream"))


@pytest.mark.parametrize("name", [n for n in golden_cases() if n.startswith("cli_")])
def test_cli_matches_reference(name, case_corpus, tmp_path):
    case, corpus = case_corpus(name)
    cfg = case["config"]
    model, vocab = str(tmp_path / "c.model"), str(tmp_path / "c.vocab")
    proc = subprocess.run([os.path.join(PKG, "bin", "trainer"), f"input={corpus}", "model_type=bpe",
                           f"output_model={model}", f"output_vocab={vocab}",
                           f"vocab_size={cfg['vocab_size']}", f"character_coverage={cfg['character_coverage']}",
                           f"min_pair_freq={cfg['min_pair_freq']}"],
                          stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=dict(os.environ, SHREDWORD_LOG="0"))
    assert proc.returncode == 0, proc.stderr  # the reference CLI segfaults here (rc 139)
    assert open(model, "rb").read() == case["model_bytes"]
    assert open(vocab, "rb").read() == case["vocab_bytes"]


@pytest.mark.parametrize("name", ["utf8_4m_v8192_mpf5", "mixed2m_v4000"])
def test_sharded_load_two_processes_on_gpu(name, case_corpus, tmp_path):
    """Two processes on the GPU, the product library end to end (dist=replicate without RCCL):
    each rank counts its byte range with k_word_count, the word lists meet over a gloo all-gather
    (shred_set_load_gather), and each rank trains the merged table on the device -- both ranks
    write the reference's bytes."""
    from test_multirank_cpu import _run_product_ranks
    case, corpus = case_corpus(name)
    infos = _run_product_ranks(corpus, case["config"], 2, tmp_path, train=True, env={"SHREDWORD_GPU_LOAD_MIN": "1"})
    assert all(i["load_on_gpu"] == 1 and i["merges"] == case["merges"] for i in infos)
    for r in range(2):
        assert open(tmp_path / f"r{r}.model", "rb").read() == case["model_bytes"]
        assert open(tmp_path / f"r{r}.vocab", "rb").read() == case["vocab_bytes"]


@pytest.mark.parametrize("path", ["hybrid", "index", "resident"])
@pytest.mark.parametrize("name", ["adv_cov05", "ascii1m_v3000_mpf2", "mixed2m_v4000", "utf8_4m_v8192_mpf5",
                                  "utf8_24m_v32000_mpf2"])
def test_opt_in_host_pipelining_matches_reference(name, path, case_corpus, tmp_path):
    """The opt-in host pipelining (early_guess: two guesses in flight; apply_helper: a second host
    thread combining the guessed merge's records) on the merge paths: the reference's bytes."""
    case, corpus = case_corpus(name)
    kw = {"hybrid": {}, "index": {"hybrid": 0}, "resident": {"index": 0}}[path]
    st = {}
    _check(case, _train(case, corpus, tmp_path, stats=st, early_guess=1, apply_helper=1, **kw))
