"""CPU tests of the product host logic (no GPU).

The product's corpus loader, tile packing, Engine (reference batch loop / trace) and Selector
(exact heap replay and FreqChangeMap ordering) run against a CPU emulation of the device
kernels (tests/native/host_harness.cpp) and must reproduce the reference goldens byte for byte.
This pins everything on the host side of the C ABI; the GPU tests pin the kernels themselves.
"""
import os

import pytest

import hostharness
from conftest import golden_cases, seq_cases


@pytest.fixture(scope="module")
def hh():
    return hostharness.load()


def _run(hh, case, corpus, tmp_path, layout):
    h = hostharness.open_case(hh, corpus, case["config"], layout)
    try:
        trace = str(tmp_path / f"t_{layout}.txt")
        merges = hh.hh_train(h, trace.encode())
        model, vocab = str(tmp_path / "h.model"), str(tmp_path / "h.vocab")
        hh.hh_save(h, model.encode(), vocab.encode(), 1)
        return merges, open(model, "rb").read(), open(vocab, "rb").read(), open(trace).read()
    finally:
        hh.hh_close(h)


@pytest.mark.parametrize("name", golden_cases())
def test_host_logic_types_layout(name, hh, case_corpus, tmp_path):
    case, corpus = case_corpus(name)
    merges, model, vocab, trace = _run(hh, case, corpus, tmp_path, "types")
    assert merges == case["merges"]
    assert trace == case["trace"]
    assert model == case["model_bytes"]
    assert vocab == case["vocab_bytes"]


@pytest.mark.parametrize("name", ["adv_unk0", "adv_unkm1", "ascii1m_unk7_cov09", "small_v300", "utf8_2m_v2000_mpf50"])
def test_host_logic_stream_layout(name, hh, case_corpus, tmp_path):
    case, corpus = case_corpus(name)
    merges, model, vocab, trace = _run(hh, case, corpus, tmp_path, "stream")
    assert (merges, trace, model, vocab) == (case["merges"], case["trace"], case["model_bytes"], case["vocab_bytes"])


def _py_word_table(data: bytes):
    """Appendix A.1 restated for NUL-free text: words split on TAB/CR/LF/SPACE, ordered by
    (djb2(word) & 4095, first occurrence)."""
    import re
    first, count = {}, {}
    for m in re.finditer(rb"[^\t\r\n ]+", data):
        w = m.group()
        if w not in first:
            first[w] = len(first)
        count[w] = count.get(w, 0) + 1

    def djb2(w):
        x = 5381
        for c in w:
            x = (x * 33 + c) & 0xFFFFFFFFFFFFFFFF
        return x
    words = sorted(first, key=lambda w: (djb2(w) & 4095, first[w]))
    return [(w, count[w]) for w in words]


@pytest.mark.parametrize("name", ["small_v300", "ascii1m_v3000_mpf2", "utf8_2m_v2000_mpf50"])
def test_word_order_matches_python_restatement(name, hh, case_corpus):
    import ctypes
    case, corpus = case_corpus(name)
    h = hostharness.open_case(hh, corpus, case["config"])
    try:
        want = _py_word_table(open(corpus, "rb").read())
        assert hh.hh_num_words(h) == len(want)
        buf = ctypes.create_string_buffer(4096)
        cnt = ctypes.c_uint64()
        for i, (w, c) in enumerate(want):
            ln = hh.hh_word(h, i, buf, len(buf), ctypes.byref(cnt))
            assert (buf.raw[:ln], cnt.value) == (w, c), i
        # coverage: keep = (size_t)(float(n) * float(coverage)) (bpe.cpp:169)
        import numpy as np
        n = hh.hh_distinct_bytes(h)
        assert hh.hh_kept_bytes(h) == int(np.float32(n) * np.float32(case["config"]["character_coverage"]))
    finally:
        hh.hh_close(h)


def test_merge_batch_matches_train(hh, case_corpus, tmp_path):
    """bpe_init + repeated bpe_merge_batch reproduces bpe_train's merges (batching is logging-only)."""
    case, corpus = case_corpus("small_v300")
    h = hostharness.open_case(hh, corpus, case["config"])
    try:
        hh.hh_init(h)
        total = 0
        while True:
            n = hh.hh_merge_batch(h, 7)
            if n <= 0 or total + n > case["merges"]:
                total += max(n, 0)
                break
            total += n
            if total >= case["merges"]:
                break
        model, vocab = str(tmp_path / "b.model"), str(tmp_path / "b.vocab")
        hh.hh_save(h, model.encode(), vocab.encode(), 1)
        got = open(model, "rb").read()
        assert got[:len(case["model_bytes"])] == case["model_bytes"]
    finally:
        hh.hh_close(h)


def run_script_harness(hh, case, ops, tmp_path):
    """One emulated trainer through a golden's call sequence: (trace, outputs, returns)."""
    cfg = case["config"]
    h = hh.hh_create(cfg["vocab_size"], cfg["unk_id"], cfg["character_coverage"], cfg["min_pair_freq"])
    trace = str(tmp_path / "seq_trace.txt")
    hh.hh_set_trace(h, trace.encode())
    hh.hh_set_verify_exact(h, 1)  # the selector's exact() claim checked against a fresh K1 after every op
    outputs, returns = [], []
    try:
        for op in ops:
            ret = 0
            if op[0] == "load":
                ret = hh.hh_load(h, op[1].encode())
            elif op[0] == "init":
                hh.hh_init(h)
            elif op[0] == "count":
                hh.hh_count(h)
            elif op[0] == "batch":
                ret = hh.hh_merge_batch(h, op[1])
            elif op[0] == "train":
                ret = hh.hh_train(h, b"")
            elif op[0] == "save":
                m, v = str(tmp_path / f"m{len(outputs)}"), str(tmp_path / f"v{len(outputs)}")
                hh.hh_save(h, m.encode(), v.encode(), 1)
                outputs.append((open(m, "rb").read(), open(v, "rb").read()))
            returns.append([op[0], str(ret)])
            hh.hh_trace_line(h, f"S {op[0]} {ret}\n".encode())
        assert hh.hh_exact_failures(h) == 0, "the selector claimed exact counts that a fresh K1 contradicts"
    finally:
        hh.hh_close(h)
    return open(trace).read(), outputs, returns


@pytest.mark.parametrize("name", seq_cases())
def test_host_logic_call_sequences(name, hh, seq_case, tmp_path):
    """The product's host code (Engine reload / count / merge_batch / train, the Selector's pair-map
    exactness and truth table) through the reference's stateful call sequences, over the emulated
    kernels: the reference's trace, every save's bytes and every return value."""
    case, ops = seq_case(name)
    trace, outputs, returns = run_script_harness(hh, case, ops, tmp_path)
    assert returns == case["returns"]
    assert trace == case["trace"]
    assert outputs == case["outputs"]


TIEBREAK_CASES = ["small_v300", "adv_unk0", "adv_unk3_cov09", "ascii1m_unk7_cov09", "ascii1m_v3000_mpf2",
                  "utf8_2m_v2000_mpf50", "ascii1m_unkm1_mpf2"]


@pytest.mark.parametrize("phase", [0, 7, 100000])
@pytest.mark.parametrize("name", TIEBREAK_CASES)
def test_tiebreak_device_host_logic_matches_oracle_rule(name, phase, hh, case_corpus, oracle_bin, tmp_path):
    """tiebreak=device (opt-in, not the reference's order): the Engine's device-selection path over
    the emulated kernels (EmuBackend::device_select: the pair-table rule of k_word_loop<true>)
    against the oracle's restatement of the same rule (bpe_oracle --tiebreak-device 0: largest
    count, ties to the smaller key, every count the reference's): the same merges and files.
    `phase`: the first merges selected on the host by the same rule (the device's resident phase,
    Engine::train_device) -- none, 7, or every merge."""
    import subprocess
    case, corpus = case_corpus(name)
    cfg = case["config"]
    h = hostharness.open_case(hh, corpus, cfg, "types")
    try:
        hh.hh_set_tiebreak_device(h, 1)
        hh.hh_set_device_phase(h, phase)
        trace = str(tmp_path / "t.txt")
        merges = hh.hh_train(h, trace.encode())
        assert hh.hh_host_phase_merges(h) == min(phase, merges)
        m, v = str(tmp_path / "h.model"), str(tmp_path / "h.vocab")
        hh.hh_save(h, m.encode(), v.encode(), 1)
    finally:
        hh.hh_close(h)
    om, ov, ot = (str(tmp_path / f"o.{k}") for k in ("model", "vocab", "trace"))
    subprocess.run([oracle_bin, corpus, str(cfg["vocab_size"]), str(cfg["unk_id"]), repr(cfg["character_coverage"]),
                    str(cfg["min_pair_freq"]), om, ov, "--trace", ot, "--tiebreak-device", "0"], check=True,
                   stderr=subprocess.DEVNULL)
    assert open(trace).read() == open(ot).read()
    assert open(m, "rb").read() == open(om, "rb").read()
    assert open(v, "rb").read() == open(ov, "rb").read()
    assert merges == os.path.getsize(om) // 12


@pytest.mark.parametrize("name", ["adv_unk0", "adv_cov05", "utf8_2m_v2000_mpf50"])
def test_sharded_load_ranges_match_reference(name, hh, case_corpus, tmp_path, monkeypatch):
    """The sharded load's word lists (3 byte ranges counted in turn, shipped with their spellings and
    merged) give the reference's files; a range holding a NUL byte (the adversarial corpora) sends
    every rank to the whole-file fgets/strlen path instead."""
    monkeypatch.setenv("SHREDWORD_LOAD_SIM_SHARDS", "3")
    case, corpus = case_corpus(name)
    merges, model, vocab, trace = _run(hh, case, corpus, tmp_path, "types")
    assert merges == case["merges"]
    assert model == case["model_bytes"] and vocab == case["vocab_bytes"]


@pytest.mark.parametrize("name", ["ascii1m_v3000_mpf2", "utf8_4m_v8192_mpf5", "mixed2m_v4000", "adv_unk3_cov09"])
def test_apply_helper_gives_the_reference_bytes(name, hh, case_corpus, tmp_path):
    """The opt-in host pipelining -- the apply helper (a second host thread combining and ordering
    the guessed merge's records while the selector selects) and the early guess (two guesses in
    flight) -- on and off: both the reference's trace and files, and the helper actually took
    merges when on."""
    case, corpus = case_corpus(name)
    for on in (1, 0):
        h = hostharness.open_case(hh, corpus, case["config"], "types")
        try:
            hh.hh_set_apply_helper(h, on)
            hh.hh_set_early_guess(h, on)
            trace = str(tmp_path / f"t{on}.txt")
            merges = hh.hh_train(h, trace.encode())
            used = hh.hh_helper_used(h)
            m, v = str(tmp_path / f"h{on}.model"), str(tmp_path / f"h{on}.vocab")
            hh.hh_save(h, m.encode(), v.encode(), 1)
        finally:
            hh.hh_close(h)
        assert merges == case["merges"]
        assert open(trace).read() == case["trace"]
        assert open(m, "rb").read() == case["model_bytes"] and open(v, "rb").read() == case["vocab_bytes"]
        assert (used > merges // 2) if on else used == 0


_POST_GUESSES = r"""
import ctypes, sys
sys.path.insert(0, {tests!r})
import hostharness
lib = hostharness.load()
h = hostharness.open_case(lib, {corpus!r}, {cfg!r})
lib.hh_init(h)
lib.hh_set_max_guesses(h, {max_guesses})
ab = (ctypes.c_int32 * 4)(116, 104, 101, 32)
print("IN_FLIGHT", lib.hh_post_guesses(h, ab, 2, 256), flush=True)
"""


@pytest.mark.parametrize("max_guesses", [1, 2])
def test_backend_refuses_a_guess_past_its_depth(max_guesses, case_corpus, tmp_path):
    """a backend that holds one guess (the launch path) must refuse a second
    unconfirmed one with a fatal error instead of running it (the stream layout miscounted with
    two).  Two guesses through Backend::post_guess: refused at max_guesses 1, held at 2."""
    import subprocess
    import sys
    case, corpus = case_corpus("small_v300")
    code = _POST_GUESSES.format(tests=os.path.dirname(os.path.abspath(__file__)), corpus=corpus,
                                cfg=case["config"], max_guesses=max_guesses)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    if max_guesses == 1:
        assert p.returncode != 0
        assert "more unconfirmed guesses than the backend holds" in p.stderr
        assert "IN_FLIGHT" not in p.stdout
    else:
        assert p.returncode == 0, p.stderr
        assert "IN_FLIGHT 2" in p.stdout


def test_batch_after_tiebreak_device_train_rebuilds_the_heap(hh, case_corpus, tmp_path):
    """train() under tiebreak=device selects on the device and never fills the host
    heap; a bpe_merge_batch after it must still merge (the heap is rebuilt from a fresh K1 of the
    merged corpus, as bpe_init would build it), not return 0.  Same files as an explicit
    bpe_init before the batch."""
    case, corpus = case_corpus("utf8_2m_v2000_mpf50")
    cfg = dict(case["config"], vocab_size=1000)
    out = []
    for explicit_init in (False, True):
        h = hostharness.open_case(hh, corpus, cfg, "types")
        try:
            hh.hh_set_tiebreak_device(h, 1)
            hh.hh_set_device_phase(h, 0)
            first = hh.hh_train(h, None)
            assert first == 1000 - 256
            if explicit_init:
                hh.hh_init(h)
            got = hh.hh_merge_batch(h, 25)
            m, v = str(tmp_path / f"m{int(explicit_init)}"), str(tmp_path / f"v{int(explicit_init)}")
            hh.hh_save(h, m.encode(), v.encode(), 1)
            out.append((got, open(m, "rb").read(), open(v, "rb").read()))
        finally:
            hh.hh_close(h)
    assert out[0][0] == 25
    assert out[0] == out[1]
    assert len(out[0][1]) == 12 * (1000 - 256 + 25)


@pytest.mark.parametrize("name", golden_cases())
def test_host_logic_with_device_ordered_changes(name, hh, case_corpus, tmp_path, monkeypatch):
    """K4 on the device (round 5): the backend hands the host the merge's changes already combined
    per pair key and in the reference's application order (Backend::records_are_changes; on the GPU
    k_word_loop's finalize_changes).  The emulation builds them the reference's way (a 1024-bucket
    FreqChangeMap fed in first-touch order); the host then only walks them
    (Selector::apply_changes) and must still give the reference's bytes."""
    monkeypatch.setenv("HH_FINALIZE", "1")
    case, corpus = case_corpus(name)
    merges, model, vocab, trace = _run(hh, case, corpus, tmp_path, "types")
    assert (merges, trace, model, vocab) == (case["merges"], case["trace"], case["model_bytes"], case["vocab_bytes"])


@pytest.mark.parametrize("name", seq_cases())
def test_host_logic_call_sequences_with_device_ordered_changes(name, hh, seq_case, tmp_path, monkeypatch):
    monkeypatch.setenv("HH_FINALIZE", "1")
    case, ops = seq_case(name)
    trace, outputs, returns = run_script_harness(hh, case, ops, tmp_path)
    assert (returns, trace, outputs) == (case["returns"], case["trace"], case["outputs"])
