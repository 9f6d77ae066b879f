"""The product host logic under AddressSanitizer + UBSan (CPU, no GPU).

tests/native builds the CPU harness (product corpus loader, tile packing, Engine, Selector + the
kernel emulation) as one sanitized executable (`make -C tests/native asan`); it trains on golden
corpora in both layouts (and with a guessed chain) and must exit cleanly -- no memory error, leak
or undefined behaviour (halt_on_error) -- with the reference's files byte for byte.
"""
import os
import subprocess

import pytest

from conftest import load_case

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "native", "_build", "hh_asan")
ENV = dict(os.environ,
           # the sanitizer runtime is linked into the executable; the link-order check would
           # trip over libraries the environment preloads
           ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def asan_exe():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "native"), "asan"], check=True)
    return EXE


@pytest.mark.parametrize("name,layout,chain", [
    ("small_v300", 0, 1), ("small_cov0_mpf0", 0, 1), ("small_v50_zero", 0, 1),
    ("adv_unk0", 0, 1), ("adv_unkm1", 1, 1), ("adv_unk3_cov09", 0, 4),
    ("ascii1m_unkm1_mpf2", 0, 1), ("ascii1m_v3000_mpf2", 1, 1), ("utf8_2m_v2000_mpf50", 0, 4),
    ("mixed2m_v4000", 0, 1),
])
def test_host_logic_under_sanitizers(name, layout, chain, asan_exe, case_corpus, tmp_path):
    case, corpus = case_corpus(name)
    c = case["config"]
    model, vocab, trace = (str(tmp_path / f) for f in ("a.model", "a.vocab", "a.trace"))
    r = subprocess.run([asan_exe, corpus, str(c["vocab_size"]), str(c["unk_id"]), repr(c["character_coverage"]),
                        str(c["min_pair_freq"]), str(layout), model, vocab, trace, str(chain)],
                       env=ENV, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert int(r.stdout.split()[-1]) == case["merges"]
    assert open(model, "rb").read() == case["model_bytes"]
    assert open(vocab, "rb").read() == case["vocab_bytes"]
    assert open(trace).read() == case["trace"]
