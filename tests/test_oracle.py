"""Pins the CPU restatement (oracle/bpe_oracle.c) to the reference's golden outputs.

The goldens were produced by the reference's own sources (zero-initialised build, SURVEY.md
§8 c1) via tests/golden/make_golden.py; this test checks the restatement reproduces every
.model byte, .vocab byte, [MERGE] line and per-batch heap size, so it may serve as the parity
checker for the HIP path and as the CPU baseline.
"""
import os
import subprocess

import pytest

from conftest import golden_cases


@pytest.mark.parametrize("name", golden_cases())
def test_oracle_matches_reference_golden(name, case_corpus, oracle_bin, tmp_path):
    case, corpus = case_corpus(name)
    cfg = case["config"]
    model, vocab, trace = (str(tmp_path / n) for n in ("o.model", "o.vocab", "o.trace"))
    subprocess.run([oracle_bin, corpus, str(cfg["vocab_size"]), str(cfg["unk_id"]),
                    repr(cfg["character_coverage"]), str(cfg["min_pair_freq"]), model, vocab,
                    "--trace", trace], check=True, stderr=subprocess.DEVNULL)
    assert open(model, "rb").read() == case["model_bytes"]
    assert open(vocab, "rb").read() == case["vocab_bytes"]
    assert open(trace).read() == case["trace"]
    assert os.path.getsize(model) == 12 * case["merges"]
