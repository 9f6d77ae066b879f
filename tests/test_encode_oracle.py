"""The encoder's checker (oracle/encode_oracle.c) pinned by the reference's own outputs: encoding a
golden corpus with the reference's .model gives id counts equal to the reference's .vocab
frequency column (the trainer's final segmentation).  Corpora with NUL bytes are
skipped: there the reference's fgets/strlen reading hides part of the file (bpe.cpp:131-153)."""
import numpy as np
import pytest

from conftest import golden_cases
from encode_ref import derived_byte_map, id_counts, model_merges, oracle_encode, token_bytes, vocab_freqs

CASES = [c for c in golden_cases() if not c.startswith("cli_")]


@pytest.mark.parametrize("name", CASES)
def test_oracle_encoding_reproduces_reference_vocab_counts(name, case_corpus):
    case, path = case_corpus(name)
    text = open(path, "rb").read()
    if b"\0" in text:
        pytest.skip("NUL bytes: the reference reads only part of each line")
    merges = model_merges(case["model_bytes"])
    toks = token_bytes(merges)
    freqs = vocab_freqs(case["vocab_bytes"], toks)
    unk = case["config"]["unk_id"]
    ids = oracle_encode(merges, derived_byte_map(merges, freqs, unk), text)
    assert np.array_equal(id_counts(ids, len(toks)), freqs)


def test_oracle_encode_semantics_small():
    # merges: (a,a)->256, (256,a)->257, (b,c)->258
    merges = [[97, 97, 256], [256, 97, 257], [98, 99, 258]]
    assert oracle_encode(merges, None, b"aaa").tolist() == [257]          # aa first, then (aa)a
    assert oracle_encode(merges, None, b"aaaa").tolist() == [256, 256]    # left to right, no overlap
    assert oracle_encode(merges, None, b" abc\tbc\n").tolist() == [97, 258, 258]
    assert oracle_encode(merges, None, b"").tolist() == []
    assert oracle_encode(merges, None, b" \r\n\t ").tolist() == []
    with pytest.raises(ValueError):
        oracle_encode(merges, None, b"x" * 1025)
