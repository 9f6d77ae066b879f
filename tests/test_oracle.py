"""Pins the CPU restatement (oracle/bpe_oracle.c) to the reference's golden outputs.

The goldens were produced by the reference's own sources (zero-initialised build, SURVEY.md
§8 c1) via tests/golden/make_golden.py; this test checks the restatement reproduces every
.model byte, .vocab byte, [MERGE] line and per-batch heap size, so it may serve as the parity
checker for the HIP path and as the CPU baseline.
"""
import concurrent.futures
import os
import subprocess

import pytest

from conftest import golden_cases, seq_cases


@pytest.fixture(scope="session")
def oracle_runs(case_corpus, oracle_bin, tmp_path_factory):
    """Every golden's oracle run, started together on a pool of host cores (the deep cases,
    31,744 and 63,744 merges of a reference-cost O(S) loop, take minutes each)."""
    out = tmp_path_factory.mktemp("oracle_runs")
    pool = concurrent.futures.ThreadPoolExecutor(max_workers=max(2, (os.cpu_count() or 4) - 1))

    def run(name, case, corpus):
        cfg = case["config"]
        model, vocab, trace = (str(out / f"{name}.{n}") for n in ("model", "vocab", "trace"))
        # the deep cases split their O(S) scans over 4 threads (same output, oracle --threads)
        threads = ["--threads", "4"] if case["merges"] > 20000 else []
        subprocess.run([oracle_bin, corpus, str(cfg["vocab_size"]), str(cfg["unk_id"]),
                        repr(cfg["character_coverage"]), str(cfg["min_pair_freq"]), model, vocab,
                        "--trace", trace] + threads, check=True, stderr=subprocess.DEVNULL)
        return model, vocab, trace

    cases = {n: case_corpus(n) for n in golden_cases()}
    # longest first: the deep runs set the wall time
    order = sorted(cases, key=lambda n: -cases[n][0]["merges"])
    futs = {n: pool.submit(run, n, *cases[n]) for n in order}
    yield lambda n: futs[n].result()
    pool.shutdown(wait=True)


@pytest.mark.parametrize("name", seq_cases())
def test_oracle_call_sequence_matches_reference(name, seq_case, oracle_bin, tmp_path):
    """The restatement driven through the same call sequence as the reference's golden (load twice,
    train twice, init + merge_batch, counts on a stale pair map ...): every save's files, every
    [MERGE]/batch line and every call's return value."""
    case, ops = seq_case(name)
    cfg = case["config"]
    argv, nsave = [], 0
    for op in ops:
        if op[0] == "load":
            argv.append("load=" + op[1])
        elif op[0] == "batch":
            argv.append(f"batch={op[1]}")
        elif op[0] == "save":
            argv.append(f"save={tmp_path}/m{nsave},{tmp_path}/v{nsave}")
            nsave += 1
        else:
            argv.append(op[0])
    trace = str(tmp_path / "trace")
    subprocess.run([oracle_bin, "--script", str(cfg["vocab_size"]), str(cfg["unk_id"]), repr(cfg["character_coverage"]),
                    str(cfg["min_pair_freq"]), trace] + argv, check=True)
    assert open(trace).read() == case["trace"]
    for i, (model, vocab) in enumerate(case["outputs"]):
        assert open(tmp_path / f"m{i}", "rb").read() == model, f"save {i}: .model"
        assert open(tmp_path / f"v{i}", "rb").read() == vocab, f"save {i}: .vocab"


@pytest.mark.parametrize("name", golden_cases())
def test_oracle_matches_reference_golden(name, case_corpus, oracle_runs):
    case, _ = case_corpus(name)
    model, vocab, trace = oracle_runs(name)
    assert open(model, "rb").read() == case["model_bytes"]
    assert open(vocab, "rb").read() == case["vocab_bytes"]
    assert open(trace).read() == case["trace"]
    assert os.path.getsize(model) == 12 * case["merges"]
