"""The product Selector alone over a recorded merge stream (tests/native/selector_replay.cpp): the
CPU harness records a vocab-32000 training's initial pair counts and every merge's delta records
(HH_RECORD); the replay re-selects every merge from them and must pick the recorded merge each
time, and the engine's depth-1 guess (heap walk + replay of the coming select, then the late
correction) must beat the slot-order guess alone."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import corpora  # noqa: E402
import hostharness  # noqa: E402

REPLAY = os.path.join(HERE, "native", "_build", "selector_replay")


@pytest.fixture(scope="module")
def record(tmp_path_factory):
    d = tmp_path_factory.mktemp("replay")
    corpus, rec = str(d / "c.txt"), str(d / "c.rec")
    corpora.gen_synthetic(corpus, 4_000_000, 21, "utf8")
    lib = hostharness.load()
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "native"), "replay"], check=True)
    os.environ["HH_RECORD"] = rec
    os.environ["HH_DIRECT"] = "0"  # records combined per key, as the device ships them
    try:
        h = hostharness.open_case(lib, corpus, dict(vocab_size=32000, unk_id=0, character_coverage=0.995,
                                                     min_pair_freq=2))
        n = lib.hh_train(h, None)
        lib.hh_close(h)
    finally:
        del os.environ["HH_RECORD"]
        del os.environ["HH_DIRECT"]
    assert n > 5000
    return rec, n


def test_replay_selects_the_recorded_merges(record):
    rec, n = record
    r = subprocess.run([REPLAY, rec, "2", "0", "1"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert f"merges {n} " in r.stdout


def _hit_rate(rec, sim):
    r = subprocess.run([REPLAY, rec, "2", "0", "-1"], capture_output=True, text=True, env=dict(os.environ, SIM=sim))
    assert r.returncode == 0, r.stderr
    guesses = hits = 0.0
    for line in r.stdout.splitlines():
        if line.startswith("merges from"):
            g = int(line.split("guesses ")[1].split()[0])
            guesses += g
            hits += g * float(line.split("hit ")[1].split("%")[0]) / 100
    assert guesses > 0, r.stdout
    return hits / guesses


def test_guess_hit_rate(record):
    """The replay of the coming select beats the slot-order guess (on this small corpus late
    merges are frequency-2 ties, many with the pair the last merge created: C3 reaches 97%)."""
    rec, _ = record
    slot, sim = _hit_rate(rec, "0"), _hit_rate(rec, "1")
    assert sim > slot + 0.05 and sim > 0.7, (slot, sim)
