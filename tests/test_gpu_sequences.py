"""GPU parity of the stateful drop-in call sequences (missing 2).

Each golden under tests/golden/seq was produced by the zero-initialised reference driven through
a sequence of its C-ABI calls on one trainer (oracle/ref_driver.c --script, make_golden.py
SEQ_CASES): a second load (the last corpus wins, the merges and the heap stay; bpe.cpp:176-183),
a second train (bpe_init re-counts the merged words, ids continue at 256 + num_merges;
:98-108, :345-386), bpe_init + bpe_merge_batch then train/save (:232-323), and sequences in which
the pair map is not the corpus's count (a count on a counted map, a batch after a reload without a
count), where the reference's recompute_freq rescan (:52-65, :251-257) decides.  Here the same
calls go through the product's C ABI (BPETrainer + cbase.lib) on every merge path; every return
value, every [MERGE]/batch line and every save's .model/.vocab bytes must equal the reference's.
"""
import pytest

from conftest import seq_cases

pytestmark = pytest.mark.gpu

PATHS = {
    "hybrid": {},                             # default: k_resident, then the indexed loop
    "index": {"hybrid": 0},                   # the indexed loop from the first merge
    "resident": {"index": 0},                 # k_resident alone
    "launch": {"index": 0, "resident": 0},    # one k_merge launch per merge
    "stream": {"layout": "stream"},           # every occurrence in corpus order
}


def run_script_gpu(case, ops, tmp_path, **opts):
    from shredword.cbase import lib
    from shredword.trainer import BPETrainer

    cfg = case["config"]
    t = BPETrainer(vocab_size=cfg["vocab_size"], unk_id=cfg["unk_id"],
                   character_coverage=cfg["character_coverage"], min_pair_freq=cfg["min_pair_freq"])
    trace = str(tmp_path / "seq_trace.txt")
    try:
        t.set_option("log", 0)
        t.set_option("trace", trace)
        t.set_option("device", 0)
        for k, v in opts.items():
            t.set_option(k, v)
        outputs, returns = [], []
        for op in ops:
            ret = 0
            if op[0] == "load":
                ret = lib.bpe_load_corpus(t.trainer, op[1].encode())
            elif op[0] == "init":
                lib.bpe_init(t.trainer)
            elif op[0] == "count":
                lib.bpe_count_bigrams(t.trainer)
            elif op[0] == "batch":
                ret = lib.bpe_merge_batch(t.trainer, op[1])
            elif op[0] == "train":
                ret = lib.bpe_train(t.trainer)
            elif op[0] == "save":
                m, v = str(tmp_path / f"m{len(outputs)}"), str(tmp_path / f"v{len(outputs)}")
                t.save(m, v)
                outputs.append((open(m, "rb").read(), open(v, "rb").read()))
            returns.append([op[0], str(ret)])
            t.set_option("trace_note", f"S {op[0]} {ret}")
        stats = t.stats()
    finally:
        t.destroy()
    return open(trace).read(), outputs, returns, stats


@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("name", seq_cases())
def test_call_sequence_matches_reference(name, path, seq_case, tmp_path):
    case, ops = seq_case(name)
    trace, outputs, returns, _ = run_script_gpu(case, ops, tmp_path, **PATHS[path])
    assert returns == case["returns"]
    assert trace == case["trace"]
    for i, (got, want) in enumerate(zip(outputs, case["outputs"])):
        assert got[0] == want[0], f"save {i}: .model"
        assert got[1] == want[1], f"save {i}: .vocab"
    assert len(outputs) == len(case["outputs"])
