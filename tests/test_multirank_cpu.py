"""World-size > 1 path on CPU (gloo): sharding by word ranges + the per-merge all-gather of every
rank's delta records must give the reference's bytes, identical on every rank (SURVEY.md §8 e1:
output bytes invariant over world size), with speculation (overlap or chains) on as on one GPU."""
import os
import socket
import subprocess
import sys

import pytest

from conftest import TESTS


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("name,layout,world,spec,chain", [
    ("small_v300", "types", 2, 1, 1), ("adv_unk0", "types", 2, 1, 1), ("adv_unkm1", "stream", 2, 1, 1),
    ("ascii1m_unk7_cov09", "types", 3, 1, 1), ("utf8_2m_v2000_mpf50", "types", 2, 1, 1),
    ("utf8_2m_v2000_mpf50", "types", 2, 0, 1), ("ascii1m_unk7_cov09", "stream", 2, 1, 4)])
def test_sharded_exchange_matches_reference(name, layout, world, spec, chain, case_corpus, tmp_path):
    case, corpus = case_corpus(name)
    cfg = case["config"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               OMP_NUM_THREADS="1")
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(TESTS, "multirank_worker.py"), corpus,
                                       str(cfg["vocab_size"]), str(cfg["unk_id"]), repr(cfg["character_coverage"]),
                                       str(cfg["min_pair_freq"]), layout, str(tmp_path), str(spec), str(chain)],
                                      env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = [p.communicate(timeout=600)[0].decode(errors="replace") for p in procs]
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    infos = [open(tmp_path / f"info_r{r}.txt").read().split() for r in range(world)]
    assert all(int(i[0]) == case["merges"] for i in infos)
    assert all(int(i[1]) > 0 for i in infos), "every rank must own a non-empty shard"
    if spec and case["merges"] > 50:
        assert all(int(i[2]) > 0 for i in infos), "speculation must confirm guesses under the exchange"
        assert len({tuple(i[2:]) for i in infos}) == 1, "every rank must make the same guesses"
    for r in range(world):
        assert open(tmp_path / f"trace_r{r}.txt").read() == case["trace"]
    assert open(tmp_path / "mr.model", "rb").read() == case["model_bytes"]
    assert open(tmp_path / "mr.vocab", "rb").read() == case["vocab_bytes"]


def test_empty_shard_rank_joins_exchange(oracle_bin, tmp_path):
    """More ranks than words: a rank with no tiles still takes part in every exchange (an empty
    bucket) and the output stays the single-rank reference's."""
    corpus = tmp_path / "tiny.txt"
    corpus.write_text("abab abab abab cdcd cdcd\n" * 3)
    world = 4
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(TESTS, "multirank_worker.py"), str(corpus), "262", "0",
                               "0.995", "2", "types", str(tmp_path), "1", "1"],
                              env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = [p.communicate(timeout=300)[0].decode(errors="replace") for p in procs]
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    infos = [open(tmp_path / f"info_r{r}.txt").read().split() for r in range(world)]
    assert any(int(i[1]) == 0 for i in infos), "the case needs a rank without tiles"
    subprocess.run([oracle_bin, str(corpus), "262", "0", "0.995", "2", str(tmp_path / "o.model"),
                    str(tmp_path / "o.vocab")], check=True, stderr=subprocess.DEVNULL)
    assert (tmp_path / "mr.model").read_bytes() == (tmp_path / "o.model").read_bytes()
    assert (tmp_path / "mr.vocab").read_bytes() == (tmp_path / "o.vocab").read_bytes()


@pytest.mark.parametrize("name,world", [("small_v300", 2), ("adv_unk0", 3), ("ascii1m_unk7_cov09", 4),
                                        ("utf8_2m_v2000_mpf50", 2), ("mixed2m_v4000", 4), ("adv_cov05", 2)])
def test_sharded_load_replicated_loop(name, world, case_corpus, tmp_path):
    """Sharded load (SURVEY.md §8 f2 multi-GPU half): every rank counts the words starting in its
    byte range, the ranks' word lists are all-gathered and merged (sums, min first occurrence,
    spellings compared), and every rank then holds the single-rank table -- same words, order,
    counts and byte cut -- and runs the merge loop replicated, with the reference's files."""
    import hostharness
    case, corpus = case_corpus(name)
    cfg = case["config"]
    lib = hostharness.load()
    h = hostharness.open_case(lib, corpus, cfg, "types")
    want = hostharness.table_fingerprint(lib, h)
    lib.hh_close(h)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               OMP_NUM_THREADS="1", SHARDED_LOAD="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(TESTS, "multirank_worker.py"), corpus,
                               str(cfg["vocab_size"]), str(cfg["unk_id"]), repr(cfg["character_coverage"]),
                               str(cfg["min_pair_freq"]), "types", str(tmp_path)],
                              env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = [p.communicate(timeout=600)[0].decode(errors="replace") for p in procs]
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    infos = [open(tmp_path / f"info_r{r}.txt").read().split() for r in range(world)]
    assert all(i[4] == want for i in infos), (want, infos)
    assert all(int(i[0]) == case["merges"] for i in infos)
    for r in range(world):
        assert open(tmp_path / f"trace_r{r}.txt").read() == case["trace"]
    assert open(tmp_path / "mr.model", "rb").read() == case["model_bytes"]
    assert open(tmp_path / "mr.vocab", "rb").read() == case["vocab_bytes"]


def _run_product_ranks(corpus, cfg, world, outdir, train=False, timeout=600, env=None):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               OMP_NUM_THREADS="1", **(env or {}))
    if train:
        env["TRAIN"] = "1"
    procs = [subprocess.Popen([sys.executable, os.path.join(TESTS, "sharded_product_worker.py"), corpus,
                               str(cfg["vocab_size"]), str(cfg["unk_id"]), repr(cfg["character_coverage"]),
                               str(cfg["min_pair_freq"]), str(outdir)],
                              env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = [p.communicate(timeout=timeout)[0].decode(errors="replace") for p in procs]
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    import json
    return [json.load(open(os.path.join(outdir, f"info_r{r}.json"))) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3])
def test_product_sharded_load_over_host_gather(world, case_corpus, tmp_path):
    """The product library's sharded load (shred_set_load_gather) with gloo as the all-gather:
    every rank counts its byte range on the host here, the merged table equals the one-process
    table (distinct words, symbols, occurrences)."""
    case, corpus = case_corpus("utf8_4m_v8192_mpf5")
    (tmp_path / "one").mkdir()
    one = _run_product_ranks(corpus, case["config"], 1, tmp_path / "one")
    many = _run_product_ranks(corpus, case["config"], world, tmp_path)
    keys = ("num_words", "num_symbols", "num_occurrences")
    assert all(tuple(i[k] for k in keys) == tuple(one[0][k] for k in keys) for i in many)


def test_product_sharded_load_gather_fallback(case_corpus, tmp_path):
    """host_load_gather(group, fallback=WORLD): when the collective on `group` raises on every rank
    (bench: the nccl group on a box where RCCL refuses it), the word lists go over the fallback
    group and the merged table is unchanged."""
    case, corpus = case_corpus("utf8_4m_v8192_mpf5")
    (tmp_path / "one").mkdir()
    one = _run_product_ranks(corpus, case["config"], 1, tmp_path / "one")
    many = _run_product_ranks(corpus, case["config"], 2, tmp_path, env={"BROKEN_GROUP": "1"})
    keys = ("num_words", "num_symbols", "num_occurrences")
    assert all(i["fell_back"] for i in many)
    assert all(tuple(i[k] for k in keys) == tuple(one[0][k] for k in keys) for i in many)


def test_product_sharded_load_gather_fallback_one_rank_fails(case_corpus, tmp_path):
    """the gather raises on ONE rank only (the others' collective returns): the ranks
    agree on a failure flag after the attempt and fall back together, so no rank waits in a gloo
    gather the others skip and every rank builds the single-rank table."""
    case, corpus = case_corpus("utf8_4m_v8192_mpf5")
    (tmp_path / "one").mkdir()
    one = _run_product_ranks(corpus, case["config"], 1, tmp_path / "one")
    many = _run_product_ranks(corpus, case["config"], 2, tmp_path, env={"BROKEN_GROUP": "last"})
    keys = ("num_words", "num_symbols", "num_occurrences")
    assert all(i["fell_back"] for i in many)
    assert all(tuple(i[k] for k in keys) == tuple(one[0][k] for k in keys) for i in many)
