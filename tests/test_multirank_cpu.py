"""World-size > 1 path on CPU (gloo): sharding by word ranges + per-merge all-reduce of the delta
tables must give the reference's bytes, identical on every rank (output bytes
invariant over world size)."""
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


@pytest.mark.parametrize("name,layout,world", [("small_v300", "types", 2), ("adv_unk0", "types", 2),
                                               ("adv_unkm1", "stream", 2), ("ascii1m_unk7_cov09", "types", 3),
                                               ("utf8_2m_v2000_mpf50", "types", 2)])
def test_sharded_exchange_matches_reference(name, layout, world, case_corpus, tmp_path):
    case, corpus = case_corpus(name)
    cfg = case["config"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               OMP_NUM_THREADS="1")
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(TESTS, "multirank_worker.py"), corpus,
                                       str(cfg["vocab_size"]), str(cfg["unk_id"]), repr(cfg["character_coverage"]),
                                       str(cfg["min_pair_freq"]), layout, str(tmp_path)],
                                      env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = [p.communicate(timeout=600)[0].decode(errors="replace") for p in procs]
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    infos = [open(tmp_path / f"info_r{r}.txt").read().split() for r in range(world)]
    assert all(int(i[0]) == case["merges"] for i in infos)
    assert all(int(i[1]) > 0 for i in infos), "every rank must own a non-empty shard"
    for r in range(world):
        assert open(tmp_path / f"trace_r{r}.txt").read() == case["trace"]
    assert open(tmp_path / "mr.model", "rb").read() == case["model_bytes"]
    assert open(tmp_path / "mr.vocab", "rb").read() == case["vocab_bytes"]
