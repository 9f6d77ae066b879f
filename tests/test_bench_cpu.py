"""bench.py's contract pieces that need no GPU: ``--gpus N`` launches N ranks itself (one process
per GPU under torch.distributed.run, rank r on device r) when no launcher set WORLD_SIZE, and the
merge-loop report divides each loop's algorithmic bytes by its own merges and launch time."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launches_n_ranks(n):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--dry-run"],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = out.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout  # stdout: rank 0's one JSON line, nothing else
    rep = json.loads(lines[0])
    assert rep["n_gpus"] == n
    # N > 1 measures ONE training by default (sharded load + merge loop on every rank), not N
    # independent jobs
    assert rep["dist"] == "replicate"
    ranks = rep["ranks"]
    assert sorted(r["rank"] for r in ranks) == list(range(n))
    assert sorted(r["local_rank"] for r in ranks) == list(range(n))
    assert len({r["pid"] for r in ranks}) == n
    assert {r["device"] for r in ranks} == {f"cuda:{i}" for i in range(n)}


def test_bench_single_rank_dry_run():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run"],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    assert rep["n_gpus"] == 1 and [r["rank"] for r in rep["ranks"]] == [0]


def test_merge_loop_report_accounting():
    sys.path.insert(0, REPO)
    import bench
    st = {k: 0 for k in ("resident_merges", "resident_kernel_ms", "resident_bytes", "resident_launches",
                         "index_merges", "index_ms", "index_candidates", "index_scanned", "index_run_ints_read",
                         "index_run_ints_written", "index_changed", "index_records", "index_dev_us", "index_undos",
                         "index_launches", "index_occurrences", "index_dev_lookup_us", "index_dev_scan_us",
                         "index_wait_us", "index_switch_merge", "index_switch_ms", "merge_launches",
                         "merge_kernel_ms", "merge_kernel_bytes", "resident_latency_us", "index_raw_records",
                         "index_finalized", "index_dev_out_us", "index_dev_fin_us", "index_fin_records")}
    st.update({f"host_{k}_seconds": 0.0 for k in ("select", "launch", "wait", "apply")})
    st.update(resident_merges=1000, resident_kernel_ms=80.0, resident_bytes=32e9, resident_launches=1,
              index_merges=30000, index_ms=500.0, index_candidates=30000 * 300, index_scanned=30000 * 100,
              index_run_ints_read=30000 * 1200, index_run_ints_written=30000 * 800, index_changed=30000 * 80,
              index_records=30000 * 120, index_dev_us=30000 * 8.0, merge_launches=31000)

    class A:
        config, layout = "zz", "types"
    rep = bench.merge_loop_report(st, 31000, 0.6, A())
    r, i = rep["resident"], rep["index"]
    assert r["algorithmic_bytes_per_merge"] == pytest.approx(32e6)
    assert r["achieved_GBps"] == pytest.approx(32e9 / 0.08 / 1e9)
    per = 16 * 300 + 8 * 100 + 4 * (1200 + 800) + 16 * 80 + 24 * 120
    assert i["algorithmic_bytes_per_merge"] == pytest.approx(per)
    assert i["achieved_GBps"] == pytest.approx(per * 30000 / 0.5 / 1e9)
    assert i["frac_of_hbm_peak"] == pytest.approx(i["achieved_GBps"] / bench.HBM_PEAK_GBS)
