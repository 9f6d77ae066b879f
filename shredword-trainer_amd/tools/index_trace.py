"""Per-merge profile of the indexed merge loop (k_word_loop) on a bench config: one warm train(),
then one timed train() with the per-merge device trace on; writes the trace (npy) and prints a
summary by merge-index bucket (device µs, listed / scanned / changed words).

    python shredword-trainer_amd/tools/index_trace.py [--config c3] [--out gpurun_out/trace_c3.npy]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--out", default="gpurun_out/index_trace.npy")
    ap.add_argument("--bytes", type=int, default=0)
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    import bench
    from shredword.trainer import BPETrainer
    cfg = dict(bench.CONFIGS[args.config])
    if args.bytes:
        cfg["bytes"] = args.bytes
    path = bench.corpus_path(cfg, args.config)
    bench.ensure_corpus(cfg, path)
    t = BPETrainer(vocab_size=cfg["vocab"], unk_id=cfg["unk"], character_coverage=cfg["cov"], min_pair_freq=cfg["mpf"])
    t.set_option("log", 0)
    t.load_corpus(path)
    t._train(t.trainer)
    t.reset()
    t.set_option("timing", 1)
    t.set_option("clear_stats", 1)
    n = t._train(t.trainer)
    st = t.stats()
    tr = t.index_trace().astype(np.int64)
    t.destroy()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    np.save(args.out, tr)
    X, listed, scanned, changed, occ, dev, look, scan, s0, s1, s2, s3, idle, undo, hflag = tr.T[:15]
    rows = []
    edges = [0, 16, 64, 256, 1024, 4096, 16384, len(tr)]
    for lo, hi in zip(edges[:-1], edges[1:]):
        if lo >= len(tr):
            break
        s = slice(lo, min(hi, len(tr)))
        rows.append({"merges": f"{lo}-{min(hi, len(tr))}", "dev_us_sum": float(dev[s].sum() / 1e3),
                     "dev_us_mean": float(dev[s].mean() / 1e3), "lookup_us_mean": float(look[s].mean() / 1e3),
                     "scan_us_mean": float(scan[s].mean() / 1e3), "listed_mean": float(listed[s].mean()),
                     "scanned_mean": float(scanned[s].mean()), "changed_mean": float(changed[s].mean()),
                     "occ_mean": float(occ[s].mean()),
                     "stamps_us_mean": [float(v[s].mean() / 1e3) for v in (s0, s1, s2, s3)],
                     "dev_idle_us_mean": float(idle[s].mean() / 1e3), "dev_undo_us_mean": float(undo[s].mean() / 1e3),
                     "host_post_to_flag_us_mean": float(hflag[s].mean() / 1e3)})
        if tr.shape[1] >= 35 and tr[s, 19:35].any():  # a -DSHRED_WL_STAMPS build
            xs = tr[s, 19:35]
            # the small-merge path's stamps (word_loop.hip, SHRED_WL_STAMPS): wave 0's clock after the
            # command at each point; [1] is the shader clock in MHz, [8] 1 when the list needed no lookup
            names = ["lookup_done", "clock_MHz_x0.01", "w0_entry_landed", "w0_run_landed", "w0_walk_done",
                     "w0_deltas_issued", "w0_writeback_issued", "w0_appended", "list_given", "merge_barrier",
                     "records_stored", "before_release", "fw_start", "fw_scanned", "fw_records_issued",
                     "unused"]
            ticks = {0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11, 12, 13, 14}
            rows[-1]["stamps"] = {nm: (float(xs[:, i].mean() / 100.0) if i in ticks else float(xs[:, i].mean()))
                                  for i, nm in enumerate(names)}
            rows[-1]["stamps_p50"] = {nm: float(np.median(xs[:, i]) / 100.0) for i, nm in enumerate(names)
                                      if i in ticks}
            rows[-1]["release_us_mean"] = float((dev[s] / 1e3 - xs[:, 11] / 100.0).mean())
    print(json.dumps({"config": args.config, "merges": int(n), "train_s": st["train_seconds"],
                      "merges_per_s": n / st["train_seconds"], "dev_s_total": float(dev.sum() / 1e9),
                      "host": {k: st[f"host_{k}_seconds"] for k in ("select", "launch", "wait", "apply")},
                      "spec": [st["spec_hits"], st["spec_misses"]],
                      "build_us_per_merge": st["index_build_us"] / max(1, st["index_merges"]),
                      "no_sub": st["index_no_sub"], "staged": st["index_staged"], "buckets": rows}, indent=1))


if __name__ == "__main__":
    main()
