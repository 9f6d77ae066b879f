#!/usr/bin/env python3
"""Diagnostic: round-trip cost of a device merge that changes nothing (a pair absent from the
corpus, so a full scan with no match), i.e. the fixed per-merge price of launch + k_merge full
scan + completion + host flag, swept over grid caps and completion modes.

    python probe_merge.py [--config c2] [--iters 2000] [--layout types]
                          [--groups 64,128,256,512] [--direct-max 0,4096]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
os.environ.setdefault("SHREDWORD_LOG", "0")


def main():
    import bench
    from shredword.trainer import BPETrainer
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--layout", default="types")
    ap.add_argument("--groups", default="256")
    ap.add_argument("--direct-max", default="32")
    args = ap.parse_args()
    cfg = dict(bench.CONFIGS[args.config])
    path = bench.corpus_path(cfg, args.config)
    bench.ensure_corpus(cfg, path)
    t = BPETrainer(vocab_size=cfg["vocab"], unk_id=cfg["unk"], character_coverage=cfg["cov"], min_pair_freq=cfg["mpf"])
    t.set_option("layout", args.layout)
    t.load_corpus(path)
    from shredword.cbase import lib
    out = []
    for g in [int(x) for x in args.groups.split(",")]:
        for dm in [int(x) for x in args.direct_max.split(",")]:
            t.set_option("merge_groups", g)
            t.set_option("direct_max", dm)
            lib.shred_probe_merge(t.trainer, 255, 255, 50)  # warm up
            us = lib.shred_probe_merge(t.trainer, 255, 255, args.iters)
            out.append({"groups": g, "direct_max": dm, "us": round(us, 2)})
    st = t.stats()
    print(json.dumps({"lib": os.environ.get("SHREDWORD_LIB", "default"), "tiles": st["num_tiles"],
                      "tokens": st["live_tokens"], "layout": args.layout, "probe": out}))


if __name__ == "__main__":
    main()
