#!/usr/bin/env python3
"""Diagnostic: round-trip cost of a device merge that changes nothing (a pair absent from the
corpus), i.e. the fixed per-merge price of launch + k_merge full scan + fused collect + flag.

    python probe_merge.py [--config c2] [--iters 2000] [--layout types]
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
    args = ap.parse_args()
    cfg = dict(bench.CONFIGS[args.config])
    path = bench.corpus_path(cfg, args.config)
    bench.ensure_corpus(cfg, path)
    t = BPETrainer(vocab_size=cfg["vocab"], unk_id=cfg["unk"], character_coverage=cfg["cov"], min_pair_freq=cfg["mpf"])
    t.set_option("layout", args.layout)
    t.load_corpus(path)
    from shredword.cbase import lib
    lib.shred_probe_merge(t.trainer, 255, 255, 50)  # warm up
    us = lib.shred_probe_merge(t.trainer, 255, 255, args.iters)
    st = t.stats()
    print(json.dumps({"probe_us_per_merge": us, "tiles": st["num_tiles"], "tokens": st["live_tokens"],
                      "layout": args.layout}))


if __name__ == "__main__":
    main()
