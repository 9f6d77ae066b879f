#!/usr/bin/env python3
"""K1 (initial pair count) alone at HBM scale: bench.pair_count_leg on a config's corpus in the
stream layout, printed as one JSON line.

    python k1_bench.py [--config c2] [--reps 10] [--bytes N]
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--bytes", type=int, default=0)
    ap.add_argument("--layout", default="stream")
    args = ap.parse_args()
    cfg = dict(bench.CONFIGS[args.config], name=args.config)
    if args.bytes:
        cfg["bytes"] = args.bytes
    path = bench.corpus_path(cfg, args.config)
    bench.ensure_corpus(cfg, path)
    print(json.dumps(bench.pair_count_leg(cfg, path, args.reps, layout=args.layout)), flush=True)


if __name__ == "__main__":
    main()
