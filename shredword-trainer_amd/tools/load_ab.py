"""load_corpus of one bench config's corpus, repeated in ONE process under several environment
variants, interleaved (A B C A B C ...), so the box's drift and the page cache treat every variant
alike; prints one JSON summary (per variant: every load's seconds, min / median).  The loader reads
its SHREDWORD_LOAD_* switches at each load, so the variants need no new process.

    python shredword-trainer_amd/tools/load_ab.py --config c3 --reps 4 \\
        --variant base= --variant seg512=SHREDWORD_LOAD_SEGMENT_MB=512,SHREDWORD_LOAD_BUFS=8
"""
import argparse
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variant", action="append", required=True)
    args = ap.parse_args()
    import bench
    from shredword.trainer import BPETrainer
    from shredword.cbase import lib
    cfg = dict(bench.CONFIGS[args.config])
    path = bench.corpus_path(cfg, args.config)
    bench.ensure_corpus(cfg, path)
    lib.shred_device_count()  # the HIP runtime comes up outside the timed loads
    variants = []
    for v in args.variant:
        name, _, spec = v.partition("=")
        env = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
        variants.append((name, env))
    keys = {k for _, env in variants for k in env}
    res = {name: [] for name, _ in variants}
    words = {}
    for r in range(args.reps):
        for name, env in variants:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            t = BPETrainer(vocab_size=cfg["vocab"], min_pair_freq=cfg["mpf"])
            t.set_option("log", 0)
            t0 = time.time()
            t.load_corpus(path)
            dt = time.time() - t0
            st = t.stats()
            words.setdefault(name, set()).add((st["num_words"], st["num_symbols"]))
            t.destroy()
            res[name].append(dt)
            print(f"[load_ab] {name} rep {r}: {dt:.3f} s", file=sys.stderr, flush=True)
    print(json.dumps({"config": args.config, "reps": args.reps,
                      "variants": {n: {"env": env, "loads_s": res[n], "min": min(res[n]),
                                       "median": statistics.median(res[n]),
                                       "words_symbols": sorted(words[n])} for n, env in variants}}, indent=1))


if __name__ == "__main__":
    main()
