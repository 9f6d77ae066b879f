"""load_corpus of a bench config's corpus once, in this process (for rocprofv3 --pmc passes of the
device word count: no child processes).  Prints the load time and the table size.

    python shredword-trainer_amd/tools/load_once.py [--config c3] [--bytes N]
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--bytes", type=int, default=0)
    args = ap.parse_args()
    import bench
    from shredword.trainer import BPETrainer
    cfg = dict(bench.CONFIGS[args.config])
    if args.bytes:
        cfg["bytes"] = args.bytes
    path = bench.corpus_path(cfg, args.config)
    bench.ensure_corpus(cfg, path)
    t = BPETrainer(vocab_size=cfg["vocab"], min_pair_freq=cfg["mpf"])
    t.set_option("log", 0)
    from shredword.cbase import lib
    th = time.time()  # the HIP runtime comes up once per process, outside the load
    lib.shred_device_count()
    print(f"{args.config}: HIP runtime init {time.time() - th:.2f} s", flush=True)
    t0 = time.time()
    t.load_corpus(path)
    st = t.stats()
    print(f"{args.config}: load {time.time() - t0:.2f} s, words {st['num_words']}, symbols {st['num_symbols']}, "
          f"gpu {st['load_on_gpu']}", flush=True)
    t.destroy()


if __name__ == "__main__":
    main()
