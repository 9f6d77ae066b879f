"""k_resident phase stamps on a bench corpus: trains to a few target vocab sizes with
SHREDWORD_RESIDENT_STAMPS=1 / SHREDWORD_RESIDENT_REPORT=1 set, so each launch's report (stderr)
gives the device phases of those merges (all regions published / prefix / loaded / combined / flag)
and the host's post -> flag.

    python shredword-trainer_amd/tools/resident_stamps.py [--config c3] [--vocab 456 1373]
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, REPO)
os.environ.setdefault("SHREDWORD_RESIDENT_STAMPS", "1")
os.environ.setdefault("SHREDWORD_RESIDENT_REPORT", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--vocab", type=int, nargs="+", default=[456, 1373])
    ap.add_argument("--index", type=int, default=0, help="0: resident only (no indexed loop, no switch)")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    import bench
    from shredword.trainer import BPETrainer
    cfg = dict(bench.CONFIGS[args.config])
    path = bench.corpus_path(cfg, args.config)
    bench.ensure_corpus(cfg, path)
    for v in args.vocab:
        t = BPETrainer(vocab_size=v, unk_id=cfg["unk"], character_coverage=cfg["cov"], min_pair_freq=cfg["mpf"])
        t.set_option("log", 0)
        t.set_option("index", args.index)
        t.load_corpus(path)
        t._train(t.trainer)  # warm
        t.reset()
        t0 = time.time()
        n = t._train(t.trainer)
        dt = time.time() - t0
        print(f"vocab {v}: {n} merges in {dt * 1e3:.1f} ms = {1e6 * dt / max(1, n):.1f} us per merge", flush=True)
        print(f"vocab {v}: stats {t.stats()}", file=sys.stderr, flush=True)
        t.destroy()


if __name__ == "__main__":
    main()
