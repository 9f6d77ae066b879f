"""Times load_corpus of a bench config's corpus: the whole-file device count and the k-range
sharded load (SHREDWORD_LOAD_SIM_SHARDS=k: the per-rank step of a k-GPU load, ranges counted in
turn), with SHREDWORD_LOAD_REPORT on.

    python shredword-trainer_amd/tools/load_probe.py [--config c4] [--bytes N] [--shards 0 2 8]
"""
import argparse
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--bytes", type=int, default=10_000_000_000)
    ap.add_argument("--shards", type=int, nargs="+", default=[0, 2, 8])
    args = ap.parse_args()
    import bench
    cfg = dict(bench.CONFIGS[args.config])
    cfg["bytes"] = args.bytes
    path = bench.corpus_path(cfg, args.config)
    bench.ensure_corpus(cfg, path)
    for k in args.shards:
        code = ("import sys, time; sys.path.insert(0, %r)\n"
                "from shredword.trainer import BPETrainer\n"
                "t = BPETrainer(vocab_size=%d, min_pair_freq=%d); t.set_option('log', 0)\n"
                "t0 = time.time(); t.load_corpus(%r); dt = time.time() - t0\n"
                "st = t.stats(); print('shards %d: load %%.2f s, words %%d, gpu %%d' %% (dt, st['num_words'], st['load_on_gpu']), flush=True)\n"
                % (os.path.dirname(HERE), cfg["vocab"], cfg["mpf"], path, k))
        env = dict(os.environ, SHREDWORD_LOAD_REPORT="1", SHREDWORD_LOAD_SIM_SHARDS=str(k))
        subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=900)


if __name__ == "__main__":
    main()
