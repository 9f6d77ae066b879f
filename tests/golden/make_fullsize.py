#!/usr/bin/env python3
"""Full-size parity fixtures for the bench configs.

The reference itself cannot train a 1-10 GB corpus here: its word counter is a fixed 4096-bucket
chained map (hash.cpp:29-53), O(tokens x W / 4096) — days at C3.  These fixtures therefore come
from the CPU restatement ``oracle/bpe_oracle`` run to completion, which is pinned to the reference
by every golden in tests/golden/*/ (tests/test_oracle.py), including the reference's own deep
31,744- and 63,744-merge runs.  Per config this writes ``tests/golden/fullsize/<name>/``:

* ``case.json``     — generator recipe, corpus md5 + unique-byte count + W + S (SURVEY.md §8 d2
                      "record W, S, corpus md5 and unique-byte count per config"), the trainer
                      config, merges, .model/.vocab md5s, oracle load/train seconds;
* ``model.bin.gz``  — the oracle's .model (so a GPU mismatch names its first differing merge);
* ``trace.txt.gz``  — "M a b freq new_id" per merge and "B batch completed heap top" per batch.

Corpora are regenerated from the recipe (bin/gen_corpus) and their md5 is checked.  Usage:
    python tests/golden/make_fullsize.py c2 [c3 ...]       (minutes for c2, ~1 h for c3)

The two largest configs (C4 80 GB, C5 100 GB; VERDICT r04 missing 1) never touch the disk: the
generator streams through ``tee`` (md5sum on the side) into the oracle's streaming reader
(``bpe_oracle /dev/stdin``, read once in order, fgets semantics unchanged), and the oracle's two
O(S) scans per merge run on ``--threads`` host threads (same output: tests/test_oracle.py).
    python tests/golden/make_fullsize.py --threads 4 c5
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import corpora  # noqa: E402

REPO = corpora.REPO
ORACLE_EXE = os.path.join(REPO, "oracle", "_build", "bpe_oracle")
OUT = os.path.join(HERE, "fullsize")

# name: (bytes, seed, script, (vocab, unk, coverage, min_pair_freq)) — bench.py CONFIGS
CASES = {
    "c2": (1_000_000_000, 2, "utf8", (8192, 0, 0.995, 2000)),
    "c3": (10_000_000_000, 3, "utf8", (32000, 0, 0.995, 2)),
    # C5's parameters (vocab 64000, coverage 0.9995, mixed script, seed 5, min_pair_freq 2000 =
    # the Python default) at 10 GB: the 100 GB corpus is out of the oracle's reach (hours per GB
    # of merges), this one pins the 64k-vocab / high-cardinality path at a size past C3
    "c5_10g": (10_000_000_000, 5, "mixed", (64000, 0, 0.9995, 2000)),
    # C4's parameters (vocab 32000, min_pair_freq 2000, seed 4) on one 10 GB shard-sized corpus:
    # the GPU test loads it as 8 byte ranges (the sharded load of C4) and must match this run
    "c4_10g": (10_000_000_000, 4, "utf8", (32000, 0, 0.995, 2000)),
    # the full-size C4 and C5 corpora of bench.py CONFIGS, streamed (no file)
    "c4": (80_000_000_000, 4, "utf8", (32000, 0, 0.995, 2000)),
    "c5": (100_000_000_000, 5, "mixed", (64000, 0, 0.9995, 2000)),
}
STREAM_FROM = 20_000_000_000   # corpora this large are streamed, not written
GEN = os.path.join(REPO, "shredword-trainer_amd", "bin", "gen_corpus")


def corpus_file(name: str, nbytes: int, seed: int, script: str) -> str:
    d = os.environ.get("SHREDWORD_BENCH_DIR", os.path.join(os.environ.get("TMPDIR", "/tmp"), "shredword_bench"))
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"{name}_{script}_{nbytes}_s{seed}.txt")
    if not (os.path.exists(path) and os.path.getsize(path) == nbytes):
        corpora.gen_synthetic(path, nbytes, seed, script)
    return path


def corpus_stats(path: str):
    """md5 and the number of distinct byte values."""
    import numpy as np
    h = hashlib.md5()
    seen = np.zeros(256, dtype=bool)
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 26), b""):
            h.update(chunk)
            seen |= np.bincount(np.frombuffer(chunk, dtype=np.uint8), minlength=256) > 0
    return h.hexdigest(), int(seen.sum())


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def md5_bytes(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


def run_streamed(name, nbytes, seed, script, oracle_args, tmp, threads, gen_threads):
    """gen_corpus -> tee (md5sum) -> bpe_oracle /dev/stdin.  Returns (stderr text, corpus md5)."""
    md5_path = tmp + ".md5"
    if os.path.exists(md5_path):
        os.unlink(md5_path)
    err_path = tmp + ".err"
    cmd = (f"set -o pipefail; {GEN} --bytes {nbytes} --seed {seed} --script {script} --out /dev/stdout "
           f"--threads {gen_threads} | tee >(md5sum > {md5_path}) | {ORACLE_EXE} /dev/stdin "
           + " ".join(oracle_args) + f" --threads {threads} 2> {err_path}")
    subprocess.run(["bash", "-c", cmd], check=True)
    for _ in range(600):   # the md5sum process substitution may end just after the pipeline
        if os.path.exists(md5_path) and os.path.getsize(md5_path) >= 32:
            break
        time.sleep(1)
    md5 = open(md5_path).read().split()[0]
    err = open(err_path).read()
    os.unlink(md5_path)
    return err, md5


def make(name: str, threads: int = 1, gen_threads: int = 3) -> None:
    nbytes, seed, script, (vocab, unk, cov, mpf) = CASES[name]
    d = os.path.join(OUT, name)
    os.makedirs(d, exist_ok=True)
    tmp = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"fullsize_{name}")
    oracle_args = [str(vocab), str(unk), repr(cov), str(mpf), tmp + ".model", tmp + ".vocab",
                   "--trace", tmp + ".trace", "--progress", "256"]
    t0 = time.time()
    streamed = nbytes >= STREAM_FROM
    if streamed:
        err, md5 = run_streamed(name, nbytes, seed, script, oracle_args, tmp, threads, gen_threads)
        nbyte = None
    else:
        path = corpus_file(name, nbytes, seed, script)
        md5, nbyte = corpus_stats(path)
        proc = subprocess.run([ORACLE_EXE, path] + oracle_args + ["--threads", str(threads)],
                              stderr=subprocess.PIPE, check=True)
        err = proc.stderr.decode()
    wall = time.time() - t0
    fields = dict(kv.split("=") for kv in err.split("TIMING", 1)[1].split())
    if nbyte is None:
        nbyte = int(fields["unique_bytes"])
    assert int(fields["bytes"]) == nbytes, (fields["bytes"], nbytes)
    # measured cost curve: cumulative train seconds after every 256 merges (bench.py extrapolates
    # its capped CPU baseline along this curve)
    curve = [[int(l.split()[1]), float(l.split()[2])] for l in err.splitlines() if l.startswith("PROGRESS ")]
    model = open(tmp + ".model", "rb").read()
    vocabb = open(tmp + ".vocab", "rb").read()
    with gzip.GzipFile(os.path.join(d, "model.bin.gz"), "wb", mtime=0) as f:
        f.write(model)
    with open(tmp + ".trace", "rb") as src, gzip.GzipFile(os.path.join(d, "trace.txt.gz"), "wb", mtime=0) as f:
        f.write(src.read())
    case = {
        "recipe": {"kind": "synthetic", "bytes": nbytes, "seed": seed, "script": script},
        "corpus_md5": md5, "unique_bytes": nbyte,
        "distinct_words": int(fields["words"]), "symbols": int(fields["symbols"]),
        "config": {"vocab_size": vocab, "unk_id": unk, "character_coverage": cov, "min_pair_freq": mpf},
        "merges": int(fields["merges"]),
        "model_md5": md5_bytes(model), "vocab_md5": md5_bytes(vocabb), "vocab_bytes": len(vocabb),
        "oracle": {"exe": "oracle/_build/bpe_oracle", "load_s": float(fields["load"]),
                   "train_s": float(fields["train"]), "wall_s": wall, "threads": threads,
                   "streamed": streamed, "cpu": cpu_model(), "progress": curve},
    }
    with open(os.path.join(d, "case.json"), "w") as f:
        json.dump(case, f, indent=1)
        f.write("\n")
    for ext in (".model", ".vocab", ".trace"):
        os.unlink(tmp + ext)
    print(name, json.dumps(case), flush=True)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="*", default=["c2"])
    ap.add_argument("--threads", type=int, default=1, help="oracle scan threads (same output)")
    ap.add_argument("--gen-threads", type=int, default=3)
    a = ap.parse_args()
    for n in a.names:
        make(n, a.threads, a.gen_threads)
