#!/usr/bin/env python3
"""CPU-baseline calibration (BASELINE.md "Calibration").

Times the CPU port (oracle/bpe_oracle.c — the `cpu_baseline` leg of bench.py) against the
REFERENCE itself (oracle/_ref/ref_driver over the zero-initialised reference build) on the same
corpus and config, both pinned to one core, and writes the ratio to
tests/golden/cpu_calibration.json.  The two must also produce identical .model/.vocab bytes.

Runs only in the build container (needs /root/reference for oracle/_ref):
    python tests/golden/calibrate_cpu.py
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import corpora  # noqa: E402

REPO = corpora.REPO
ORACLE = os.path.join(REPO, "oracle")

# name: (corpus recipe, (vocab, unk, coverage, min_pair_freq))
CASES = {
    "C1 10 MB ASCII (SURVEY.md §8 d2)": ({"bytes": 10_000_000, "seed": 1, "script": "ascii"}, (8192, 0, 0.995, 2000)),
    "100 MB ASCII, vocab 8192, min_pair_freq 2 (BASELINE.md calibration point)":
        ({"bytes": 100_000_000, "seed": 1, "script": "ascii"}, (8192, 0, 0.995, 2)),
}


def pin():
    os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})


def run(exe, corpus, cfg, out):
    vocab, unk, cov, mpf = cfg
    p = subprocess.run([exe, corpus, str(vocab), str(unk), repr(cov), str(mpf), out + ".model", out + ".vocab"],
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, preexec_fn=pin, check=True)
    line = [ln for ln in p.stderr.decode().splitlines() if ln.startswith("TIMING load=")][0]
    f = dict(kv.split("=") for kv in line.split()[1:])
    digest = hashlib.md5(open(out + ".model", "rb").read() + open(out + ".vocab", "rb").read()).hexdigest()
    return float(f["load"]), float(f["train"]), int(f["merges"]), digest


def main():
    subprocess.run(["make", "-s", "-C", ORACLE, "port", "ref"], check=True)
    port = os.path.join(ORACLE, "_build", "bpe_oracle")
    ref = os.path.join(ORACLE, "_ref", "ref_driver")
    cpu = next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")), "?")
    rows = []
    with tempfile.TemporaryDirectory() as tmp:
        for name, (recipe, cfg) in CASES.items():
            corpus = os.path.join(tmp, "corpus.txt")
            corpora.gen_synthetic(corpus, recipe["bytes"], recipe["seed"], recipe["script"])
            rl, rt, rm, rd = run(ref, corpus, cfg, os.path.join(tmp, "ref"))
            pl, pt, pm, pd = run(port, corpus, cfg, os.path.join(tmp, "port"))
            if (rm, rd) != (pm, pd):
                raise SystemExit(f"{name}: port output differs from the reference")
            rows.append({
                "case": name, "corpus": dict(recipe, md5=corpora.md5_file(corpus)),
                "config": dict(zip(("vocab_size", "unk_id", "character_coverage", "min_pair_freq"), cfg)),
                "merges": rm, "outputs_identical": True,
                "reference": {"load_s": rl, "train_s": rt, "merges_per_s": rm / rt if rt else None},
                "port": {"load_s": pl, "train_s": pt, "merges_per_s": pm / pt if pt else None},
                "train_time_ratio_port_over_reference": pt / rt if rt else None,
                "load_time_ratio_port_over_reference": pl / rl if rl else None,
            })
            print(json.dumps(rows[-1]), flush=True)
    out = {"what": "CPU port (oracle/bpe_oracle.c) vs the zero-init reference build, 1 pinned core each",
           "cpu": cpu, "rows": rows}
    with open(os.path.join(HERE, "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
