#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the survey/build container (needs /root/reference): it compiles the reference's
own BPE sources with zero-initialised malloc (oracle/Makefile target ``ref``)
and drives them through their C ABI (oracle/ref_driver.c) or their CLI (trainer.cpp), capturing

* ``model.bin``  — the reference .model bytes (bpe.cpp:419-427),
* ``vocab.txt``  — the reference .vocab bytes (bpe.cpp:416-418),
* ``trace.txt.gz`` — "M a b freq new_id" per [MERGE] line (bpe.cpp:260) and
  "B batch completed heap_size top_freq" per batch line (bpe.cpp:369),
* ``case.json``  — corpus recipe + md5, config, merge count, output md5s.

Corpora are not committed: tests rebuild them from the recipe and check the md5.
Usage: python tests/golden/make_golden.py [case-name ...]
"""
from __future__ import annotations

import gzip
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import corpora  # noqa: E402

REPO = corpora.REPO
ORACLE = os.path.join(REPO, "oracle")

# name: (corpus recipe, (vocab, unk, coverage, min_pair_freq), via)
CASES = {
    "c1_ascii10m_v8192": ({"kind": "synthetic", "bytes": 10_000_000, "seed": 1, "script": "ascii"},
                          (8192, 0, 0.995, 2000), "api"),
    "ascii1m_v3000_mpf2": ({"kind": "synthetic", "bytes": 1_000_000, "seed": 11, "script": "ascii"},
                           (3000, 0, 0.995, 2), "api"),
    "utf8_2m_v3000_cov9995": ({"kind": "synthetic", "bytes": 2_000_000, "seed": 12, "script": "utf8"},
                              (3000, 0, 0.9995, 2), "api"),
    "utf8_2m_v2000_mpf50": ({"kind": "synthetic", "bytes": 2_000_000, "seed": 13, "script": "utf8"},
                            (2000, 0, 0.995, 50), "api"),
    "ascii1m_unk7_cov09": ({"kind": "synthetic", "bytes": 1_000_000, "seed": 14, "script": "ascii"},
                           (1000, 7, 0.9, 3), "api"),
    "mixed2m_v4000": ({"kind": "synthetic", "bytes": 2_000_000, "seed": 15, "script": "mixed"},
                      (4000, 0, 0.9995, 2), "api"),
    "utf8_4m_v8192_mpf5": ({"kind": "synthetic", "bytes": 4_000_000, "seed": 16, "script": "utf8"},
                           (8192, 0, 0.995, 5), "api"),
    "ascii1m_unkm1_mpf2": ({"kind": "synthetic", "bytes": 1_000_000, "seed": 17, "script": "ascii"},
                           (2000, -1, 0.995, 2), "api"),
    "adv_unk0": ({"kind": "adversarial", "seed": 1}, (600, 0, 0.995, 2), "api"),
    "adv_unk3_cov09": ({"kind": "adversarial", "seed": 2}, (600, 3, 0.9, 2), "api"),
    "adv_cov05": ({"kind": "adversarial", "seed": 3}, (600, 0, 0.5, 3), "api"),
    "adv_unkm1": ({"kind": "adversarial", "seed": 4}, (600, -1, 0.995, 2), "api"),
    "small_v300": ({"kind": "small"}, (300, 0, 0.995, 2), "api"),
    "small_v50_zero": ({"kind": "small"}, (50, 0, 0.995, 1000), "api"),
    "small_v256_zero": ({"kind": "small"}, (256, 0, 0.995, 2), "api"),
    "small_cov0_mpf0": ({"kind": "small"}, (400, 0, 0.0, 0), "api"),
    # deep runs (VERDICT r1 "pin parity at the untested configs"): the C3 vocab/min_pair_freq to the
    # full 31,744 merges, and vocab 64000 / coverage 0.9995 on a mixed-script corpus with > 4,000
    # distinct code points, deep (ids past 32,767, all 63,744 merges) and at min_pair_freq 2000
    # (heap exhaustion).
    "utf8_24m_v32000_mpf2": ({"kind": "synthetic", "bytes": 24_000_000, "seed": 21, "script": "utf8"},
                             (32000, 0, 0.995, 2), "api"),
    "mixed24m_v64000_cov9995_mpf2": ({"kind": "synthetic", "bytes": 24_000_000, "seed": 22, "script": "mixed"},
                                     (64000, 0, 0.9995, 2), "api"),
    "mixed24m_v64000_cov9995": ({"kind": "synthetic", "bytes": 24_000_000, "seed": 22, "script": "mixed"},
                                (64000, 0, 0.9995, 2000), "api"),
    "cli_ascii10m": ({"kind": "synthetic", "bytes": 10_000_000, "seed": 1, "script": "ascii"},
                     (8192, -1, 0.9995, 2000), "cli"),
    "cli_utf8_2m_mpf20": ({"kind": "synthetic", "bytes": 2_000_000, "seed": 18, "script": "utf8"},
                          (3000, -1, 0.9995, 20), "cli"),
}

# Stateful call sequences through one trainer (missing 2), written to
# tests/golden/seq/<name>/.  Ops: ("load", recipe) bpe_load_corpus, ("init",) bpe_init,
# ("count",) bpe_count_bigrams, ("batch", k) bpe_merge_batch, ("train",) bpe_train, ("save",)
# bpe_save (save i writes model<i>.bin / vocab<i>.txt).  Every script keeps num_merges within
# target_vocab_size, where the reference's merge_ops (bpe.cpp:81, :261) and bpe_save stay in bounds.
_A = {"kind": "synthetic", "bytes": 1_000_000, "seed": 31, "script": "ascii"}
_B = {"kind": "synthetic", "bytes": 1_000_000, "seed": 32, "script": "utf8"}
_C = {"kind": "synthetic", "bytes": 1_000_000, "seed": 33, "script": "utf8"}
_D = {"kind": "synthetic", "bytes": 1_000_000, "seed": 34, "script": "ascii"}
SEQ_CASES = {
    # load twice: the last corpus wins (bpe.cpp:176-183)
    "seq_load_twice_train": ((400, 0, 0.995, 2), [("load", _A), ("load", _B), ("train",), ("save",)]),
    # a second corpus trained on top of the first: ids continue at 256 + num_merges, the .model
    # holds both trainings, the .vocab counts the second corpus
    "seq_train_load_train": ((420, 0, 0.995, 2), [("load", _A), ("train",), ("save",), ("load", _B), ("train",),
                                                  ("save",)]),
    # train twice: bpe_init re-counts the merged words (bpe.cpp:98-108), ids continue
    "seq_train_twice": ((450, 0, 0.995, 2), [("load", _C), ("train",), ("save",), ("train",), ("save",)]),
    "seq_train_twice_unk7": ((400, 7, 0.9, 3), [("load", _D), ("train",), ("train",), ("save",)]),
    # the first train exhausts the heap: the second finds nothing
    "seq_train_twice_exhaust": ((3000, 0, 0.995, 50),
                                [("load", {"kind": "synthetic", "bytes": 2_000_000, "seed": 13, "script": "utf8"}),
                                 ("train",), ("train",), ("save",)]),
    # bpe_init + bpe_merge_batch by hand, then bpe_save
    "seq_init_batches": ((3000, 0, 0.995, 2),
                         [("load", {"kind": "synthetic", "bytes": 1_000_000, "seed": 11, "script": "ascii"}),
                          ("init",), ("batch", 1), ("batch", 5), ("batch", 10), ("batch", 0), ("batch", 100),
                          ("save",)]),
    # merge_batch, then train (re-init over the merged words)
    "seq_init_batch_train": ((450, 0, 0.995, 2), [("load", _C), ("init",), ("batch", 50), ("save",), ("train",),
                                                  ("save",)]),
    # bpe_count_bigrams without bpe_init right after a load (a fresh pair map, an empty heap)
    "seq_count_batch": ((600, 0, 0.995, 2), [("load", {"kind": "adversarial", "seed": 1}), ("count",), ("batch", 40),
                                             ("save",)]),
    "seq_save_untrained": ((300, 0, 0.995, 2), [("load", {"kind": "small"}), ("save",)]),
    # vocab below 256: train() does nothing, merge_batch still merges (no target check)
    "seq_batch_vocab_small": ((50, 0, 0.995, 2), [("load", {"kind": "small"}), ("train",), ("init",), ("batch", 20),
                                                  ("save",)]),
    # --- the pair map is not the corpus's exact count: the reference's recompute_freq rescan
    #     (bpe.cpp:52-65, :251-257) decides
    # count after init: every count doubled, every pair pushed again (bpe.cpp:207-211, :218-227)
    "seq_count_twice": ((800, 0, 0.995, 2), [("load", _C), ("init",), ("count",), ("batch", 60), ("save",)]),
    # count after a training, without init: the merged words are added to the trained pair map
    "seq_train_count_batch": ((500, 0, 0.995, 2), [("load", _A), ("train",), ("count",), ("batch", 30), ("save",)]),
    # merge_batch after a reload without a count: the heap still holds the first corpus's entries,
    # the pair map is fresh (bpe.cpp:183)
    "seq_reload_batch": ((500, 0, 0.995, 2), [("load", _A), ("train",), ("load", _B), ("batch", 30), ("save",)]),
    # a reload and a count on top of the first corpus's heap
    "seq_reload_count_batch": ((500, 0, 0.995, 2), [("load", _A), ("init",), ("batch", 20), ("load", _B), ("count",),
                                                    ("batch", 20), ("save",)]),
    "seq_batch_before_count": ((400, 0, 0.995, 2), [("load", _A), ("batch", 5), ("count",), ("batch", 10),
                                                    ("save",)]),
}

MERGE_RE = re.compile(rb"^\[MERGE\]\t Merging \((-?\d+),(-?\d+)\) freq=(\d+) -> new_id=(-?\d+)")
BATCH_RE = re.compile(rb"^\[INFO\]\t Processing batch of (-?\d+) merges \(completed: (-?\d+)/-?\d+, "
                      rb"heap size: (\d+), top freq: (\d+)\)")
SCRIPT_RE = re.compile(rb"^\[SCRIPT\]\t (\w+) (-?\d+)")


def build_corpus(recipe: dict, path: str) -> None:
    kind = recipe["kind"]
    if kind == "synthetic":
        corpora.gen_synthetic(path, recipe["bytes"], recipe["seed"], recipe["script"])
    elif kind == "adversarial":
        corpora.write_adversarial(path, recipe["seed"])
    elif kind == "small":
        corpora.write_small_corpus(path)
    else:
        raise ValueError(kind)


def parse_trace(stdout: bytes) -> str:
    out = []
    for line in stdout.splitlines():
        m = MERGE_RE.match(line)
        if m:
            out.append("M %s %s %s %s" % tuple(g.decode() for g in m.groups()))
            continue
        m = BATCH_RE.match(line)
        if m:
            out.append("B %s %s %s %s" % tuple(g.decode() for g in m.groups()))
            continue
        m = SCRIPT_RE.match(line)
        if m:
            out.append("S %s %s" % tuple(g.decode() for g in m.groups()))
    return "\n".join(out) + ("\n" if out else "")


def run_case(name: str, tmp: str) -> None:
    recipe, (vocab, unk, cov, mpf), via = CASES[name]
    corpus = os.path.join(tmp, name + ".txt")
    build_corpus(recipe, corpus)
    model = os.path.join(tmp, name + ".model")
    vocabf = os.path.join(tmp, name + ".vocab")
    if via == "api":
        cmd = [os.path.join(ORACLE, "_ref", "ref_driver"), corpus, str(vocab), str(unk), repr(cov),
               str(mpf), model, vocabf]
    else:
        # the CLI aborts after saving (unk_id=-1, bpe.cpp:413): line-buffer stdout to keep the trace
        cmd = ["stdbuf", "-oL", os.path.join(ORACLE, "_ref", "trainer_ref"), f"input={corpus}", "model_type=bpe",
               f"output_model={model}", f"output_vocab={vocabf}", f"vocab_size={vocab}",
               f"character_coverage={cov}", f"min_pair_freq={mpf}"]
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    # unk_id < 0 makes the reference write freq[-1] (bpe.cpp:413) and abort in free() after
    # both files are closed; any other failure is fatal.
    if via == "api" and proc.returncode != 0 and unk >= 0:
        raise RuntimeError(f"{name}: reference failed rc={proc.returncode}: {proc.stderr[-2000:]!r}")
    if not (os.path.exists(model) and os.path.exists(vocabf)):
        raise RuntimeError(f"{name}: reference produced no files (rc={proc.returncode})")
    d = os.path.join(HERE, name)
    os.makedirs(d, exist_ok=True)
    shutil.copyfile(model, os.path.join(d, "model.bin"))
    shutil.copyfile(vocabf, os.path.join(d, "vocab.txt"))
    trace = parse_trace(proc.stdout)
    with gzip.open(os.path.join(d, "trace.txt.gz"), "wt") as f:
        f.write(trace)
    merges = os.path.getsize(model) // 12
    case = {
        "name": name,
        "corpus": dict(recipe, md5=corpora.md5_file(corpus), size=os.path.getsize(corpus)),
        "config": {"vocab_size": vocab, "unk_id": unk, "character_coverage": cov, "min_pair_freq": mpf},
        "via": via,
        "reference_returncode": proc.returncode,
        "merges": merges,
        "model_md5": corpora.md5_file(model),
        "vocab_md5": corpora.md5_file(vocabf),
        "generator": "tests/golden/make_golden.py (zero-init reference, oracle/Makefile ref)",
    }
    with open(os.path.join(d, "case.json"), "w") as f:
        json.dump(case, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"{name}: merges={merges} rc={proc.returncode}")


def seq_argv(ops, corpus_of, tmp, name):
    """The script's ops as ref_driver / bpe_oracle --script arguments (saves numbered from 0)."""
    argv, nsave = [], 0
    for op in ops:
        if op[0] == "load":
            argv.append("load=" + corpus_of(op[1]))
        elif op[0] == "batch":
            argv.append(f"batch={op[1]}")
        elif op[0] == "save":
            argv.append("save=%s,%s" % (os.path.join(tmp, f"{name}.model{nsave}"),
                                        os.path.join(tmp, f"{name}.vocab{nsave}")))
            nsave += 1
        else:
            argv.append(op[0])
    return argv, nsave


def run_seq_case(name: str, tmp: str) -> None:
    (vocab, unk, cov, mpf), ops = SEQ_CASES[name]
    corpora_made = {}

    def corpus_of(recipe):
        key = json.dumps(recipe, sort_keys=True)
        if key not in corpora_made:
            path = os.path.join(tmp, f"{name}.corpus{len(corpora_made)}.txt")
            build_corpus(recipe, path)
            corpora_made[key] = path
        return corpora_made[key]

    argv, nsave = seq_argv(ops, corpus_of, tmp, name)
    cmd = [os.path.join(ORACLE, "_ref", "ref_driver"), "--script", str(vocab), str(unk), repr(cov), str(mpf)] + argv
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    if proc.returncode != 0:
        raise RuntimeError(f"{name}: reference failed rc={proc.returncode}: {proc.stderr[-2000:]!r}")
    d = os.path.join(HERE, "seq", name)
    os.makedirs(d, exist_ok=True)
    saves = []
    for i in range(nsave):
        model, vocabf = (os.path.join(tmp, f"{name}.{k}{i}") for k in ("model", "vocab"))
        shutil.copyfile(model, os.path.join(d, f"model{i}.bin"))
        shutil.copyfile(vocabf, os.path.join(d, f"vocab{i}.txt"))
        saves.append({"merges": os.path.getsize(model) // 12, "model_md5": corpora.md5_file(model),
                      "vocab_md5": corpora.md5_file(vocabf)})
    trace = parse_trace(proc.stdout)
    with gzip.open(os.path.join(d, "trace.txt.gz"), "wt") as f:
        f.write(trace)
    script = []
    for op in ops:
        if op[0] == "load":
            path = corpus_of(op[1])
            script.append(["load", dict(op[1], md5=corpora.md5_file(path), size=os.path.getsize(path))])
        else:
            script.append(list(op))
    case = {
        "name": name,
        "config": {"vocab_size": vocab, "unk_id": unk, "character_coverage": cov, "min_pair_freq": mpf},
        "script": script,
        "returns": [line.split()[1:] for line in trace.splitlines() if line.startswith("S ")],
        "saves": saves,
        "generator": "tests/golden/make_golden.py (zero-init reference, oracle/ref_driver.c --script)",
    }
    with open(os.path.join(d, "case.json"), "w") as f:
        json.dump(case, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"{name}: saves={[s['merges'] for s in saves]} returns={case['returns']}")


def main() -> None:
    subprocess.run(["make", "-C", ORACLE, "ref"], check=True, stdout=subprocess.DEVNULL)
    names = sys.argv[1:] or list(CASES) + list(SEQ_CASES)
    with tempfile.TemporaryDirectory() as tmp:
        for n in names:
            if n in SEQ_CASES:
                run_seq_case(n, tmp)
            else:
                run_case(n, tmp)


if __name__ == "__main__":
    main()
