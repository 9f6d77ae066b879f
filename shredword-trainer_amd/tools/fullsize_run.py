"""One full-size BASELINE config on one GPU, end to end (SURVEY.md §8 d2 records + the
size-independent parity invariants of tests/test_gpu_api.py::test_full_size_invariants):

  generate the corpus (bin/gen_corpus, the bench's deterministic generator) into /dev/shm when it
  has room, else $TMPDIR; load_corpus (C4: the 8 byte ranges of the sharded load counted in turn
  and merged, SHREDWORD_LOAD_SIM_SHARDS=8, as each of 8 ranks would); one warm train(), `--steps`
  timed train() (reset between, load outside); then one train() with the K5 device argmax check
  every `--verify` merges and the merge trace, saved and checked:
    * merges > 0, ids 256.. in order, operands created before their merge;
    * byte conservation: Σ len(token) x freq over the .vocab = the corpus's non-delimiter bytes;
    * merge frequencies non-increasing and >= min_pair_freq;
    * every K5 check passed (device recount max = the host heap pick = its own count);
  and the d2 records: corpus md5, unique bytes, W (distinct words), S (symbols), occurrences.
Prints progress lines (one per phase) and writes one JSON.

    python shredword-trainer_amd/tools/fullsize_run.py --config c5 --out gpurun_out/c5_full.json
"""
import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, REPO)


def say(msg):
    print(f"[fullsize {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def stream_stats(path, chunk=1 << 30):
    """md5, byte histogram -> unique bytes, non-delimiter bytes ([\\t\\r\\n ] are the delimiters)."""
    import numpy as np
    md5 = hashlib.md5()
    hist = np.zeros(256, dtype=np.int64)
    done = 0
    size = os.path.getsize(path)
    with open(path, "rb") as f:
        while True:
            buf = f.read(chunk)
            if not buf:
                break
            md5.update(buf)
            hist += np.bincount(np.frombuffer(buf, dtype=np.uint8), minlength=256)
            done += len(buf)
            if done % (10 << 30) < chunk:
                say(f"stats {done / 1e9:.0f} / {size / 1e9:.0f} GB")
    word_bytes = int(hist.sum() - hist[32] - hist[10] - hist[9] - hist[13])
    return md5.hexdigest(), int((hist > 0).sum()), word_bytes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--bytes", type=int, default=0)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--verify", type=int, default=500)
    ap.add_argument("--dir", default="")
    ap.add_argument("--out", default="gpurun_out/fullsize.json")
    ap.add_argument("--keep", action="store_true", help="keep the corpus file")
    ap.add_argument("--known", default="", help="a committed record of the same corpus (generator, seed, size): "
                    "its md5, unique bytes and word bytes are used instead of a streaming pass")
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    import bench
    from shredword.trainer import BPETrainer

    cfg = dict(bench.CONFIGS[args.config])
    if args.bytes:
        cfg["bytes"] = args.bytes
    need = int(cfg["bytes"] * 1.02) + (2 << 30)
    d = args.dir
    if not d:
        for cand in ("/dev/shm", os.environ.get("TMPDIR", "/tmp")):
            try:
                if shutil.disk_usage(cand).free >= need:
                    d = os.path.join(cand, "shredword_full")
                    break
            except OSError:
                continue
    if not d:
        raise SystemExit(f"no filesystem with {need / 1e9:.0f} GB free for the {args.config} corpus")
    os.environ["SHREDWORD_BENCH_DIR"] = d
    path = bench.corpus_path(cfg, args.config)
    say(f"{args.config}: {cfg['bytes'] / 1e9:.0f} GB corpus in {d}")
    import threading
    done = threading.Event()

    def heartbeat():  # generation takes minutes: a line every 30 s keeps the run visibly alive
        while not done.wait(30):
            try:
                say(f"generating: {os.path.getsize(path + '.part') / 1e9:.1f} GB written")
            except OSError:
                say("generating")
    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    try:
        gen_s = bench.ensure_corpus(cfg, path, cpus=bench.gpu_numa_cpus(0))  # pages on the GPU's node
    finally:
        done.set()
        hb.join()
    say(f"generated in {gen_s:.0f} s")
    env_shards = cfg.get("shards")
    if env_shards:
        os.environ["SHREDWORD_LOAD_SIM_SHARDS"] = str(env_shards)
    res = {"config": args.config, "workload": cfg["desc"], "corpus_bytes": cfg["bytes"], "seed": cfg["seed"],
           "script": cfg["script"], "vocab_size": cfg["vocab"], "min_pair_freq": cfg["mpf"],
           "character_coverage": cfg["cov"], "unk_id": cfg["unk"], "corpus_dir": d, "corpus_gen_s": gen_s,
           "sharded_load_ranges": env_shards}
    t = BPETrainer(vocab_size=cfg["vocab"], unk_id=cfg["unk"], character_coverage=cfg["cov"], min_pair_freq=cfg["mpf"])
    t.set_option("log", 0)
    from shredword.cbase import lib
    th = time.time()  # the HIP runtime comes up once per process, outside the load
    lib.shred_device_count()
    res["hip_init_s"] = time.time() - th
    t0 = time.time()
    t.load_corpus(path)
    res["load_s"] = time.time() - t0
    st = t.stats()
    res.update({"distinct_words": st["num_words"], "symbols": st["num_symbols"], "occurrences": st["num_occurrences"],
                "tiles": st["num_tiles"], "load_on_gpu": st.get("load_on_gpu")})
    say(f"loaded in {res['load_s']:.1f} s: W={st['num_words']} S={st['num_symbols']} occurrences={st['num_occurrences']}")
    n0 = t._train(t.trainer)
    say(f"warm train: {n0} merges")
    times = []
    for _ in range(args.steps):
        t.reset()
        torch.cuda.synchronize()
        s0 = time.perf_counter()
        n = t._train(t.trainer)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - s0)
        if n != n0:
            raise SystemExit(f"train() gave {n} merges after {n0}")
    res["merges"] = n0
    res["train_s"] = times
    res["merges_per_s"] = n0 / (sum(times) / len(times))
    say(f"timed: {res['merges_per_s']:.0f} merges/s ({[round(x, 3) for x in times]} s)")
    t.reset()
    tmpd = os.environ.get("TMPDIR", "/tmp")
    trace, model, vocab = (os.path.join(tmpd, f"full_{args.config}.{e}") for e in ("trace", "model", "vocab"))
    t.set_option("trace", trace)
    t.set_option("verify_argmax", args.verify)
    n = t._train(t.trainer)
    t.set_option("trace", "")
    t._save(t.trainer, model.encode(), vocab.encode())
    st = t.stats()
    t.destroy()
    say(f"verified train: {n} merges, K5 checks {st['verify_checks']} failures {st['verify_failures']}")
    mb, vb = open(model, "rb").read(), open(vocab, "rb").read()
    res["model_md5"] = hashlib.md5(mb).hexdigest()
    res["vocab_md5"] = hashlib.md5(vb).hexdigest()
    ops = np.frombuffer(mb, dtype="<i4").reshape(-1, 3)
    T = 256 + n
    spell = [bytes([i]) if i else b"" for i in range(256)]
    for a, b, _x in ops:
        spell.append(spell[a] + spell[b])
    toks, pos = [], 0
    for tok in spell:
        pos += len(tok)
        end = vb.index(b"\n", pos + 1)
        toks.append((tok, int(vb[pos + 1:end])))
        pos = end + 1
    freqs = [int(ln.split()[3]) for ln in open(trace) if ln.startswith("M ")]
    known = json.load(open(args.known)) if args.known else None
    if known and all(known.get(k) == res[k] for k in ("corpus_bytes", "seed", "script")):
        md5, uniq, word_bytes = known["corpus_md5"], known["unique_bytes"], known["word_bytes"]
        res["corpus_stats_from"] = args.known
    else:
        md5, uniq, word_bytes = stream_stats(path)
    res.update({"corpus_md5": md5, "unique_bytes": uniq, "word_bytes": word_bytes})
    conserved = sum(len(tok) * f for tok, f in toks[1:]) + toks[0][1]
    checks = {
        "merges_equal_across_trains": n == n0,
        "merges_positive_within_target": 0 < n <= cfg["vocab"] - 256,
        "ids_in_order": bool((ops[:, 2] == np.arange(256, T)).all()),
        "operands_before_merge": bool((ops[:, :2] < ops[:, 2:3]).all()),
        "vocab_lines": len(toks) == T and pos == len(vb),
        "byte_conservation": conserved == word_bytes,
        "freqs_non_increasing": all(x >= y for x, y in zip(freqs, freqs[1:])) and len(freqs) == n,
        "freqs_at_least_min_pair_freq": bool(freqs) and freqs[-1] >= cfg["mpf"],
        "k5_checks": st["verify_checks"], "k5_failures": st["verify_failures"],
        "k5_all_passed": (st["verify_checks"] >= n // args.verify if args.verify > 0 else True)
                         and st["verify_failures"] == 0,
    }
    if known and "corpus_stats_from" in res:  # another run of the same corpus and config: the same bytes
        checks["model_vocab_md5_equal_known_run"] = (res["model_md5"], res["vocab_md5"]) == (known["model_md5"],
                                                                                            known["vocab_md5"])
    res["invariants"] = checks
    res["all_invariants_hold"] = all(v for k, v in checks.items() if not k.startswith("k5_") or k == "k5_all_passed")
    res["last_merge_freq"] = freqs[-1] if freqs else None
    json.dump(res, open(args.out, "w"), indent=1)
    say(f"invariants {'hold' if res['all_invariants_hold'] else 'FAIL'}: {checks}")
    if not args.keep:
        os.remove(path)
    print(json.dumps(res), flush=True)
    return 0 if res["all_invariants_hold"] else 1


if __name__ == "__main__":
    sys.exit(main())
