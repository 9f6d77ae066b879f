"""One full-size config, loaded once, trained under several option settings (set_option key=value
pairs; "-" = the defaults), two timed train()s each, the files' md5 checked equal for every
setting: an A/B of engine options on the same box and the same load.

    python shredword-trainer_amd/tools/option_sweep.py --config c4 --set - early_guess=0 apply_helper=0
"""
import argparse
import hashlib
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, REPO)


def say(msg):
    print(f"[sweep {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--set", nargs="+", default=["-"], help="settings: '-' or comma-joined key=value options")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/switch_sweep.json")
    args = ap.parse_args()
    import torch
    import bench
    from shredword.trainer import BPETrainer
    cfg = dict(bench.CONFIGS[args.config])
    d = "/dev/shm/shredword_full"
    os.environ["SHREDWORD_BENCH_DIR"] = d
    path = bench.corpus_path(cfg, args.config)
    done = threading.Event()

    def heartbeat():
        while not done.wait(30):
            say("generating")
    threading.Thread(target=heartbeat, daemon=True).start()
    try:
        gen_s = bench.ensure_corpus(cfg, path)
    finally:
        done.set()
    say(f"generated in {gen_s:.0f} s")
    t = BPETrainer(vocab_size=cfg["vocab"], unk_id=cfg["unk"], character_coverage=cfg["cov"], min_pair_freq=cfg["mpf"])
    t.set_option("log", 0)
    t0 = time.time()
    t.load_corpus(path)
    say(f"loaded in {time.time() - t0:.1f} s")
    res = {"config": args.config, "corpus_bytes": cfg["bytes"], "runs": []}
    tmpd = os.environ.get("TMPDIR", "/tmp")
    defaults = {"early_guess": "1", "apply_helper": "0", "switch_occ": "4000", "early_max_records": str(2**63)}
    for setting in args.set:
        opts = dict(defaults)
        if setting != "-":
            opts.update(kv.split("=", 1) for kv in setting.split(","))
        for k, v in opts.items():
            t.set_option(k, v)
        t.reset()
        n0 = t._train(t.trainer)  # warm
        times = []
        for _ in range(args.steps):
            t.reset()
            torch.cuda.synchronize()
            s0 = time.perf_counter()
            n = t._train(t.trainer)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - s0)
        m, v = os.path.join(tmpd, "sw.model"), os.path.join(tmpd, "sw.vocab")
        t._save(t.trainer, m.encode(), v.encode())
        st = t.stats()
        run = {"setting": setting, "merges": n, "train_s": times, "merges_per_s": n / (sum(times) / len(times)),
               "switch_merge": st.get("index_switch_merge"), "resident_merges": st.get("resident_merges"),
               "model_md5": hashlib.md5(open(m, "rb").read()).hexdigest(),
               "vocab_md5": hashlib.md5(open(v, "rb").read()).hexdigest()}
        res["runs"].append(run)
        say(json.dumps(run))
        if n0 != n:
            raise SystemExit("merge count changed between trains")
    t.destroy()
    os.remove(path)
    res["md5_equal_across_settings"] = len({(r["model_md5"], r["vocab_md5"]) for r in res["runs"]}) == 1
    json.dump(res, open(args.out, "w"), indent=1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
