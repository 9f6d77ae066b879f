"""Per-merge host phases of one train() (SHREDWORD_ENGINE_TRACE file: merge, hit, select, launch,
wait, apply µs, records) summarised by merge range, as committed under profiles/*_engine_phases.json.

    python engine_phases.py TRACE OUT_JSON [--bench BENCH_JSON] [--note TEXT]
"""
import argparse
import json

import numpy as np

EDGES = [0, 200, 500, 1117, 2000, 3500, 5657, 8000, 16000, 24000, 1 << 30]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("out")
    ap.add_argument("--bench", default=None)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    t = np.loadtxt(a.trace)
    m, hit, sel, post, wait, app, rec = (t[:, i] for i in range(7))
    tot = sel + post + wait + app
    res = {"source": ("SHREDWORD_ENGINE_TRACE of one C3 train(), host clock per merge: select = heap replay, "
                      "post_and_guess = guess (heap walk + replayed select) and posting, wait = collect (device "
                      "records), apply = combine + order + info updates + pushes"),
           "note": a.note, "total_ms": float(tot.sum() / 1e3), "phases": []}
    if a.bench:
        b = json.load(open(a.bench))
        res["bench_value_same_run"] = b["value"]
        res["hybrid_switch_merge"] = b["merge_loop"].get("index", {}).get("hybrid_switch_merge")
    n = len(m)
    for lo, hi in zip(EDGES, EDGES[1:]):
        s = (m >= lo) & (m < hi)
        if not s.any():
            continue
        res["phases"].append({
            "merges": f"{lo}-{min(hi, n)}", "hit_rate": round(float(hit[s].mean()), 4),
            "select_us": round(float(sel[s].mean()), 2), "post_and_guess_us": round(float(post[s].mean()), 2),
            "wait_us": round(float(wait[s].mean()), 2), "apply_us": round(float(app[s].mean()), 2),
            "total_us": round(float(tot[s].mean()), 2), "records": round(float(rec[s].mean()), 1),
            "sum_ms": round(float(tot[s].sum() / 1e3), 1)})
    json.dump(res, open(a.out, "w"), indent=1)
    for p in res["phases"]:
        print(p)


if __name__ == "__main__":
    main()
