"""Joins a rocprofv3 kernel-trace database with a SHREDWORD_MERGE_LOG file (launch order = seq
order) and reports k_merge duration against tiles visited and occurrences merged."""
import sqlite3
import sys

import numpy as np


def main(db, log):
    cur = sqlite3.connect(db).cursor()
    dur = [e - s for n, s, e in cur.execute("select name, start, end from kernels order by start") if "k_merge" in n]
    ent = {}
    for line in open(log):
        f = line.split()
        seq = int(f[1])
        if f[0] == "C":
            ent[seq] = dict(kind="C", tiles=int(f[3]), grid=int(f[4]), direct=int(f[5]), merged=int(f[6]), recs=int(f[7]))
        else:
            ent[seq] = dict(kind="R", tiles=int(f[3]), grid=int(f[4]), direct=int(f[5]), merged=-1, recs=-1)
    seqs = sorted(ent)
    if len(seqs) != len(dur):
        print(f"warning: {len(seqs)} logged launches vs {len(dur)} k_merge kernels; joining the common prefix")
    n = min(len(seqs), len(dur))
    rows = [(ent[seqs[i]], dur[i] / 1e3) for i in range(n)]
    d = np.array([r[1] for r in rows])
    tiles = np.array([r[0]["tiles"] for r in rows])
    merged = np.array([r[0]["merged"] for r in rows])
    recs = np.array([r[0]["recs"] for r in rows])
    print(f"{n} launches, total {d.sum() / 1e3:.1f} ms, mean {d.mean():.2f} us")
    print("tiles visited        n   mean_us  min_us  share_of_time")
    for lo, hi in [(0, 16), (16, 128), (128, 768), (768, 2000), (2000, 1 << 40)]:
        m = (tiles >= lo) & (tiles < hi)
        if m.sum():
            print(f"[{lo:5d},{hi if hi < 1 << 40 else 'inf'}) {m.sum():6d} {d[m].mean():8.2f} {d[m].min():7.2f} {d[m].sum() / d.sum():7.1%}")
    full = tiles >= 2000
    if full.sum():
        print("full scans by occurrences merged:")
        for lo, hi in [(-1, 0), (0, 1000), (1000, 10000), (10000, 100000), (100000, 1 << 40)]:
            m = full & (merged >= lo) & (merged < hi)
            if m.sum():
                print(f"  merged [{lo},{hi}) n={m.sum():5d} mean {d[m].mean():7.2f} us  recs {recs[m].mean():8.1f}")
        x = merged[full & (merged >= 0)]
        y = d[full & (merged >= 0)]
        if len(x) > 10:
            A = np.vstack([np.ones_like(x, dtype=float), x]).T
            c = np.linalg.lstsq(A, y, rcond=None)[0]
            print(f"  fit: duration ~ {c[0]:.2f} us + {c[1] * 1e3:.3f} ns x merged occurrences")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
