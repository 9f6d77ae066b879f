"""Summarises a rocprofv3 kernel-trace database (rocpd sqlite): per-kernel count/avg/min/p50/p90
duration, gaps between consecutive k_merge launches, and k_merge duration by grid size."""
import collections
import sqlite3
import sys

import numpy as np


def main(path):
    cur = sqlite3.connect(path).cursor()
    rows = cur.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    by = collections.defaultdict(list)
    for n, s, e, g, w in rows:
        by[n.split("(")[0][-48:]].append((s, e, g // max(1, w)))
    print("calls  kernel                                             avg_us  min_us  p50_us  p90_us")
    for n, v in sorted(by.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1])):
        d = np.array([e - s for s, e, _ in v]) / 1e3
        print(f"{len(v):6d} {n:50s} {d.mean():7.2f} {d.min():7.2f} {np.median(d):7.2f} {np.percentile(d, 90):7.2f}")
    km = [(s, e, g) for n, s, e, g, w in ((r[0], r[1], r[2], r[3] // max(1, r[4]), r[4]) for r in rows) if "k_merge" in n]
    if len(km) > 1:
        gaps = np.array([km[i + 1][0] - km[i][1] for i in range(len(km) - 1)]) / 1e3
        print("k_merge launch-to-launch gap us: p10 %.2f p50 %.2f p90 %.2f" % tuple(np.percentile(gaps, [10, 50, 90])))
        grids = np.array([g for _, _, g in km])
        dur = np.array([e - s for s, e, _ in km]) / 1e3
        for lo, hi in [(0, 8), (8, 64), (64, 192), (192, 256), (256, 1 << 30)]:
            m = (grids > lo) & (grids <= hi)
            if m.sum():
                print(f"k_merge grid ({lo},{hi}]: n={m.sum()} avg {dur[m].mean():.2f} min {dur[m].min():.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
