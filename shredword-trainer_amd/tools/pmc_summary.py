"""Per-kernel HBM traffic from two rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE), corrected
as MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE (KiB) reports half the bytes of the
16-B-per-lane streaming reads these kernels issue, so it is doubled; WRITE_SIZE (KiB) is exact.

    python pmc_summary.py FETCH_CSV WRITE_CSV OUT_JSON --workload c2 --layout types
"""
import argparse
import collections
import csv
import json
import re


def per_kernel(path):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        m = re.search(r"(k_[a-z_0-9]+)(<[^<>()]*>)?", name)
        key = (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0]
        out[key].append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--layout", default="types")
    a = ap.parse_args()
    f, w = per_kernel(a.fetch), per_kernel(a.write)
    res = {"workload": a.workload, "layout": a.layout,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (KiB per dispatch); "
                     "read bytes = 2 x FETCH_SIZE (gfx950 16-B/lane reads), write bytes = WRITE_SIZE",
           "calibration": "the x2 on FETCH_SIZE is calibrated for 16-B/lane streaming reads only "
                          "(MI355X_MICROARCH.md, HBM); other access widths are uncalibrated, so for kernels that "
                          "read by hash probes, atomics and random lines (k_word_count, k_cache_*) the read bytes "
                          "lie between hbm_bytes_per_launch_fetch_raw and hbm_bytes_per_launch; Infinity Cache "
                          "hits are counted, not excluded",
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fv, wv = f.get(k, []), w.get(k, [])
        rd = 2.0 * 1024.0 * (sum(fv) / len(fv)) if fv else None
        wr = 1024.0 * (sum(wv) / len(wv)) if wv else None
        res["kernels"][k] = {"launches": max(len(fv), len(wv)), "read_bytes_per_launch": rd,
                             "write_bytes_per_launch": wr,
                             "hbm_bytes_per_launch": (rd or 0.0) + (wr or 0.0),
                             # FETCH_SIZE as counted (no x2): the lower bound for kernels whose
                             # reads are not 16-B/lane streams (hash probes, atomics, random lines)
                             "hbm_bytes_per_launch_fetch_raw": (rd or 0.0) / 2.0 + (wr or 0.0)}
    json.dump(res, open(a.out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k:28s} launches {v['launches']:6d}  HBM bytes/launch {v['hbm_bytes_per_launch'] / 1e6:10.3f} MB")


if __name__ == "__main__":
    main()
