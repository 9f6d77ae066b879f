"""Per-kernel totals of any rocprofv3 --pmc counter pass (run_counter_collection.csv): launches,
sum and mean per launch of every counter, plus the LDS ratios the merge loops are judged by
(bank-conflict cycles per LDS-active cycle, LDS-wait share of wave cycles).

    python pmc_counters.py COUNTER_CSV OUT_JSON [--kernels k_resident k_word_loop] [--note TEXT]
"""
import argparse
import collections
import csv
import json
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("out")
    ap.add_argument("--kernels", nargs="*", default=None)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(a.csv)):
        m = re.search(r"(k_[a-z_]+)(<[a-z, ]+>)?", r["Kernel_Name"])
        key = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"].split("(")[0][-60:]
        if a.kernels and not any(key.startswith(k) for k in a.kernels):
            continue
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {"source": a.csv, "note": a.note, "kernels": {}}
    for k, cs in sorted(vals.items()):
        ent = {"launches": max(len(v) for v in cs.values()),
               "sum": {c: sum(v) for c, v in cs.items()},
               "per_launch": {c: sum(v) / len(v) for c, v in cs.items()}}
        s = ent["sum"]
        if s.get("SQ_LDS_IDX_ACTIVE"):
            ent["lds_bank_conflict_per_lds_active"] = s.get("SQ_LDS_BANK_CONFLICT", 0.0) / s["SQ_LDS_IDX_ACTIVE"]
        if s.get("SQ_WAVE_CYCLES"):
            ent["lds_wait_share_of_wave_cycles"] = s.get("SQ_WAIT_INST_LDS", 0.0) / s["SQ_WAVE_CYCLES"]
            ent["any_wait_share_of_wave_cycles"] = s.get("SQ_WAIT_ANY", 0.0) / s["SQ_WAVE_CYCLES"]
            ent["active_inst_share_of_wave_cycles"] = s.get("SQ_ACTIVE_INST_ANY", 0.0) / s["SQ_WAVE_CYCLES"]
        res["kernels"][k] = ent
    json.dump(res, open(a.out, "w"), indent=1)
    for k, e in res["kernels"].items():
        print(k, e["launches"], {x: round(y, 4) for x, y in e.items() if isinstance(y, float)})


if __name__ == "__main__":
    main()
