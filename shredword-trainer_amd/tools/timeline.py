"""Host/device timeline of the indexed merge loop from an index trace (tools/index_trace.py --out):
aligns the device clock (100 MHz) to the host clock (10 ns units) so that the fastest post ->
command-seen is ONE_WAY_US (the one-way latency measured by tools/pingpong.hip), then prints per
merge range the mean of: host post -> device command seen, device command -> header written,
header -> host flag seen (the release and the flag's trip), and the device's gap before the
next command.

    python shredword-trainer_amd/tools/timeline.py gpurun_out/index_trace_c3.npy [--from 16000]
"""
import argparse
import json

import numpy as np

ONE_WAY_US = 1.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npy")
    ap.add_argument("--one-way-us", type=float, default=ONE_WAY_US)
    args = ap.parse_args()
    tr = np.load(args.npy).astype(np.int64)
    if tr.shape[1] < 19:
        raise SystemExit("trace without absolute clocks")
    post = tr[:, 15] * 1e-2          # us, host
    seen = tr[:, 16] * 1e-2
    dcmd = np.unwrap(tr[:, 17].astype(np.float64), period=2.0**32) * 1e-2  # us, device
    dwait = np.unwrap(tr[:, 18].astype(np.float64), period=2.0**32) * 1e-2
    dev = tr[:, 5] * 1e-3             # command -> header written (before the flag's release)
    off = np.min(dcmd - post) - args.one_way_us  # device clock = host clock + off
    cmd_h = dcmd - off
    wait_h = dwait - off
    fence_h = cmd_h + dev
    # the release (L2 write-back + flag store) of merge i, reported in merge i + 1's header
    rel = np.zeros(len(tr))
    if tr.shape[1] >= 37:
        rel[:-1] = tr[1:, 35] * 1e-2
    released_h = fence_h + rel
    seen_dev = (np.unwrap(tr[:, 36].astype(np.float64), period=2.0**32) * 1e-2 - off) if (
        tr.shape[1] >= 37 and tr[:, 36].any()) else None
    rows = []
    edges = [0, 256, 1024, 4096, 8192, 16384, 24576, len(tr)]
    for lo, hi in zip(edges[:-1], edges[1:]):
        if lo >= len(tr) - 1:
            break
        s = slice(max(lo, 1), min(hi, len(tr)))
        prev_fence = fence_h[s.start - 1:s.stop - 1]
        prev_seen = seen[s.start - 1:s.stop - 1]
        rows.append({
            "merges": f"{lo}-{min(hi, len(tr))}",
            "post_to_cmd_us": float(np.mean(cmd_h[s] - post[s])),
            "cmd_to_header_us": float(np.mean(dev[s])),
            "header_to_seen_us": float(np.mean(seen[s] - fence_h[s])),
            "release_us": float(np.mean(rel[s])),
            "released_to_seen_us": float(np.mean(seen[s] - released_h[s])),
            "post_to_poller_saw_us": float(np.mean(seen_dev[s] - post[s])) if seen_dev is not None else None,
            "poller_saw_to_cmd_us": float(np.mean(cmd_h[s] - seen_dev[s])) if seen_dev is not None else None,
            "prev_seen_to_post_us": float(np.mean(post[s] - prev_seen)),
            "prev_header_to_cmd_us": float(np.mean(cmd_h[s] - prev_fence)),
            "wait_start_to_cmd_us": float(np.mean(cmd_h[s] - wait_h[s])),
            "post_before_prev_header": float(np.mean(post[s] < prev_fence)),
            "cycle_us": float(np.mean(np.diff(seen[s.start - 1:s.stop]))),
        })
    print(json.dumps({"clock_offset_us": float(off), "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
