"""A/B runs on one GPU box: the same command under several variants (a library build via
SHREDWORD_LIB and/or environment settings), interleaved A B A B ... so box drift hits every variant
alike; prints one JSON summary (per variant: every run's metric, min / median / max).

    python shredword-trainer_amd/tools/ab.py --runs 2 --tag fast \\
        --variant base=lib:variants/libtrainer_r06a.so --variant new=lib:variants/libtrainer_r06b.so \\
        --variant nofast=env:SHREDWORD_WL_FAST=0 \\
        [--cmd "python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"] [--metric value]

Variants are NAME=SPEC, SPEC a comma list of lib:PATH and env:KEY=VALUE items ("default" for
none).  --cmd is run through the shell with {out} replaced by a per-run JSON path under
gpurun_out/; the metric is read from the last JSON line of stdout (or of {out} when the command
writes one).  Replaces round 5's per-experiment shell wrappers (ab.sh, env_ab.sh, switch_ab.sh ...).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

DEFAULT_CMD = ("python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --pair-count-reps 0 --encode-reps 0 "
               "--device-leg-steps 0")


def parse_variant(text):
    name, _, spec = text.partition("=")
    lib, env = None, {}
    for item in [x for x in spec.split(",") if x and x != "default"]:
        kind, _, val = item.partition(":")
        if kind == "lib":
            lib = val
        elif kind == "env":
            k, _, v = val.partition("=")
            env[k] = v
        else:
            raise SystemExit(f"bad variant item {item!r}")
    return name, lib, env


def last_json(text):
    for line in reversed(text.strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except json.JSONDecodeError:
                continue
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", required=True)
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--tag", default="ab")
    ap.add_argument("--cmd", default=DEFAULT_CMD)
    ap.add_argument("--metric", default="value")
    ap.add_argument("--timeout", type=int, default=300)
    a = ap.parse_args()
    variants = [parse_variant(v) for v in a.variant]
    os.makedirs("gpurun_out", exist_ok=True)
    res = {name: [] for name, _, _ in variants}
    for i in range(a.runs):
        for name, lib, env in variants:
            out = f"gpurun_out/ab_{a.tag}_{name}_{i}.json"
            e = dict(os.environ, **env)
            if lib:
                e["SHREDWORD_LIB"] = os.path.abspath(lib)
            cmd = a.cmd.replace("{out}", out)
            p = subprocess.run(["timeout", "-k", "10", str(a.timeout), "bash", "-c", cmd], env=e,
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
            with open(out + ".err", "w") as f:
                f.write(p.stderr)
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                raise SystemExit(f"{name} run {i}: exit {p.returncode}")
            d = last_json(p.stdout)
            if d is None and os.path.exists(out):
                d = last_json(open(out).read())
            if d is None:
                raise SystemExit(f"{name} run {i}: no JSON output")
            with open(out, "w") as f:
                json.dump(d, f)
            v = d
            for k in a.metric.split("."):
                v = v[k]
            res[name].append(float(v))
            print(f"[ab] {name} run {i}: {a.metric} = {v}", file=sys.stderr, flush=True)
    summary = {"tag": a.tag, "cmd": a.cmd, "metric": a.metric,
               "variants": {n: {"spec": {"lib": lib, "env": env}, "runs": res[n], "min": min(res[n]),
                                "median": statistics.median(res[n]), "max": max(res[n])}
                            for n, lib, env in variants}}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
