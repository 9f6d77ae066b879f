#!/usr/bin/env python3
"""Benchmark of the BPE merge path on MI355X (BASELINE.json metric: BPE merges/sec to vocab=32k +
pair-count HBM GB/s).

A step is one full ``train()`` of the HBM-resident corpus (pair count K1 + heap build + every
merge to the target vocab or heap exhaustion), preceded by ``reset()`` which restores the
unmerged word table on the device.  The default workload is BASELINE.json configs[2] (C3), the
config the metric is quoted on ("to vocab=32k") and which fits one GPU: vocab_size=32000,
min_pair_freq=2 (coverage 0.995, unk 0 = the reference Python defaults) on a 10 GB synthetic
UTF-8 corpus from the committed generator (seed 3).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|...] [--layout types|stream]

Legs beside the timed steps (all on the same corpus):
* ``roofline``: K1 ``k_pair_hist`` over the corpus in the stream layout (every occurrence as
  int32 tokens, the north star's flat token array; 4 B/token + 12 B/tile), HIP events on the
  trainer stream, against the 8 TB/s HBM peak; ``traffic`` from the committed PMC passes.
* ``merge_loop``: the dominant kernel of the timed step (the persistent merge loop), which is
  bound by the per-merge round trip, not by bandwidth: µs per merge, device dispatch -> flag.
* ``cpu_baseline``: oracle/bpe_oracle (the reference-faithful CPU restatement) on one host core,
  started AFTER the timed region (the host replay is most of the merge chain, so the baseline
  must not share the host while it runs), train() capped at --cpu-seconds.  ``value`` is the
  measured merges/s of that capped prefix; the full-run estimate along the cost curve committed
  in tests/golden/fullsize/<config>/case.json is reported beside it (``extrapolated_value``).

N GPUs: ``--gpus N`` with N > 1 launches N ranks itself (torch.distributed.run, one process per
GPU, rank r on device r) unless WORLD_SIZE is already set (the driver's own torchrun).
``--dist`` picks what the ranks do:
* ``replicate`` (the default for N > 1): ONE training.  The load is sharded (rank r counts byte
  range r of the corpus on its GPU, the word lists are all-gathered over torch.distributed's RCCL
  -- an nccl group; ``--load-gather rccl`` uses the library's own communicator instead -- and
  merged) and the merge loop runs on every rank.  The merge loop is a serial chain of dependent merges (merge
  m+1's selection needs merge m's exact frequency changes), so ``value`` (merges
  of the one training / max-over-ranks train() time) does not grow with N; ``load`` reports
  the part that does shard (max-over-ranks load_corpus time) and ``end_to_end_s`` = load + one
  train.  ``scaling`` "strong".  When ranks share a device (a rehearsal on fewer GPUs than
  ranks, where RCCL refuses duplicate GPUs) the word lists meet over gloo instead
  (shredword.dist.host_load_gather).
* ``exchange``: ONE training over word-range shards with one RCCL all-gather of the merge's
  records per merge (stream layout); ``value`` as for replicate.
* ``replicas`` (opt-in): N INDEPENDENT jobs, every rank trains its own replica of the workload;
  ``value`` = merges of all ranks / max-over-ranks time, ``scaling`` "weak".  Not a scaling of
  one training.
The K1 leg counts every rank's copy (replicas) or shard of the stream and reports aggregate GB/s.
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "shredword-trainer_amd")
sys.path.insert(0, PKG)
os.environ.setdefault("SHREDWORD_LOG", "0")  # stdout carries exactly one JSON line

CONFIGS = {
    "c1": dict(bytes=10_000_000, seed=1, script="ascii", vocab=8192, mpf=2000, cov=0.995, unk=0,
               desc="C1: BPE vocab_size=8192 min_pair_freq=2000 on 10 MB synthetic ASCII corpus"),
    "c2": dict(bytes=1_000_000_000, seed=2, script="utf8", vocab=8192, mpf=2000, cov=0.995, unk=0,
               desc="C2: BPE vocab_size=8192 (min_pair_freq=2000) on 1 GB synthetic UTF-8 corpus"),
    "c3": dict(bytes=10_000_000_000, seed=3, script="utf8", vocab=32000, mpf=2, cov=0.995, unk=0,
               desc="C3: BPE vocab_size=32000 min_pair_freq=2 on 10 GB synthetic UTF-8 corpus"),
    "c4": dict(bytes=80_000_000_000, seed=4, script="utf8", vocab=32000, mpf=2000, cov=0.995, unk=0, shards=8,
               desc="C4: BPE vocab_size=32000 min_pair_freq=2000 on 80 GB synthetic UTF-8 corpus (8 x 10 GB "
                    "shards of one logical corpus: the byte ranges the ranks of a sharded load count)"),
    "c5": dict(bytes=100_000_000_000, seed=5, script="mixed", vocab=64000, mpf=2000, cov=0.9995, unk=0,
               desc="C5: BPE vocab_size=64000 coverage=0.9995 on 100 GB mixed-script corpus"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def size_label(nbytes: int) -> str:
    for unit, div in (("GB", 10**9), ("MB", 10**6), ("kB", 10**3)):
        if nbytes >= div:
            v = nbytes / div
            return f"{v:g} {unit}"
    return f"{nbytes} B"


def workload_label(name: str, cfg: dict, default_bytes: int) -> str:
    """config.workload: the named config's description, or, when --bytes changed the corpus size,
    the parameters actually run (a 10 GB run was labelled "100 GB")."""
    if cfg["bytes"] == default_bytes:
        return cfg["desc"]
    script = {"ascii": "ASCII", "utf8": "UTF-8", "mixed": "mixed-script"}[cfg["script"]]
    return (f"{name.upper()} parameters at {size_label(cfg['bytes'])}: BPE vocab_size={cfg['vocab']} "
            f"min_pair_freq={cfg['mpf']} coverage={cfg['cov']} on a {size_label(cfg['bytes'])} synthetic {script} "
            f"corpus (seed {cfg['seed']}; the {name.upper()} config itself is {size_label(default_bytes)})")


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def corpus_path(cfg, name):
    d = os.environ.get("SHREDWORD_BENCH_DIR", os.path.join(os.environ.get("TMPDIR", "/tmp"), "shredword_bench"))
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, f"{name}_{cfg['script']}_{cfg['bytes']}_s{cfg['seed']}.txt")


def ensure_corpus(cfg, path, cpus=None):
    """Generates the corpus file once.  cpus: the generator runs on these CPUs (the bench passes
    the GPU's NUMA node), so the file's page-cache pages sit on the node whose threads read them,
    as they would for a file the loader's own readers page in from disk (read right after a
    generator on the other socket wrote them, 100 GB load at ~20 GB/s instead of ~50;
    profiles/r05_c5_load_first_vs_later.txt)."""
    if os.path.exists(path) and os.path.getsize(path) == cfg["bytes"]:
        return 0.0
    gen = os.path.join(PKG, "bin", "gen_corpus")
    if not os.path.exists(gen):
        subprocess.run(["make", "-s", "-C", PKG, os.path.join(PKG, "bin", "gen_corpus")], check=True)
    t0 = time.time()
    tmp = path + ".part"
    threads = str(min(16, os.cpu_count() or 8))
    # the child inherits this process's affinity: set around the spawn, restored after
    mine = set(os.sched_getaffinity(0))
    near = mine & set(cpus) if cpus else set()
    if near:
        os.sched_setaffinity(0, near)
    try:
        subprocess.run([gen, "--bytes", str(cfg["bytes"]), "--seed", str(cfg["seed"]), "--script", cfg["script"],
                        "--out", tmp, "--threads", threads], check=True)
    finally:
        if near:
            os.sched_setaffinity(0, mine)
    os.replace(tmp, path)
    return time.time() - t0


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def l3_domain(cpu):
    """The CPUs sharing `cpu`'s last-level cache (sysfs), within this process's affinity set."""
    allowed = os.sched_getaffinity(0)
    try:
        idx = sorted(os.listdir(f"/sys/devices/system/cpu/cpu{cpu}/cache"))
        for name in reversed(idx):
            if not name.startswith("index"):
                continue
            with open(f"/sys/devices/system/cpu/cpu{cpu}/cache/{name}/shared_cpu_list") as f:
                cpus = set()
                for part in f.read().strip().split(","):
                    lo, _, hi = part.partition("-")
                    cpus.update(range(int(lo), int(hi or lo) + 1))
            return sorted(cpus & allowed) or [cpu]
    except (OSError, ValueError):
        pass
    return [cpu]


def gpu_numa_cpus(dev):
    """The CPUs of the NUMA node the GPU `dev` hangs off (sysfs of its PCI function), or None."""
    try:
        import torch
        pr = torch.cuda.get_device_properties(dev)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read().strip())
        if node < 0:
            return None
        cpus = set()
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            for part in f.read().strip().split(","):
                lo, _, hi = part.partition("-")
                cpus.update(range(int(lo), int(hi or lo) + 1))
        return cpus
    except Exception:  # noqa: BLE001 (no sysfs entry, no torch property: keep the plain choice)
        return None


def pin_host_loop(local_rank, dev=None):
    """Keeps this rank's threads on one last-level-cache domain (the host replay's heap and pair
    table live in that cache; a migration to another CCD starts cold).  Rank r takes the (r+1)-th
    domain of the allowed CPUs; the last CPU stays free for the CPU baseline.  The domains come
    from the NUMA node of the rank's GPU (the records and commands cross PCIe to pinned host memory
    every merge: C3 A/B on one box 54.8-55.6 k on the far socket, 56.1-56.3 k on the GPU's;
    SHREDWORD_PIN_NUMA=0 for the plain choice)."""
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 4:
        return None
    seen, domains = set(), []
    for c in allowed[:-1]:
        if c in seen:
            continue
        d = [x for x in l3_domain(c) if x != allowed[-1]]
        seen.update(d)
        domains.append(d)
    near = gpu_numa_cpus(dev) if (dev is not None and os.environ.get("SHREDWORD_PIN_NUMA", "1") == "1") else None
    if near:
        local = [d for d in domains if set(d) <= near]
        if local:
            # ranks on the same node take its domains in turn; past CPU 0's domain when possible
            start = 1 if len(local) > 1 and 0 in local[0] else 0
            return _pin(local[(start + local_rank) % len(local)])
    # the domain of CPU 0 takes most of the OS's interrupts and housekeeping: start past it
    dom = domains[(local_rank + 1) % len(domains)] if len(domains) > 1 else domains[0]
    return _pin(dom)


def _pin(dom):
    try:
        os.sched_setaffinity(0, set(dom))
    except OSError:
        return None
    return dom


def host_thp():
    """Transparent huge pages of this process (the selector's heap and pair table ask for them:
    a select walks the heap's levels, one TLB entry per 2 MiB instead of per 4 KiB) and the
    kernel's THP settings."""
    out = {}
    try:
        with open("/proc/self/smaps_rollup") as f:
            for line in f:
                if line.startswith(("AnonHugePages:", "Anonymous:")):
                    k, v = line.split(":", 1)
                    out[k.strip() + "_kB"] = int(v.split()[0])
    except OSError:
        pass
    for name in ("enabled", "defrag"):
        try:
            with open(f"/sys/kernel/mm/transparent_hugepage/{name}") as f:
                out[name] = f.read().strip()
        except OSError:
            pass
    return out


def pin_exclusive(dom):
    """The host loop (this thread) alone on one core of its L3 domain: the thread on the domain's
    second core, every other thread of the process (HIP runtime, torch, loaders) moved off that
    core and its SMT sibling.  Threads this one starts later inherit its one-CPU mask, so call it
    after the load.  Returns the CPU, or None when the domain is too small."""
    if not dom or len(dom) < 4:
        return None
    cpu = sorted(dom)[1]
    sib = {cpu}
    try:
        with open(f"/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list") as f:
            for part in f.read().strip().split(","):
                lo, _, hi = part.partition("-")
                sib.update(range(int(lo), int(hi or lo) + 1))
    except OSError:
        pass
    others = set(range(os.cpu_count() or 1)) - sib  # (the kernel intersects it with the cpuset)
    me = threading.get_native_id()
    try:
        for tid in os.listdir("/proc/self/task"):
            if int(tid) != me and others:
                try:
                    os.sched_setaffinity(int(tid), others)
                except OSError:
                    pass
        os.sched_setaffinity(0, {cpu})
    except OSError:
        return None
    return cpu


def cpu_baseline_start(cfg, path, seconds):
    """Starts the CPU port (oracle/bpe_oracle.c: the reference-faithful merge loop, SURVEY.md §8
    d5) on ONE host core — the last core of this process's affinity set — with train() capped at
    `seconds`.  main() starts it after the timed region (it overlaps only the untimed legs);
    cpu_baseline_finish() collects it."""
    exe = os.path.join(REPO, "oracle", "_build", "bpe_oracle")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "port"], check=True)
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), "shredword_cpu_baseline")
    cores = sorted(os.sched_getaffinity(0))
    core = cores[-1]

    def pin():
        try:
            os.sched_setaffinity(0, {core})
        except OSError:
            pass

    errf = open(out + ".err", "w+b")
    proc = subprocess.Popen([exe, path, str(cfg["vocab"]), str(cfg["unk"]), repr(cfg["cov"]), str(cfg["mpf"]),
                             out + ".model", out + ".vocab", "--max-seconds", str(seconds), "--progress", "256"],
                            stdout=subprocess.DEVNULL, stderr=errf, preexec_fn=pin)
    return {"proc": proc, "err": errf, "core": core, "seconds": seconds, "t0": time.time()}


def fullsize_case(cfg_name):
    """The committed full-size oracle run of this config (tests/golden/make_fullsize.py)."""
    try:
        return json.load(open(os.path.join(REPO, "tests", "golden", "fullsize", cfg_name, "case.json")))
    except (OSError, ValueError):
        return None


def cpu_baseline_finish(h, cfg_name, target_merges, gpu_merges, timeout=600, corpus_bytes=None):
    """merges/s of the capped CPU run.  When it stopped early, the full train() time is
    extrapolated along the measured cost curve of the committed full-size run of the same
    corpus and config (the oracle's cumulative train seconds every 256 merges, measured in the
    build container): T_full = t_cap(k) x curve(full) / curve(k), k = merges the capped run
    reached.  The merge loop's per-merge cost falls as the word table shrinks, so this is the
    reference cost model of SURVEY.md §8 d5 (~c x S_live per merge) taken from measurement."""
    try:
        h["proc"].wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        h["proc"].kill()
        raise
    h["err"].seek(0)
    err = h["err"].read().decode()
    h["err"].close()
    if h["proc"].returncode != 0 or "TIMING" not in err:
        raise RuntimeError(f"bpe_oracle failed (rc {h['proc'].returncode}): {err[-300:]}")
    line = err.split("TIMING", 1)[1].splitlines()[0]
    fields = dict(kv.split("=", 1) for kv in line.split() if "=" in kv)
    merges, train_s, load_s = int(fields["merges"]), float(fields["train"]), float(fields["load"])
    res = {
        "value": merges / train_s if train_s > 0 else None, "unit": "merges/s", "cores": 1, "kind": "port",
        "sample": (f"train() of the same corpus/config capped at {h['seconds']:.0f} s: {merges} of "
                   f"{target_merges} merges in {train_s:.1f} s (load {load_s:.1f} s excluded); "
                   f"oracle/bpe_oracle.c pinned to core {h['core']} of {cpu_model()} (nproc={os.cpu_count()}), "
                   f"started after the timed GPU steps (it overlaps only the untimed K1/encode/HBM legs); "
                   f"value = merges/s of this measured prefix"),
        "capped_merges": merges, "capped_train_s": train_s, "load_s": load_s,
        "load_GBps": (corpus_bytes / load_s / 1e9) if corpus_bytes and load_s > 0 else None,
        "calibration": calibration_note(),
    }
    case = fullsize_case(cfg_name)
    if merges < target_merges and case and case.get("oracle", {}).get("progress"):
        curve = case["oracle"]["progress"]
        full_m, full_s = case["merges"], case["oracle"]["train_s"]
        # the container's time to reach `merges`, interpolated on the curve (0 at 0 merges)
        pts = [(0, 0.0)] + [(m, t) for m, t in curve]
        at = None
        for (m0, t0), (m1, t1) in zip(pts, pts[1:]):
            if m0 <= merges <= m1:
                at = t0 + (t1 - t0) * (merges - m0) / max(1, m1 - m0)
                break
        if at and at > 0:
            est = train_s * full_s / at
            res.update({
                "extrapolated_value": full_m / est, "extrapolated_train_s": est,
                "extrapolation": (f"the full train() estimated along the measured cost curve of the full run "
                                  f"(tests/golden/fullsize/{cfg_name}/case.json: {full_s:.0f} s for {full_m} merges on "
                                  f"{case['oracle'].get('cpu', 'the build container')}, a different machine), scaled "
                                  f"by this host's time on the measured prefix (x{train_s / at:.2f}); the per-merge "
                                  f"cost falls as the word table shrinks, so the prefix rate understates the full run"),
            })
    elif merges < target_merges:
        res["note"] = "capped run, no committed full-run curve for this config: value = merges/s of the capped prefix"
    if gpu_merges:
        res["gpu_merges_per_step"] = gpu_merges
    return res


def encode_cpu_baseline(model, vocab, unk, path, sample_bytes=200_000_000):
    """The encoder's CPU port (oracle/encode_oracle.c: the literal merge replay with a per-word
    cache) on one core over the first `sample_bytes` of the corpus (cut at a newline), with the
    same byte map the GPU encoder derives; checks that the ids equal the GPU encoder's."""
    import ctypes
    import numpy as np
    from shredword.encoder import BPEEncoder
    lib_path = os.path.join(REPO, "oracle", "_build", "libbpe_oracle.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "port"], check=True)
    lib = ctypes.CDLL(lib_path)
    lib.or_encode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                              ctypes.c_void_p, ctypes.c_size_t]
    lib.or_encode.restype = ctypes.c_int64
    with open(path, "rb") as f:
        text = f.read(sample_bytes)
    text = text[:text.rfind(b"\n") + 1] or text
    merges = np.fromfile(model, dtype=np.int32).reshape(-1, 3).copy()
    enc = BPEEncoder(model, vocab, unk_id=unk)
    bm = enc.byte_map
    gpu_ids = enc.encode(text)
    enc.destroy()
    buf = np.frombuffer(text, dtype=np.uint8)
    out = np.empty(len(text), dtype=np.int32)
    t0 = time.perf_counter()
    r = lib.or_encode(merges.ctypes.data, merges.shape[0], bm.ctypes.data, buf.ctypes.data, len(text),
                      out.ctypes.data, out.size)
    dt = time.perf_counter() - t0
    return {"value": len(text) / dt / 1e9, "unit": "GB/s of text", "cores": 1, "kind": "port",
            "sample": f"first {len(text)} bytes of the same corpus, oracle/encode_oracle.c (word-cached replay), 1 thread",
            "ids_equal_gpu": bool(r == gpu_ids.size and np.array_equal(out[:max(r, 0)], gpu_ids))}


def calibration_note():
    """The port's speed relative to the reference itself (tests/golden/cpu_calibration.json)."""
    try:
        rows = json.load(open(os.path.join(REPO, "tests", "golden", "cpu_calibration.json")))["rows"]
        ratios = ", ".join(f"{r['train_time_ratio_port_over_reference']:.2f}" for r in rows)
        return (f"port train time / reference train time = {ratios} on C1 and 100 MB "
                f"(same outputs, 1 core each): the reference itself is slower than this baseline")
    except (OSError, ValueError, KeyError):
        return None


PMC_NOTE = ("HBM bytes per k_merge launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, "
            "FETCH doubled for gfx950 16-B reads), committed as profiles/r01_<config>_<layout>_pmc_traffic.json "
            "by shredword-trainer_amd/tools/pmc_summary.py")


HERE = os.path.dirname(os.path.abspath(__file__))


def _pmc_files(cfg_name):
    """The committed PMC summaries of this config, newest first: the round number of the file name
    (rNN_...), then the name (r05_final_c3 before r05_c3).  A summary holds every kernel of its
    profiled bench run (both layouts: the K1 stream leg runs in the same command)."""
    import glob
    import re
    out = []
    for path in glob.glob(os.path.join(HERE, "profiles", "r*_pmc_traffic.json")):
        name = os.path.basename(path)
        m = re.match(r"r(\d+)_", name)
        if m and f"_{cfg_name}_" in name:
            out.append((int(m.group(1)), name, path))
    return [p for _r, _n, p in sorted(out, reverse=True)]


def _pmc_entry(cfg_name, kernel):
    """(summary path, kernel entry) of the newest summary holding `kernel` (a name or a tuple of
    names, first match wins within a file), or (None, None)."""
    names = (kernel,) if isinstance(kernel, str) else tuple(kernel)
    for path in _pmc_files(cfg_name):
        try:
            k = json.load(open(path))["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        for n in names:
            if n.endswith("*"):  # any template instance (one per profiled run)
                hit = [v for kk, v in sorted(k.items()) if kk.startswith(n[:-1]) and v]
                if hit:
                    return path, hit[0]
            elif k.get(n):
                return path, k[n]
    return None, None


def pmc_source(cfg_name, layout, kernel):
    """The committed PMC summary pmc_traffic() reads for this kernel (the newest holding it)."""
    path, _ent = _pmc_entry(cfg_name, kernel)
    if path is None:
        return None
    return ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (FETCH doubled for gfx950 16-B reads): "
            + os.path.relpath(path, HERE))


def pmc_traffic(cfg_name, layout, kernel=None, all_launches=False, raw=False):
    """Measured HBM bytes per launch of `kernel` (default k_merge) for this workload, from the
    newest committed PMC summary holding it (profiles/rNN_*<config>*_pmc_traffic.json).
    all_launches: the sum over the profiled run's launches (the load's segmented count: one load =
    all of them).  raw: FETCH_SIZE as counted (no x2), the lower bound for probe/atomic reads."""
    if kernel is None:
        kernel = "k_merge<true>" if layout == "types" else "k_merge<false>"
    _path, ent = _pmc_entry(cfg_name, kernel)
    if not ent:
        return None
    v = ent["hbm_bytes_per_launch_fetch_raw"] if raw else ent["hbm_bytes_per_launch"]
    return v * (ent.get("launches", 1) if all_launches else 1)


def _per_load(per_launch, nbytes):
    """k_word_count bytes of one load: the per-launch PMC figure x the load's segment launches."""
    if per_launch is None:
        return None
    seg = max(1, int(os.environ.get("SHREDWORD_LOAD_SEGMENT_MB", "512"))) << 20
    return per_launch * -(-int(nbytes) // seg)


def pair_count_leg(cfg, path, reps, device=0, layout="stream", dist=None, shard=False):
    """K1 at HBM scale: the same corpus in the stream layout (every occurrence as int32 tokens,
    the north-star data layout), `reps` x (reset + bpe_init).  k_pair_hist counts the bulk of the
    stream (every occurrence past each type's first) and is timed alone with HIP events on the
    trainer's stream; algorithmic bytes = 4 B per token (word headers are the boundaries) + 12 B
    per tile descriptor (stream mode).  Under N ranks every rank counts its own
    shard of the stream (the per-rank lists are merged over RCCL inside bpe_init) and the leg
    reports the aggregate: sum over ranks of bytes per launch / the slowest rank's launch time."""
    from shredword.cbase import lib
    from shredword.trainer import BPETrainer
    t = BPETrainer(vocab_size=cfg["vocab"], unk_id=cfg["unk"], character_coverage=cfg["cov"], min_pair_freq=cfg["mpf"])
    t.set_option("log", 0)
    t.set_option("device", device)
    t.set_option("layout", layout)
    t0 = time.time()
    t.load_corpus(path)
    load_s = time.time() - t0
    lib.bpe_init(t.trainer)  # warm-up
    t.set_option("timing", 1)
    t.set_option("clear_stats", 1)
    for _ in range(reps):
        t.reset()
        lib.bpe_init(t.trainer)
    st = t.stats()
    t.destroy()
    n = max(1, st["hist_launches"])
    us = 1e3 * st["hist_kernel_ms"] / n
    b = st["hist_kernel_bytes"] / n
    if dist is not None:
        import torch
        tb = torch.tensor([b], dtype=torch.float64)
        dist.all_reduce(tb, op=dist.ReduceOp.SUM)
        tu = torch.tensor([us], dtype=torch.float64)
        dist.all_reduce(tu, op=dist.ReduceOp.MAX)
        b, us = float(tb.item()), float(tu.item())
    achieved = b / (us * 1e-6) / 1e9 if us > 0 else None
    k1_us = 1e3 * st["count_kernel_ms"] / max(1, st["count_launches"])
    return {
        "kernel": "k_pair_hist (K1 bulk, stream layout: packed 16-bit LDS pair table, one workgroup per CU)",
        "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS if achieved else None,
        "traffic": pmc_traffic(cfg.get("name", "c2"), "stream", "k_pair_hist"),
        "traffic_source": pmc_source(cfg.get("name", "c2"), "stream", "k_pair_hist"),
        "avg_launch_us": us, "bytes_per_launch": b, "launches": st["hist_launches"],
        "k1_total_us": k1_us,
        "k1_total_GBps": (st["count_kernel_bytes"] / max(1, st["count_launches"])) / (k1_us * 1e-6) / 1e9 if k1_us > 0 else None,
        "stream_tokens": st["live_tokens"], "tiles": st["num_tiles"], "load_s": load_s,
        "ranks": 1 if dist is None else dist.get_world_size(),
        "aggregate": (("sum of per-rank bytes / slowest rank's avg launch; each rank counts "
                       + ("its shard of the stream" if shard else "its own copy of the stream"))
                      if dist is not None else None),
    }


def encode_leg(model, vocab, unk, path, reps, device=0, cfg_name="c3"):
    """Encoder: the model this run trained applied to its own HBM-resident corpus
    (word-cache kernels + hipCUB scan + k_encode_emit, HIP events on the encoder's stream).  Checks
    the size-independent property that the id counts equal the .vocab frequency column."""
    import numpy as np
    import torch
    from shredword.encoder import BPEEncoder
    enc = BPEEncoder(model, vocab, unk_id=unk, device=device)
    text = torch.from_numpy(np.fromfile(path, dtype=np.uint8)).to(f"cuda:{device}")
    n = text.numel()
    out = torch.empty(n, dtype=torch.int32, device=text.device)
    ids, _ = enc.encode_device(text, out)  # warm-up (scratch allocation)
    times = []
    for _ in range(reps):
        ids, ms = enc.encode_device(text, out)
        times.append(ms)
    ms = sorted(times)[len(times) // 2]
    nids = ids.numel()
    # .vocab frequency column: record i = token i (C string) + " " + freq + "\n" (bpe.cpp:417)
    raw = open(model, "rb").read()
    merges = np.frombuffer(raw, dtype=np.int32).reshape(-1, 3)
    toks = [bytes([b]) for b in range(256)]
    for a, b, _ in merges:
        toks.append(toks[a] + toks[b])
    vb, pos, freq = open(vocab, "rb").read(), 0, []
    for t in toks:
        pos += len(t.replace(b"\0", b"")) + 1
        end = vb.index(b"\n", pos)
        freq.append(int(vb[pos:end]))
        pos = end + 1
    valid = ids[(ids >= 0) & (ids < len(toks))].long()
    counts = torch.bincount(valid, minlength=len(toks)).cpu().numpy()
    alg = n + 4.0 * nids
    enc.destroy()
    del text, out
    torch.cuda.empty_cache()
    per = {k: pmc_traffic(cfg_name, "types", k) for k in
           ("k_cache_insert", "k_cache_encode<true>", "k_cache_words")}
    traffic = sum(v or 0.0 for v in per.values())
    return {"kernel": ("k_cache_insert + k_cache_encode + k_cache_words (ids written in place after a decoupled "
                       "look-back over chunk sums; word cache; median of reps, HIP events)"),
            "traffic_by_kernel": per, "traffic_x_algorithmic": (traffic / alg) if traffic else None,
            "traffic_bytes": traffic or None,
            "text_bytes": n, "ids": nids, "ms": ms, "text_GBps": n / (ms * 1e-3) / 1e9,
            "algorithmic_bytes": alg, "achieved_GBps": alg / (ms * 1e-3) / 1e9,
            "frac_of_hbm_peak": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "counts_match_vocab": bool(np.array_equal(counts, np.array(freq, dtype=np.int64))),
            "note": ("latency of word-cache probes and first-occurrence reads (L2/MALL), not HBM bandwidth; "
                     f"traffic_bytes = PMC bytes of the word-cache kernels per call from the committed {cfg_name} profile")}


def merge_loop_report(st, merges, elapsed, args):
    """The timed step's merge loops with their own algorithmic bytes, each over
    its own merges and its own launch time (HIP events around each persistent launch, the
    durations rocprofv3 --kernel-trace reports for the same kernels):
    * resident (k_resident, merges while they change many words): 4 B per live token per merge
      (K2: the scan of the token table a merge stands for; LDS signatures let it skip tiles);
    * index (k_word_loop, the rest): per merge 16 B per listed pool entry + 8 B weight per scanned
      word + 4 B per run int read (length + tokens) and written back + 16 B per new pool entry
      (changed word) + 24 B per delta record to host memory.
    Both loops are bound by the per-merge round trip (host select/apply <-> device), not by HBM:
    the fractions are reported to show that, not as targets."""
    res_n, idx_n = st["resident_merges"], st["index_merges"]
    out = {
        "bound": "latency (serial merge chain: host heap replay <-> device merge per merge)",
        "us_per_merge": 1e6 * elapsed / max(1, merges),
        "host_s": {k: st[f"host_{k}_seconds"] for k in ("select", "launch", "wait", "apply")},
        "launches": st["merge_launches"],
    }
    if res_n:
        ms = st["resident_kernel_ms"]
        b = st["resident_bytes"]
        gbps = b / (ms * 1e-3) / 1e9 if ms > 0 else None
        out["resident"] = {
            "kernel": "k_resident (persistent, whole chip: LDS signatures, wave-level match + deltas + compaction)",
            "merges": res_n, "launches": st["resident_launches"], "kernel_ms": ms,
            "us_per_merge": 1e3 * ms / res_n, "algorithmic_bytes": b, "algorithmic_bytes_per_merge": b / res_n,
            # K3: the dirty tiles a merge rewrites, read + written (4 B a token each way)
            "k3_dirty_tile_bytes_per_merge": st.get("resident_k3_bytes", 0.0) / res_n,
            "achieved_GBps": gbps, "frac_of_hbm_peak": gbps / HBM_PEAK_GBS if gbps else None,
            "traffic_bytes_per_launch": pmc_traffic(args.config, args.layout, "k_resident*"),
            "traffic_source": pmc_source(args.config, args.layout, "k_resident*"),
            "dispatch_to_flag_us": st.get("resident_latency_us"),
        }
    if idx_n:
        ri, rw = st["index_run_ints_read"], st["index_run_ints_written"]
        b = (16.0 * st["index_candidates"] + 8.0 * st["index_scanned"] + 4.0 * (ri + rw)
             + 16.0 * st["index_changed"] + 24.0 * st["index_records"])
        ms = st["index_ms"]
        gbps = b / (ms * 1e-3) / 1e9 if ms > 0 else None
        busy = st["index_dev_us"]
        wl_names = ("k_word_loop<false, 32>", "k_word_loop<false>")
        wl_traffic = pmc_traffic(args.config, args.layout, wl_names)
        wl_raw = pmc_traffic(args.config, args.layout, wl_names, raw=True)
        per_launch_alg = b / max(1, st["index_launches"])
        out["index"] = {
            "kernel": "k_word_loop (indexed persistent loop, one workgroup: word lists, filter, register merge, "
                      "neighbour deltas, in-place compaction)",
            "merges": idx_n, "undos": st["index_undos"], "launches": st["index_launches"], "kernel_ms": ms,
            "us_per_merge": 1e3 * ms / idx_n,
            "algorithmic_bytes": b, "algorithmic_bytes_per_merge": b / idx_n,
            "bytes_breakdown_per_merge": {
                "pool_entries_listed": 16.0 * st["index_candidates"] / idx_n,
                "weights": 8.0 * st["index_scanned"] / idx_n,
                "runs_read": 4.0 * ri / idx_n, "runs_written": 4.0 * rw / idx_n,
                "pool_entries_appended": 16.0 * st["index_changed"] / idx_n,
                "records_to_host": 24.0 * st["index_records"] / idx_n},
            "achieved_GBps": gbps, "frac_of_hbm_peak": gbps / HBM_PEAK_GBS if gbps else None,
            # PMC of the profiled run's k_word_loop launch (one launch per train()), against this
            # step's algorithmic bytes per launch; the doubled FETCH is the upper bound, raw the lower
            "traffic_bytes_per_launch": wl_traffic, "traffic_bytes_per_launch_fetch_raw": wl_raw,
            "traffic_x_algorithmic": (wl_traffic / per_launch_alg) if wl_traffic else None,
            "traffic_x_algorithmic_fetch_raw": (wl_raw / per_launch_alg) if wl_raw else None,
            "traffic_source": pmc_source(args.config, args.layout, wl_names),
            "device_busy_us_per_merge": busy / idx_n,
            "achieved_GBps_while_busy": b / (busy * 1e-6) / 1e9 if busy > 0 else None,
            "words_listed_per_merge": st["index_candidates"] / idx_n,
            "words_scanned_per_merge": st["index_scanned"] / idx_n,
            "words_changed_per_merge": st["index_changed"] / idx_n,
            "occurrences_per_merge": st["index_occurrences"] / idx_n,
            "k4_on_device": {"merges_finalized": st["index_finalized"],
                             "device_records_out_us_per_merge": st["index_dev_out_us"] / idx_n,
                             "device_finalize_us_per_finalized_merge": st["index_dev_fin_us"] / max(1, st["index_finalized"]),
                             "raw_records_per_finalized_merge": st["index_fin_records"] / max(1, st["index_finalized"]),
                             "raw_records_per_merge": st["index_raw_records"] / idx_n,
                             "changes_or_records_to_host_per_merge": st["index_records"] / idx_n,
                             "note": "finalize_changes: records combined per pair key and ordered (bucket, first "
                                     "touch desc) on the device; the host only walks them"},
            "device_lookup_us_per_merge": st["index_dev_lookup_us"] / idx_n,
            "device_scan_us_per_merge": st["index_dev_scan_us"] / idx_n,
            "host_post_to_flag_us_per_merge": st["index_wait_us"] / idx_n,
            "hybrid_switch_merge": st["index_switch_merge"],
            "hybrid_switch_ms_total": st["index_switch_ms"],
        }
    if not res_n and not idx_n and st["merge_launches"]:
        ms = st["merge_kernel_ms"]
        b = st["merge_kernel_bytes"]
        gbps = b / (ms * 1e-3) / 1e9 if ms > 0 else None
        out["launch"] = {"kernel": "k_merge (one launch per merge)", "merges": st["merge_launches"],
                         "kernel_ms": ms, "us_per_merge": 1e3 * ms / st["merge_launches"],
                         "algorithmic_bytes_per_merge": b / st["merge_launches"], "achieved_GBps": gbps,
                         "frac_of_hbm_peak": gbps / HBM_PEAK_GBS if gbps else None,
                         "traffic_bytes_per_launch": pmc_traffic(args.config, args.layout)}
    return out


def tiebreak_report(st, merges, elapsed, args, out_prefix):
    """tiebreak=device: the device's own selection (k_word_loop<true>), with the size-independent
    checks of its output: non-increasing merge frequencies >= min_pair_freq (from the .model's
    order and the .vocab) are not recomputable without a trace, so the line reports the weighted
    symbol count of the .vocab (invariant under any merge order) beside the exact mode's."""
    import numpy as np
    model, vocab = out_prefix + ".model", out_prefix + ".vocab"
    ops = np.fromfile(model, dtype="<i4").reshape(-1, 3)
    spell = [bytes([i]) if i else b"" for i in range(256)]
    size = [1] * 256
    for a, b, _x in ops:
        spell.append(spell[a] + spell[b])
        size.append(size[a] + size[b])
    vb, pos, sym = open(vocab, "rb").read(), 0, 0
    for tok, sz in zip(spell, size):
        pos += len(tok)
        end = vb.index(b"\n", pos + 1)
        sym += int(vb[pos + 1:end]) * sz
        pos = end + 1
    n = max(1, st["sel_merges"])
    return {
        "mode": "device: merges selected by the largest pair count, ties to the smaller pair key -- the early ones "
                "on the host from exact counts while the whole-chip resident loop merges, then every merge on the GPU "
                "inside k_word_loop<true> (pair table + frontier argmax); NOT the reference's merge order",
        "merges_per_s": merges / elapsed, "sel_merges": st["sel_merges"], "host_phase_merges": st["sel_host_merges"],
        "launches": st["sel_launches"],
        "rebuilds": st["sel_rebuilds"], "rebuild_ms": st["sel_rebuild_ms"], "kernel_ms": st["sel_kernel_ms"],
        "device_select_us_per_merge": st["sel_select_us"] / n, "device_merge_us_per_merge": st["sel_merge_us"] / n,
        "device_table_update_us_per_merge": st["sel_table_us"] / n,
        "table_pairs": st["sel_table_pairs"], "table_slots": st["sel_table_slots"],
        "operands_before_merge": bool((ops[:, :2] < ops[:, 2:3]).all()),
        "weighted_symbols": sym,
    }


def hbm_probe_leg(device=0, nbytes=4 << 30, reps=10):
    """Achievable HBM bandwidth on this box: streaming read and copy kernels
    of the library (shred_hbm_probe), beside the nominal 8 TB/s peak."""
    import ctypes
    from shredword.cbase import lib
    r, c = ctypes.c_double(), ctypes.c_double()
    if lib.shred_hbm_probe(device, nbytes, reps, ctypes.byref(r), ctypes.byref(c)) != 0:
        return {"error": "shred_hbm_probe failed"}
    return {"read_GBps": r.value, "copy_GBps": c.value, "bytes": nbytes, "reps": reps,
            "read_frac_of_nominal": r.value / HBM_PEAK_GBS,
            "kernels": "k_hbm_read (4 x 16 B nontemporal loads per lane in flight), k_hbm_copy"}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv):
    """--gpus N without a surrounding launcher: N ranks under torch.distributed.run (one process
    per GPU, rank r on device r), started as a child before this process touches the GPU; the
    exit code is the launcher's.  Rank 0's JSON line reaches stdout through the inherited pipe."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    log(f"bench: launching {n} ranks: {' '.join(cmd[1:7])} ...")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--layout", default="types", choices=["types", "stream"])
    ap.add_argument("--dist", default="replicate", choices=["replicas", "replicate", "exchange"],
                    help="N > 1: one training with a sharded load (replicate, the default) or a per-merge RCCL "
                         "exchange (exchange), or N independent jobs (replicas); see the module docstring")
    ap.add_argument("--load-gather", default="torch", choices=["torch", "rccl"],
                    help="N > 1 replicate, a GPU per rank: the sharded load's word-list all-gather over "
                         "torch.distributed's RCCL (an nccl group, default) or the library's own RCCL "
                         "communicator (dist_allgather_bytes)")
    ap.add_argument("--tiebreak", default="exact", choices=["exact", "device"],
                    help="merge selection: exact (the reference's heap replay, bit-exact files; default) or device "
                         "(opt-in K5 mode: every merge selected on the GPU, ties to the smaller pair key)")
    ap.add_argument("--bytes", type=int, default=0, help="override the corpus size (testing)")
    ap.add_argument("--device-leg-steps", type=int, default=2,
                    help="untimed leg after the timed steps: tiebreak=device trains on the same corpus (0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--encode-reps", type=int, default=5, help="encoder leg repetitions (0 = skip)")
    ap.add_argument("--no-pin", action="store_true", help="do not keep the host loop on one L3 domain")
    ap.add_argument("--pair-count-reps", type=int, default=10,
                    help="K1 roofline leg on the stream layout of the same corpus (0: skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank bookkeeping only (no GPU, no corpus): rank 0 prints the ranks it saw")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    # Under N ranks, libraries print to the process's stdout (gloo's "[Gloo] Rank r is connected
    # to ..." lines, from C++): fd 1 goes to stderr for the whole run and rank 0 writes its one
    # JSON line to the saved stdout, so the launcher's stdout carries exactly that line.
    json_out = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        sys.stdout.flush()
        json_out = os.dup(1)
        os.dup2(2, 1)

    cfg = dict(CONFIGS[args.config], name=args.config)
    if args.bytes:
        cfg["bytes"] = args.bytes
    # the committed full-size oracle run of this corpus (tests/golden/fullsize/<case>): the config's
    # own size, or e.g. c5_10g for --config c5 --bytes 10000000000
    case_name = args.config if not args.bytes else (
        f"{args.config}_{args.bytes // 10**9}g" if args.bytes % 10**9 == 0 else None)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher's world size is used")

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    if args.dry_run:
        seen = [None] * world
        me = {"rank": rank, "local_rank": local, "world": world, "pid": os.getpid(),
              "device": f"cuda:{local}"}
        if dist is not None:
            dist.all_gather_object(seen, me)
        else:
            seen = [me]
        if rank == 0:
            line = json.dumps({"dry_run": True, "n_gpus": world, "dist": args.dist, "ranks": seen}) + "\n"
            if json_out is not None:
                os.write(json_out, line.encode())
            else:
                sys.stdout.write(line)
                sys.stdout.flush()
        if dist is not None:
            dist.destroy_process_group()
        return

    # rank r on device r; on a box with fewer GPUs than ranks (a rehearsal of the N-GPU run on
    # one card) the ranks share devices round-robin (device_count() does not initialise the GPU)
    ndev = max(1, torch.cuda.device_count())
    dev = local % ndev
    if ndev < world:
        log(f"bench: {world} ranks on {ndev} device(s): rank {rank} shares device {dev} (rehearsal, not a scaling number)")
    torch.cuda.set_device(dev)

    def barrier():
        if dist is not None:
            dist.barrier()

    path = corpus_path(cfg, args.config)
    gen_s = ensure_corpus(cfg, path, cpus=None if args.no_pin else gpu_numa_cpus(dev)) if local == 0 else 0.0
    barrier()
    # C4's corpus is 8 shards of one logical corpus: on one GPU the load counts the 8 byte ranges
    # in turn and merges their word lists, as 8 ranks of a sharded load would (corpus.cpp)
    sim_shards = cfg.get("shards") if world == 1 else None
    if sim_shards:
        os.environ.setdefault("SHREDWORD_LOAD_SIM_SHARDS", str(sim_shards))

    allowed0 = set(os.sched_getaffinity(0))
    pinned = None if args.no_pin else pin_host_loop(local, dev)
    # The pin is for the merge loop (the host replay's tables in one L3).  A load runs on the
    # process's whole CPU share: its 16 readers confined to one 8-core domain measured 0.65 s for
    # C3 against 0.47-0.50 s on the GPU's NUMA node (profiles/r06_load_pin_ab.json);
    # SHREDWORD_BENCH_LOAD_PIN=1 keeps the load on the domain too.
    load_unpinned = pinned is not None and os.environ.get("SHREDWORD_BENCH_LOAD_PIN", "0") != "1"

    def load(p):
        if load_unpinned:
            os.sched_setaffinity(0, allowed0)
        try:
            t.load_corpus(p)
        finally:
            if load_unpinned:
                os.sched_setaffinity(0, set(pinned))
    from shredword import dist as sdist
    from shredword.cbase import lib
    from shredword.trainer import BPETrainer
    one_job = world > 1 and args.dist != "replicas"  # the ranks train ONE model together
    share = world > ndev  # RCCL refuses two ranks on one GPU: the load's gather goes over gloo
    if one_job and share and args.dist == "exchange":
        raise SystemExit("bench: --dist exchange needs one GPU per rank (RCCL per merge); use --dist replicate")
    gather_via = None
    gather_state = {}
    # replicate on a GPU per rank: the load's gather over torch.distributed's RCCL (an nccl group
    # beside the gloo one) unless --load-gather rccl asks for the library's own communicator;
    # exchange needs the library's communicator (a collective per merge)
    # (SHREDWORD_BENCH_NCCL_GATHER=1 takes that path even on a shared card: a rehearsal of the
    # gloo fallback, since RCCL refuses the group there)
    force_nccl = os.environ.get("SHREDWORD_BENCH_NCCL_GATHER", "0") == "1"
    torch_gather = one_job and (not share or force_nccl) and args.dist == "replicate" and args.load_gather == "torch"
    if one_job and not share and not torch_gather:
        sdist.init_from_env(device=dev)
        gather_via = "RCCL all-gather over xGMI (dist_allgather_bytes)"
    rccl_ranks = lib.shred_dist_ranks() if one_job and not share and not torch_gather else 0

    t = BPETrainer(vocab_size=cfg["vocab"], unk_id=cfg["unk"], character_coverage=cfg["cov"], min_pair_freq=cfg["mpf"])
    t.set_option("log", 0)
    t.set_option("device", dev)
    t.set_option("layout", args.layout)
    t.set_option("tiebreak", args.tiebreak)
    if torch_gather:
        try:
            ggroup = dist.new_group(backend="nccl")
            gather_via = "torch.distributed all_gather_object over an nccl (RCCL, xGMI) group"
        except Exception as e:  # noqa: BLE001
            print(f"[WARNING]\t nccl group unavailable ({e!r}); the load gathers over gloo", file=sys.stderr)
            ggroup = None
            gather_via = "torch.distributed all_gather_object over the gloo group (nccl unavailable)"
        t.set_load_gather(rank, world, sdist.host_load_gather(ggroup, fallback=dist.group.WORLD, state=gather_state))
        if share and args.layout == "types":
            t.set_option("resident", 0)
    elif one_job and not share:
        t.set_option("dist", args.dist)
    elif one_job:
        t.set_load_gather(rank, world, sdist.host_load_gather())
        gather_via = "gloo all-gather (shredword.dist.host_load_gather: ranks share a device)"
        if args.layout == "types":
            t.set_option("resident", 0)  # ranks share one GPU: a whole-chip persistent loop per rank would not be co-resident
    barrier()
    t0 = time.time()
    load(path)
    load_s = time.time() - t0
    load_s_max = load_s
    if gather_state.get("fell_back"):
        gather_via = ("torch.distributed all_gather_object over the gloo group (the nccl gather raised: "
                      + gather_state["fell_back"].splitlines()[-1][:160] + ")")
    if dist is not None:
        tl = torch.tensor([load_s], dtype=torch.float64)
        dist.all_reduce(tl, op=dist.ReduceOp.MAX)
        load_s_max = float(tl.item())

    def train_step():
        t.reset()
        n = t._train(t.trainer)  # the BPETrainer.train() ABI call, without its stdout line
        if n < 0:
            raise RuntimeError("bpe_train failed")
        return n

    excl = pin_exclusive(pinned) if (pinned and os.environ.get("SHREDWORD_PIN_EXCLUSIVE", "0") == "1") else None
    for _ in range(args.warmup):
        train_step()
    t.set_option("timing", 1)
    t.set_option("clear_stats", 1)
    # timed region: exactly K steps, bracketed by barrier + device sync
    barrier()
    torch.cuda.synchronize()
    start = time.perf_counter()
    merges = 0
    for _ in range(args.steps):
        merges += train_step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - start
    thp = host_thp()  # while the trainer's selector tables are still mapped
    if excl is not None:
        os.sched_setaffinity(0, set(pinned))  # the later legs and the CPU baseline on the domain again
    all_merges = merges
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tm = torch.tensor([merges], dtype=torch.int64)
        dist.all_reduce(tm, op=dist.ReduceOp.SUM)
        all_merges = int(tm.item())
    st = t.stats()
    tmpd = os.environ.get("TMPDIR", "/tmp")
    t._save(t.trainer, os.path.join(tmpd, f"bench_r{rank}.model").encode(),
            os.path.join(tmpd, f"bench_r{rank}.vocab").encode())
    # untimed leg: the opt-in tiebreak=device mode on the same loaded corpus and box (not the
    # reference's merge order, so never `value`): one warm train, then --device-leg-steps timed
    device_leg = None
    if (rank == 0 and world == 1 and args.tiebreak == "exact" and args.layout == "types"
            and args.device_leg_steps > 0):
        try:
            t.set_option("tiebreak", "device")
            train_step()
            t.set_option("clear_stats", 1)
            torch.cuda.synchronize()
            d0 = time.perf_counter()
            dm = 0
            for _ in range(args.device_leg_steps):
                dm += train_step()
            torch.cuda.synchronize()
            de = time.perf_counter() - d0
            std = t.stats()
            dpre = os.path.join(tmpd, f"bench_r{rank}_device")
            t._save(t.trainer, (dpre + ".model").encode(), (dpre + ".vocab").encode())
            device_leg = tiebreak_report(std, dm, de, args, dpre)
            device_leg["steps"] = args.device_leg_steps
            device_leg["exact_merges_per_s_same_run"] = merges / elapsed
            device_leg["ratio_to_exact_same_run"] = (dm / de) / (merges / elapsed)
        except Exception as e:  # the exact line stands on its own
            device_leg = {"error": repr(e)}
    # a second load of the same file (untimed, one rank): the step's load above is the first of this
    # process -- the first after the corpus was generated when gen_s > 0, with the file's page-cache
    # pages fresh -- and later loads (the pinned ring kept, pages warm) are faster
    later_load_s = None
    if world == 1:
        try:
            t1 = time.time()
            load(path)
            later_load_s = time.time() - t1
        except Exception:  # noqa: BLE001 (the line stands without it)
            later_load_s = None
    # the CPU baseline starts only now: the timed steps ran with the host to themselves
    cpu_h = None
    if world == 1 and not args.no_cpu_baseline:
        try:
            cpu_h = cpu_baseline_start(cfg, path, args.cpu_seconds)
        except Exception as e:  # the GPU number stands on its own
            cpu_h = {"error": repr(e)}
    t.destroy()

    # K1 HBM leg (the metric's "pair-count HBM GB/s"): every rank counts its stream copy / shard
    pair_count = None
    if args.pair_count_reps > 0:
        try:
            pair_count = pair_count_leg(cfg, path, args.pair_count_reps, device=dev, dist=dist,
                                        shard=one_job)
        except Exception as e:
            pair_count = {"error": repr(e)}

    encode = None
    if args.encode_reps > 0 and rank == 0:
        try:
            encode = encode_leg(os.path.join(tmpd, f"bench_r{rank}.model"), os.path.join(tmpd, f"bench_r{rank}.vocab"),
                                cfg["unk"], path, args.encode_reps, device=dev, cfg_name=args.config)
        except Exception as e:
            encode = {"error": repr(e)}

    if rank == 0:
        per_step_merges = merges / max(1, args.steps)
        value = (all_merges if not one_job else merges) / elapsed
        if one_job:
            parallelism = (f"dp{world} one training: sharded load (byte ranges, RCCL all-gather of word lists) + "
                           f"merge loop replicated on every rank" if args.dist == "replicate" else
                           f"dp{world} one training: word-range shards + one RCCL all-gather of records per merge")
        elif world > 1:
            parallelism = (f"replicas{world}: N INDEPENDENT jobs, every rank trains its own replica of the workload "
                           f"(not one training; the merge chain is serial, DESIGN.md §5); value = merges of all ranks "
                           f"/ slowest rank's time")
        else:
            parallelism = "single GPU"
        result = {
            "metric": "BPE merges/sec",
            "value": value,
            "unit": "merges/s",
            "n_gpus": min(world, ndev),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if one_job else "weak",
            "tiebreak": args.tiebreak,
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (committed deterministic generator, SURVEY.md §8 d2)",
            "config": {
                "workload": workload_label(args.config, cfg, CONFIGS[args.config]["bytes"]),
                "corpus_bytes": cfg["bytes"], "seed": cfg["seed"], "script": cfg["script"],
                "vocab_size": cfg["vocab"], "min_pair_freq": cfg["mpf"], "character_coverage": cfg["cov"],
                "unk_id": cfg["unk"], "layout": args.layout,
                "parallelism": parallelism, "dist": args.dist if world > 1 else None, "rccl_ranks": rccl_ranks,
                "ranks": world, "devices": ndev if world > 1 else 1,
                "ranks_share_devices": world > ndev,
                "load_gather": gather_via,
                "merges_per_step": per_step_merges, "distinct_words": st["num_words"],
                "symbols": st["num_symbols"], "occurrences": st["num_occurrences"], "tiles": st["num_tiles"],
            },
            "roofline": None,
            "merge_loop": merge_loop_report(st, merges, elapsed, args),
            "pair_count_types": {
                "kernel": "k_pair_dense (K1 of this train(): types layout, weighted, first touch)",
                "avg_launch_us": 1e3 * st["count_kernel_ms"] / max(1, st["count_launches"]),
                "bytes_per_launch": st["count_kernel_bytes"] / max(1, st["count_launches"]),
            },
            "load_s": load_s_max, "corpus_gen_s": gen_s,
            "train_s": elapsed / args.steps,
            "end_to_end_s": load_s_max + elapsed / args.steps,
            "load": {"kernel": "k_word_count (one pass, LDS-staged tiles, byte-exact in-pass verification)",
                     "algorithmic_bytes": cfg["bytes"],
                     "load_s_max_over_ranks": load_s_max, "load_s_rank0": load_s,
                     "first_load_s": load_s, "first_load_after_generation": gen_s > 0,
                     "later_load_s": later_load_s,
                     "bytes_per_rank": cfg["bytes"] / world if one_job else cfg["bytes"],
                     # one load = one k_word_count launch per 512 MiB segment (the profiled run holds two loads)
                     "traffic_bytes": _per_load(pmc_traffic(args.config, args.layout, "k_word_count*"), cfg["bytes"]),
                     "traffic_bytes_fetch_raw": _per_load(pmc_traffic(args.config, args.layout, "k_word_count*", raw=True),
                                                          cfg["bytes"]),
                     "traffic_source": pmc_source(args.config, args.layout, "k_word_count*"),
                     "note": ("load_corpus: page-in + PCIe upload + device word count + host table; outside the timed "
                              "step" + ("; each rank counts its byte range, the word lists are all-gathered and "
                                        "merged on every rank" if one_job else ""))},
            "host_thp": thp,
            "host_cpus": (f"pinned to the L3 domain {pinned[0]}-{pinned[-1]} ({len(pinned)} CPUs)"
                          + (f"; the host loop alone on CPU {excl} (no other thread on its core)" if excl is not None else "")
                          if pinned
                          else "not pinned"),
            "host_breakdown_s": {k: st[f"host_{k}_seconds"] for k in ("select", "launch", "wait", "apply")},
            "host_apply_split_s": {k: st[f"host_apply_{k}_seconds"]
                                   for k in ("combine", "correct", "finish", "early", "offer")},
            "init_s_last_step": st["init_seconds"],
            "selector_last_step": {k: st[k] for k in ("heap_pops", "heap_stale_pops", "heap_pushes", "delta_records",
                                                      "apply_cycles_combine", "apply_cycles_order",
                                                      "apply_cycles_walk", "apply_cycles_push",
                                                      "helper_adopted")},
            "tiles_visited_per_merge": st["tiles_visited"] / max(1, merges),
            "speculation": {"hits": st["spec_hits"], "misses": st["spec_misses"],
                            "hit_rate": st["spec_hits"] / max(1, st["spec_hits"] + st["spec_misses"])},
        }
        k1 = result["pair_count_types"]
        k1["achieved_GBps"] = (k1["bytes_per_launch"] / (k1["avg_launch_us"] * 1e-6) / 1e9
                               if k1["avg_launch_us"] > 0 else None)
        if args.tiebreak == "device":
            result["tiebreak_device"] = tiebreak_report(st, merges, elapsed, args, os.path.join(tmpd, f"bench_r{rank}"))
        if device_leg is not None:
            result["tiebreak_device_leg"] = device_leg
        case = fullsize_case(case_name) if case_name else None
        if case and case["recipe"]["bytes"] == cfg["bytes"] and args.tiebreak == "exact":
            result["config"]["corpus_md5_expected"] = case["corpus_md5"]
            result["config"]["unique_bytes"] = case["unique_bytes"]
            # size-independent parity at full size: the bench's own .model/.vocab against the
            # committed full-run oracle output of this corpus (tests/golden/fullsize/)
            import hashlib
            mm = hashlib.md5(open(os.path.join(tmpd, f"bench_r{rank}.model"), "rb").read()).hexdigest()
            vm = hashlib.md5(open(os.path.join(tmpd, f"bench_r{rank}.vocab"), "rb").read()).hexdigest()
            result["parity_fullsize"] = {"model_md5_equal": mm == case["model_md5"],
                                         "vocab_md5_equal": vm == case["vocab_md5"],
                                         "merges_equal": per_step_merges == case["merges"],
                                         "reference": f"tests/golden/fullsize/{case_name}/case.json"}
        if pair_count is not None:
            result["pair_count"] = pair_count
            if pair_count.get("achieved"):
                result["roofline"] = {k: pair_count[k] for k in ("kernel", "bound", "achieved", "peak", "unit", "frac",
                                                                 "traffic")}
                result["roofline"]["traffic_unit"] = "HBM bytes per launch (PMC)"
                result["roofline"]["traffic_source"] = pair_count.get("traffic_source")
                result["roofline"]["algorithmic_bytes_per_launch"] = pair_count["bytes_per_launch"]
                result["roofline"]["avg_launch_us"] = pair_count["avg_launch_us"]
                result["roofline"]["note"] = ("K1, the pair-count scan the north star sets the HBM-roofline target on; "
                                              "the timed step's dominant kernels are the latency-bound merge loops "
                                              "(merge_loop.resident, merge_loop.index)")
        if encode is not None:
            result["encode"] = encode
        try:
            result["hbm_achievable"] = hbm_probe_leg(device=dev)
            if (result.get("pair_count") or {}).get("achieved"):
                result["pair_count"]["frac_of_achievable_read"] = (
                    result["pair_count"]["achieved"] / world / result["hbm_achievable"]["read_GBps"])
        except Exception as e:
            result["hbm_achievable"] = {"error": repr(e)}
        if cpu_h is not None:
            try:
                if "error" in cpu_h:
                    raise RuntimeError(cpu_h["error"])
                result["cpu_baseline"] = cpu_baseline_finish(cpu_h, case_name or args.config, cfg["vocab"] - 256,
                                                             per_step_merges, corpus_bytes=cfg["bytes"])
            except Exception as e:  # the GPU number stands on its own
                result["cpu_baseline"] = {"value": None, "error": repr(e)}
            if isinstance(encode, dict) and "ms" in encode:
                try:
                    encode["cpu_baseline"] = encode_cpu_baseline(os.path.join(tmpd, f"bench_r{rank}.model"),
                                                                 os.path.join(tmpd, f"bench_r{rank}.vocab"),
                                                                 cfg["unk"], path)
                except Exception as e:
                    encode["cpu_baseline"] = {"value": None, "error": repr(e)}
        if json_out is not None:
            os.write(json_out, (json.dumps(result) + "\n").encode())
        else:
            print(json.dumps(result), flush=True)
    if one_job and not share:
        sdist.finalize()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
