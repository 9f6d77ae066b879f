"""GPU diagnostic: trains the same corpus with and without speculation in lock step
(bpe_merge_batch chunks) and reports the first chunk after which the device token streams
differ; also checks that shred_probe_rollback leaves the stream unchanged."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "shredword-trainer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("SHREDWORD_LOG", "0")
import corpora  # noqa: E402
from shredword import BPETrainer  # noqa: E402
from shredword.cbase import lib  # noqa: E402


def mk(path, layout, spec):
    t = BPETrainer(vocab_size=6000, unk_id=0, character_coverage=0.9995, min_pair_freq=20)
    t.set_option("layout", layout)
    t.set_option("speculate", spec)
    t.load_corpus(path)
    lib.bpe_init(t.trainer)
    return t


def main():
    layout = sys.argv[1] if len(sys.argv) > 1 else "stream"
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    path = "/tmp/dbg_m.txt"
    corpora.gen_synthetic(path, 12_000_000, 31, "mixed")
    a, b = mk(path, layout, 0), mk(path, layout, 1)
    ta = a.tokens()
    # rollback probe on a few pairs present at the start
    for pair in [(101, 32), (32, 116), (116, 104), (104, 101), (101, 101), (108, 108)]:
        lib.shred_probe_rollback(a.trainer, *pair)
        tb = a.tokens()
        same = ta.shape == tb.shape and bool((ta == tb).all())
        print("probe_rollback", pair, "unchanged" if same else "CHANGED", flush=True)
        if not same:
            d = np.nonzero(ta[: min(len(ta), len(tb))] != tb[: min(len(ta), len(tb))])[0]
            print("  len", len(ta), len(tb), "first diff", d[:5], flush=True)
            ta = tb
    done = 0
    while True:
        na = lib.bpe_merge_batch(a.trainer, chunk)
        nb = lib.bpe_merge_batch(b.trainer, chunk)
        done += na
        xa, xb = a.tokens(), b.tokens()
        sa, sb = a.stats(), b.stats()
        if na != nb or xa.shape != xb.shape or not (xa == xb).all():
            print(f"DIVERGED after {done} merges (chunk {chunk}): na={na} nb={nb} len {len(xa)} {len(xb)}"
                  f" spec hits {sb['spec_hits']} misses {sb['spec_misses']}", flush=True)
            for t, nm in ((a, "a"), (b, "b")):
                t._save(t.trainer, f"/tmp/dbg_{nm}.model".encode(), f"/tmp/dbg_{nm}.vocab".encode())
            ma = np.fromfile("/tmp/dbg_a.model", dtype=np.int32).reshape(-1, 3)
            mb = np.fromfile("/tmp/dbg_b.model", dtype=np.int32).reshape(-1, 3)
            dm = np.nonzero((ma != mb).any(axis=1))[0] if ma.shape == mb.shape else [-1]
            print("  merges identical" if len(dm) == 0 else f"  merges differ first at {dm[0]}: {ma[dm[0]]} {mb[dm[0]]}",
                  flush=True)
            m = min(len(xa), len(xb))
            d = np.nonzero(xa[:m] != xb[:m])[0]
            if len(d):
                i = d[0]
                print("  first diff at", i, "nospec", xa[max(0, i - 6): i + 6].tolist(), flush=True)
                print("                    spec  ", xb[max(0, i - 6): i + 6].tolist(), flush=True)
                for tok in set(xa[max(0, i - 6): i + 6].tolist()) | set(xb[max(0, i - 6): i + 6].tolist()):
                    if 256 <= tok < 256 + len(ma):
                        print("   merge", tok, "=", ma[tok - 256][:2].tolist(), flush=True)
            return 1
        if na <= 0:
            break
    print(f"identical through {done} merges; spec hits {b.stats()['spec_hits']} misses {b.stats()['spec_misses']}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
