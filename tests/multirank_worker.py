"""One rank of the CPU multi-rank test (torch.distributed gloo, 127.0.0.1).

Runs the product host Engine over the test harness's kernel emulation on this rank's word-range
shard (tiles.h shard_range); the dense per-merge delta tables, the initial pair table and the
final token histogram are all-reduced over gloo (sum / min) — the exchange the RCCL path does
over xGMI.  Rank 0 writes .model/.vocab/trace.

usage: multirank_worker.py CORPUS VOCAB UNK COV MPF LAYOUT OUTDIR
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import hostharness  # noqa: E402

U64_MAX = np.uint64(0xFFFFFFFFFFFFFFFF)
I64_MAX = np.int64(0x7FFFFFFFFFFFFFFF)


def main():
    corpus, vocab, unk, cov, mpf, layout, outdir = sys.argv[1:8]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = hostharness.load() if rank == 0 else None
    dist.barrier()
    if lib is None:
        lib = hostharness.load()

    def exchange(_ctx, psum, pmin, n):
        s = np.ctypeslib.as_array(psum, shape=(n,))
        m = np.ctypeslib.as_array(pmin, shape=(n,))
        ts = torch.from_numpy(s.view(np.int64).copy())
        dist.all_reduce(ts, op=dist.ReduceOp.SUM)
        mi = m.copy().view(np.int64)
        mi[m == U64_MAX] = I64_MAX
        tm = torch.from_numpy(mi)
        dist.all_reduce(tm, op=dist.ReduceOp.MIN)
        r = tm.numpy()
        back = r.copy().view(np.uint64)
        back[r == I64_MAX] = U64_MAX
        s[:] = ts.numpy().view(np.uint64)
        m[:] = back

    cb = hostharness.EXCHANGE_CB(exchange)
    cfg = {"vocab_size": int(vocab), "unk_id": int(unk), "character_coverage": float(cov), "min_pair_freq": int(mpf)}
    h = hostharness.open_case(lib, corpus, cfg, layout, rank, world)
    lib.hh_set_exchange(h, cb, None)
    tiles = lib.hh_num_tiles(h)
    trace = os.path.join(outdir, f"trace_r{rank}.txt")
    merges = lib.hh_train(h, trace.encode())
    lib.hh_save(h, os.path.join(outdir, "mr.model").encode(), os.path.join(outdir, "mr.vocab").encode(),
                1 if rank == 0 else 0)
    with open(os.path.join(outdir, f"info_r{rank}.txt"), "w") as f:
        f.write(f"{merges} {tiles}\n")
    lib.hh_close(h)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
