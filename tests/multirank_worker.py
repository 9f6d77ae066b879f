"""One rank of the CPU multi-rank test (torch.distributed gloo, 127.0.0.1).

Runs the product host Engine over the test harness's kernel emulation on this rank's word-range
shard (tiles.h shard_range).  Each merge's delta records are all-gathered over gloo (every
rank's list, concatenated in rank order — the records exchange the device path does with RCCL
over xGMI); the initial pair table and the final token histogram are all-reduced (sum / min).
Rank 0 writes .model/.vocab/trace.

With SHARDED_LOAD=1 the load is sharded instead (corpus.h LoadOptions::shard_*: each rank counts
its byte range, the word lists are merged over the same gloo all-gather) and the merge loop runs
replicated over the full table, with no per-merge exchange; info_r<rank>.txt then also carries the
table's fingerprint.

usage: multirank_worker.py CORPUS VOCAB UNK COV MPF LAYOUT OUTDIR [SPECULATE [CHAIN]]
"""
import ctypes
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
    speculate = int(sys.argv[8]) if len(sys.argv) > 8 else 1
    chain = int(sys.argv[9]) if len(sys.argv) > 9 else 1
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

    keep = {}

    def gather(_ctx, send, nbytes, out_bytes):
        mine = np.frombuffer(ctypes.string_at(send, nbytes), dtype=np.uint8) if nbytes else np.zeros(0, np.uint8)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([nbytes], dtype=torch.int64))
        top = max(int(t.item()) for t in sizes)
        buf = torch.zeros(max(top, 1), dtype=torch.uint8)
        buf[:nbytes] = torch.from_numpy(mine.copy())
        parts = [torch.zeros(max(top, 1), dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, buf)
        cat = b"".join(bytes(p[:int(sz.item())].numpy()) for p, sz in zip(parts, sizes))
        keep["buf"] = ctypes.create_string_buffer(cat, max(len(cat), 1))
        out_bytes[0] = len(cat)
        return ctypes.addressof(keep["buf"])

    cb = hostharness.EXCHANGE_CB(exchange)
    gcb = hostharness.GATHER_CB(gather)
    cfg = {"vocab_size": int(vocab), "unk_id": int(unk), "character_coverage": float(cov), "min_pair_freq": int(mpf)}
    sharded = os.environ.get("SHARDED_LOAD") == "1"
    if sharded:
        h = lib.hh_open_sharded(corpus.encode(), cfg["vocab_size"], cfg["unk_id"], cfg["character_coverage"],
                                cfg["min_pair_freq"], rank, world, gcb, None)
        assert h, corpus
    else:
        h = hostharness.open_case(lib, corpus, cfg, layout, rank, world)
        lib.hh_set_exchange(h, cb, gcb, None)
    spec = (ctypes.c_uint64 * 2)()
    lib.hh_spec(h, speculate, spec)
    lib.hh_set_chain(h, chain)
    tiles = lib.hh_num_tiles(h)
    trace = os.path.join(outdir, f"trace_r{rank}.txt")
    merges = lib.hh_train(h, trace.encode())
    lib.hh_save(h, os.path.join(outdir, "mr.model").encode(), os.path.join(outdir, "mr.vocab").encode(),
                1 if rank == 0 else 0)
    with open(os.path.join(outdir, f"info_r{rank}.txt"), "w") as f:
        lib.hh_spec(h, -1, spec)
        f.write(f"{merges} {tiles} {spec[0]} {spec[1]}" +
                (f" {hostharness.table_fingerprint(lib, h)}" if sharded else "") + "\n")
    lib.hh_close(h)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
