"""Multi-GPU bootstrap: one process per MI355X, RCCL over xGMI (include/shredword_bpe.h).

``init_from_env()`` reads RANK / WORLD_SIZE / LOCAL_RANK (torchrun), has rank 0 create the RCCL
unique id, broadcasts it with torch.distributed (already initialised by the caller, any backend)
and initialises the library's communicator.  Trainers created afterwards shard the word table.
"""
import ctypes
import os

from .cbase import lib


def init_from_env(device=None):
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0")) if device is None else int(device)
    if world <= 1:
        return 0
    buf = ctypes.create_string_buffer(512)
    uid = [None]
    if rank == 0:
        n = lib.shred_dist_unique_id(buf, 512)
        if n <= 0:
            raise RuntimeError("shred_dist_unique_id failed")
        uid[0] = bytes(buf.raw[:n])
    dist.broadcast_object_list(uid, src=0)
    raw = uid[0]
    rc = lib.shred_dist_init(rank, world, ctypes.c_char_p(raw), len(raw), local)
    if rc != 0:
        raise RuntimeError(f"shred_dist_init failed on rank {rank}")
    return world


def finalize():
    lib.shred_dist_finalize()


def host_load_gather(group=None, fallback=None, state=None):
    """A shred_gather_fn over torch.distributed (BPETrainer.set_load_gather): the sharded load's
    word-list all-gather on `group` -- gloo when ranks share a GPU, an nccl group (torch's RCCL over
    xGMI) when each rank has its own, the bench's default for replicate; `fallback` (e.g. the
    default gloo group) is used when the collective on `group` raises on ANY rank: after every
    attempt the ranks agree over `fallback` (all_reduce MAX of a failure flag) and fall back all
    together, for the rest of the load (state["fell_back"] = the error, when a dict is given).
    Before the first attempt the ranks also agree over `fallback` on whether `group` came up on
    every rank, so a rank whose group is missing never leaves the others blocked inside its
    collective.  Not covered: a collective on `group` that hangs after it started on every rank
    (that waits for the process group's own timeout).  The returned callback
    keeps its last result alive until its next call, as the C ABI requires."""
    import torch.distributed as dist

    from .cbase import GATHER_FN
    keep = {}

    def agree_failed(failed):
        """Every rank's verdict on the attempt, over the fallback group: the gather falls back only
        all together (all_gather_object is two collectives; a rank that fell back alone would wait in
        a gloo gather the others never join)."""
        import torch
        flag = torch.tensor([1 if failed else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=fallback)
        return bool(flag.item())

    def gather(_ctx, send, nbytes, out_bytes):
        # An exception must not cross the C boundary (ctypes would print it and return 0 bytes,
        # which reads as "no words"): report a NULL result and the library fails load_corpus.
        try:
            mine = ctypes.string_at(send, nbytes) if nbytes else b""
            parts = None
            if fallback is not None and "checked" not in keep:
                keep["checked"] = True
                try:  # the group exists here and spans the same ranks as the fallback
                    up = dist.get_world_size(group) == dist.get_world_size(fallback)
                except Exception:  # noqa: BLE001
                    up = False
                if agree_failed(not up):
                    import sys
                    why = "the gather's group did not come up on every rank"
                    print(f"[WARNING]\t host_load_gather: {why}; every rank gathers over the fallback group",
                          file=sys.stderr)
                    keep["fell_back"] = True
                    if state is not None:
                        state["fell_back"] = why
            if not keep.get("fell_back"):
                err = None
                try:
                    parts = [None] * dist.get_world_size(group)
                    dist.all_gather_object(parts, mine, group=group)
                except Exception as e:  # noqa: BLE001 (e.g. the nccl group failed to come up)
                    if fallback is None:
                        raise
                    err = e
                if fallback is not None and agree_failed(err is not None):
                    import sys
                    why = (str(err) or repr(err)) if err is not None else "the gather raised on another rank"
                    print(f"[WARNING]\t host_load_gather: {why}; every rank gathers over the fallback group",
                          file=sys.stderr)
                    keep["fell_back"] = True
                    if state is not None:
                        state["fell_back"] = why
            if keep.get("fell_back"):
                parts = [None] * dist.get_world_size(fallback)
                dist.all_gather_object(parts, mine, group=fallback)
            blob = b"".join(parts)
            keep["buf"] = ctypes.create_string_buffer(blob, max(1, len(blob)))
            out_bytes[0] = len(blob)
            return ctypes.addressof(keep["buf"])
        except BaseException as e:  # noqa: BLE001 (reported, then turned into the C error)
            import sys
            print(f"[ERROR]\t host_load_gather: {e!r}", file=sys.stderr)
            keep.pop("buf", None)
            out_bytes[0] = 0
            return None

    return GATHER_FN(gather)
