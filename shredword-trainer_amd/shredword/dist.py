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
    default gloo group) is used when the collective on `group` raises (state["fell_back"] = the
    error, when a dict is given).  The returned callback
    keeps its last result alive until its next call, as the C ABI requires."""
    import torch.distributed as dist

    from .cbase import GATHER_FN
    keep = {}

    def gather(_ctx, send, nbytes, out_bytes):
        # An exception must not cross the C boundary (ctypes would print it and return 0 bytes,
        # which reads as "no words"): report a NULL result and the library fails load_corpus.
        try:
            mine = ctypes.string_at(send, nbytes) if nbytes else b""
            try:
                if keep.get("fell_back"):
                    raise RuntimeError("an earlier gather on this group raised")
                parts = [None] * dist.get_world_size(group)
                dist.all_gather_object(parts, mine, group=group)
            except Exception as e:  # noqa: BLE001 (e.g. the nccl group failed to come up on every rank)
                if fallback is None:
                    raise
                if not keep.get("fell_back"):
                    import sys
                    print(f"[WARNING]\t host_load_gather: {e!r}; gathering over the fallback group", file=sys.stderr)
                    keep["fell_back"] = True
                    if state is not None:
                        state["fell_back"] = str(e) or repr(e)
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
