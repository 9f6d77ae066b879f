"""One rank of a sharded load through the PRODUCT library (shred_set_load_gather): torch.distributed
gloo on 127.0.0.1 carries the word-list all-gather instead of RCCL.  The rank counts its byte range
of the corpus (on the GPU when one is present), the lists are merged, and then -- with TRAIN=1, on
the GPU -- the merge loop runs on every rank (dist=replicate).  Writes info_r<rank>.json (table
sizes, load on GPU) and, when trained, r<rank>.model / r<rank>.vocab.

usage: sharded_product_worker.py CORPUS VOCAB UNK COV MPF OUTDIR
"""
import json
import os
import sys

import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "shredword-trainer_amd"))


def main():
    corpus, vocab, unk, cov, mpf, outdir = sys.argv[1:7]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from shredword import dist as sdist
    from shredword.trainer import BPETrainer
    t = BPETrainer(vocab_size=int(vocab), unk_id=int(unk), character_coverage=float(cov), min_pair_freq=int(mpf))
    t.set_option("log", 0)
    if os.environ.get("TRAIN") == "1":
        t.set_option("resident", 0)  # ranks share one GPU here: the whole-chip loop would not be co-resident
    state = {}
    if os.environ.get("BROKEN_GROUP") == "1":  # a group whose gather raises on every rank: the fallback carries it
        t.set_load_gather(rank, world, sdist.host_load_gather(object(), fallback=dist.group.WORLD, state=state))
    elif os.environ.get("BROKEN_GROUP") == "last":
        # only the last rank's gather raises; the others' "succeeds" on a group without it (a
        # partial list): every rank must still fall back together and build the whole table
        alone = dist.new_group(list(range(world - 1)))
        grp = object() if rank == world - 1 else alone
        t.set_load_gather(rank, world, sdist.host_load_gather(grp, fallback=dist.group.WORLD, state=state))
    else:
        t.set_load_gather(rank, world, sdist.host_load_gather())
    t.load_corpus(corpus)
    st = t.stats()
    info = {"rank": rank, "num_words": st["num_words"], "num_symbols": st["num_symbols"],
            "num_occurrences": st["num_occurrences"], "load_on_gpu": st["load_on_gpu"],
            "fell_back": bool(state.get("fell_back"))}
    if os.environ.get("TRAIN") == "1":
        info["merges"] = t._train(t.trainer)
        t._save(t.trainer, os.path.join(outdir, f"r{rank}.model").encode(),
                os.path.join(outdir, f"r{rank}.vocab").encode())
    json.dump(info, open(os.path.join(outdir, f"info_r{rank}.json"), "w"))
    t.destroy()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
