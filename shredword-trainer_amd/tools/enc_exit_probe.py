"""Diagnostic: which call sequence before torch's first CUDA use makes the process abort at exit."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
v = sys.argv[1]
from shredword.cbase import lib

merges = np.array([[97, 97, 256], [256, 97, 257], [98, 99, 258]], np.int32)
if v == "H":
    lib.shred_device_count()
elif v == "G":
    from shredword.trainer import BPETrainer
    d = tempfile.mkdtemp()
    p = os.path.join(d, "c.txt")
    open(p, "w").write("ab abc aab bca " * 2000)
    t = BPETrainer(vocab_size=270, min_pair_freq=2)
    t.set_option("log", 0)
    t.load_corpus(p)
    t.train()
    t.destroy()
elif v in ("D", "F", "I"):
    from shredword.encoder import BPEEncoder
    e = BPEEncoder.from_merges(merges)
    if v != "I":
        e.encode(b"ab c aaa " * 100)
    e.destroy()
import torch
if v != "F":
    t = torch.from_numpy(np.frombuffer(b"xaaa bc " * 1000, np.uint8).copy()).cuda()
print("variant", v, "done", flush=True)
