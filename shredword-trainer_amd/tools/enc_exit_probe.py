"""Diagnostic: which encoder call sequence makes the process abort at exit (variants A-E)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
v = sys.argv[1]
if v == "C":
    import torch
    torch.zeros(1).cuda()
from shredword.encoder import BPEEncoder

merges = np.array([[97, 97, 256], [256, 97, 257], [98, 99, 258]], np.int32)
e = BPEEncoder.from_merges(merges)
sizes = [1] if v == "B" else [1, 400, 5000, 100_000, 3]
for n in sizes:
    e.encode(b"ab c " * (n // 5 + 1))
e.destroy()
if v != "E":
    import torch
    t = torch.from_numpy(np.frombuffer(b"xaaa bc " * 1000, np.uint8).copy()).cuda()
    if v != "D":
        e2 = BPEEncoder.from_merges(merges)
        ids, ms = e2.encode_device(t[1:])
        e2.destroy()
print("variant", v, "done", flush=True)
