"""Encoder timing on one corpus: python enc_bench.py prepare CORPUS BYTES DIR  (generate + train + save)
                                   python enc_bench.py run CORPUS DIR [reps]     (SHREDWORD_LIB picks the build)"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
mode, corpus = sys.argv[1], sys.argv[2]
if mode == "prepare":
    nbytes, d = int(sys.argv[3]), sys.argv[4]
    os.makedirs(d, exist_ok=True)
    subprocess.run([os.path.join(HERE, "..", "bin", "gen_corpus"), "--bytes", str(nbytes), "--seed", "2",
                    "--script", "utf8", "--out", corpus], check=True)
    from shredword.trainer import BPETrainer
    t = BPETrainer(vocab_size=8192, min_pair_freq=2000)
    t.set_option("log", 0)
    t.load_corpus(corpus)
    t._train(t.trainer)
    t._save(t.trainer, os.path.join(d, "m.model").encode(), os.path.join(d, "m.vocab").encode())
    t.destroy()
else:
    d = sys.argv[3]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    import torch
    from shredword.encoder import BPEEncoder
    enc = BPEEncoder(os.path.join(d, "m.model"), os.path.join(d, "m.vocab"), unk_id=0)
    text = torch.from_numpy(np.fromfile(corpus, dtype=np.uint8)).cuda()
    out = torch.empty(text.numel(), dtype=torch.int32, device="cuda")
    ids, _ = enc.encode_device(text, out)
    ms = sorted(enc.encode_device(text, out)[1] for _ in range(reps))
    print(os.environ.get("SHREDWORD_LIB", "default"), "ids", ids.numel(), "ms", ms[len(ms) // 2],
          "GB/s", text.numel() / ms[len(ms) // 2] / 1e6, flush=True)
    enc.destroy()
