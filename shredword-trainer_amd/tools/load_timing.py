import os, sys, time
sys.path.insert(0, "shredword-trainer_amd")
from shredword.trainer import BPETrainer
p = sys.argv[1]
for gpu in (1, 0, 1):
    t = BPETrainer(vocab_size=8192, min_pair_freq=2000)
    t.set_option("log", 0)
    t.set_option("gpu_load", gpu)
    t0 = time.time(); t.load_corpus(p); dt = time.time() - t0
    print("gpu_load", gpu, "load_s %.3f" % dt, t.stats()["load_on_gpu"], flush=True)
    t.destroy()
