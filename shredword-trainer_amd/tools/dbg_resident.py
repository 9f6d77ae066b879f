import os, sys, tempfile
sys.path.insert(0, "shredword-trainer_amd"); sys.path.insert(0, "tests")
import corpora
from shredword.trainer import BPETrainer
d = tempfile.mkdtemp()
c = os.path.join(d, "c.txt")
corpora.write_small_corpus(c)
t = BPETrainer(vocab_size=300, min_pair_freq=2)
t.set_option("log", 0)
t.load_corpus(c)
print("merges", t.train(), t.stats()["resident_launches"], flush=True)
