"""tiebreak=device on one golden case, against the oracle's rule: prints the first differing trace
line, the host-phase / device merge counts and the verify result (debug aid for the GPU box).

    python shredword-trainer_amd/tools/tiebreak_debug.py ascii1m_unk7_cov09 [verify_every]
"""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import conftest
    name = sys.argv[1]
    every = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    case = conftest.load_case(name)
    tmp = tempfile.mkdtemp()
    corpus = os.path.join(tmp, "corpus.txt")
    conftest.build_corpus(case["corpus"], corpus)
    cfg = case["config"]
    from shredword.trainer import BPETrainer
    t = BPETrainer(vocab_size=cfg["vocab_size"], unk_id=cfg["unk_id"], character_coverage=cfg["character_coverage"],
                   min_pair_freq=cfg["min_pair_freq"])
    t.set_option("log", 0)
    tr = os.path.join(tmp, "d.trace")
    t.set_option("trace", tr)
    t.set_option("tiebreak", "device")
    if every:
        t.set_option("verify_argmax", every)
    t.load_corpus(corpus)
    n = t._train(t.trainer)
    st = t.stats()
    t.destroy()
    print(f"{name}: {n} merges; host phase {st['sel_host_merges']}, device {st['sel_merges']}, launches "
          f"{st['sel_launches']}, rebuilds {st['sel_rebuilds']}, verify {st['verify_checks']}/{st['verify_failures']}",
          flush=True)
    ob = os.path.join(REPO, "oracle", "_build", "bpe_oracle")
    ot = os.path.join(tmp, "o.trace")
    subprocess.run([ob, corpus, str(cfg["vocab_size"]), str(cfg["unk_id"]), repr(cfg["character_coverage"]),
                    str(cfg["min_pair_freq"]), os.path.join(tmp, "o.model"), os.path.join(tmp, "o.vocab"),
                    "--trace", ot, "--tiebreak-device", "0"], check=True, stderr=subprocess.DEVNULL)
    a = [ln for ln in open(tr).read().splitlines() if ln.startswith("M ")]
    b = [ln for ln in open(ot).read().splitlines() if ln.startswith("M ")]
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            print(f"first difference at merge {i}: device '{x}' oracle '{y}'")
            print("  context device:", a[max(0, i - 2):i + 3])
            print("  context oracle:", b[max(0, i - 2):i + 3])
            break
    else:
        print(f"traces agree on {min(len(a), len(b))} merges; lengths {len(a)} / {len(b)}")


if __name__ == "__main__":
    main()
