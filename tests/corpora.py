"""Deterministic test corpora for the BPE path.

* Synthetic corpora come from the committed generator ``gen_corpus``;
  fixtures record the generator arguments and the corpus md5 so drift is caught.
* Adversarial corpora are built here with a seeded PRNG: runs such as
  ``aaaa…`` and ``abab…`` (the a==b greedy rule, Appendix A.5), CR/TAB delimiters, lines longer
  than the reference's 4096-byte line buffer (bpe.cpp:131-147), words longer than one device
  tile, multi-byte UTF-8, rare control bytes (coverage cut) and NUL bytes (strlen truncation).
"""
from __future__ import annotations

import hashlib
import os
import random
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "shredword-trainer_amd")
GEN = os.path.join(PKG, "bin", "gen_corpus")

SMALL_TEXTS = [  # the reference's own pytest fixture corpus (test/test_bpe.py:8-30), x100
    "The quick brown fox jumps over the lazy dog.",
    "Machine learning is a subset of artificial intelligence.",
    "Natural language processing involves computational linguistics.",
    "Deep learning models require large amounts of training data.",
    "Tokenization is an important preprocessing step in NLP.",
    "Subword tokenization helps handle out-of-vocabulary words.",
    "Byte pair encoding and SentencePiece are popular tokenization methods.",
    "Transformer models have revolutionized natural language understanding.",
    "BERT, GPT, and T5 are examples of pre-trained language models.",
    "Fine-tuning allows adapting pre-trained models to specific tasks.",
    "The attention mechanism enables models to focus on relevant parts.",
    "Positional encoding helps models understand sequence order.",
    "Multi-head attention processes different representation subspaces.",
    "Layer normalization stabilizes training in deep networks.",
    "Dropout prevents overfitting by randomly zeroing activations.",
    "Gradient descent optimizes model parameters during training.",
    "Backpropagation computes gradients for parameter updates.",
    "Cross-entropy loss is commonly used for classification tasks.",
    "Regularization techniques prevent models from memorizing training data.",
    "Evaluation metrics measure model performance on test datasets.",
]


def md5_file(path: str) -> str:
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def write_small_corpus(path: str) -> None:
    with open(path, "w", encoding="utf-8") as f:
        f.write("\n".join(SMALL_TEXTS * 100) + "\n")


def gen_synthetic(path: str, nbytes: int, seed: int, script: str) -> None:
    if not os.path.exists(GEN):
        raise FileNotFoundError(f"{GEN} missing: run __graft_entry__.build() first")
    subprocess.run([GEN, "--bytes", str(nbytes), "--seed", str(seed), "--script", script,
                    "--out", path], check=True)


def adversarial_bytes(seed: int, reps: int = 60) -> bytes:
    rnd = random.Random(seed)
    words = [
        b"a", b"aa", b"aaa", b"aaaa", b"aaaaa", b"aaaaaaa", b"aaaaaaaaaaaaaaaa",
        b"ab", b"abab", b"ababab", b"abababab", b"aabbaabb", b"abcabc", b"abba", b"baab",
        b"bbbb", b"bab", b"aab", b"abb", b"cacaca", b"the", b"then", b"there", b"other",
        "αβγ".encode(), "ααα".encode(), "привет".encode(), "日本語".encode(), "한국어".encode(),
        "naïve".encode(), "café".encode(), b"x\x01y", b"\x7f\x7f", b"z\xffz", b"q\x02",
    ]
    lines = []
    for _ in range(reps):
        k = rnd.randint(3, 14)
        parts = [rnd.choice(words) for _ in range(k)]
        seps = [rnd.choice([b" ", b" ", b" ", b"\t", b"  ", b"\r"]) for _ in range(k - 1)]
        line = parts[0]
        for s, p in zip(seps, parts[1:]):
            line += s + p
        lines.append(line + rnd.choice([b"\n", b"\r\n", b"\n"]))
    # lines far beyond the reference's 4096-byte starting line buffer
    long_line = b" ".join(rnd.choice(words) for _ in range(2500)) + b"\n"
    lines.insert(len(lines) // 3, long_line)
    lines.insert(2 * len(lines) // 3, long_line)
    # one word longer than a device tile (and than the line buffer)
    lines.append(b"ab" * 5000 + b"a" * 333 + b"\n")
    lines.append((b"a" * 4100) + b" " + (b"ba" * 2100) + b"\n")
    # NUL bytes: strlen truncation of a short line and of a line crossing the 4096-byte buffer
    lines.append(b"abab then\x00hidden words here\n")
    lines.append(b"the " * 1100 + b"\x00" + b"never seen " * 10 + b"\n")
    lines.append(b"x" * 4095 + b"\x00tail abab\n")
    body = b"".join(lines)
    return body * 3 + b"no final newline abab"


def write_adversarial(path: str, seed: int) -> None:
    with open(path, "wb") as f:
        f.write(adversarial_bytes(seed))
