"""The drop-in boundary without a GPU: libtrainer.so loads, exports every symbol that
include/shredword_bpe.h and include/shredword_encode.h declare (the reference's 8 BPE + 13 Unigram symbols bound by
cbase.py:50-71, plus extensions), keeps the reference BPEConfig layout, and fails loudly — never
silently on the CPU — when no GPU is present."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO

HEADERS = [os.path.join(REPO, "include", h) for h in ("shredword_bpe.h", "shredword_encode.h")]
REFERENCE_BPE = ["create_trainer", "bpe_trainer_destroy", "bpe_init", "bpe_count_bigrams", "bpe_load_corpus",
                 "bpe_merge_batch", "bpe_train", "bpe_save"]
REFERENCE_UNIGRAM = ["trainerCreate", "trainerDestroy", "addTextToTrainer", "preprocessTexts",
                     "extractInitialSubwords", "computeLoss", "computeTokenLoss", "pruneVocabStep",
                     "updateTokenScores", "trainUnigram", "getVocab", "saveVocab", "loadVocab"]


def declared_functions():
    text = "".join(open(h).read() for h in HEADERS)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{}]*\)\s*;", text)
    return sorted(set(n for n in names if n not in ("if", "while", "sizeof")))


def test_library_exports_every_declared_symbol():
    from shredword.cbase import lib, _lib_path
    assert os.path.dirname(_lib_path) == os.path.join(PKG, "shredword")
    names = declared_functions()
    for n in REFERENCE_BPE + REFERENCE_UNIGRAM:
        assert n in names, f"{n} missing from the header"
    for n in names:
        assert hasattr(lib, n), f"libtrainer.so does not export {n}"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib_path], capture_output=True, text=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    assert set(names) <= exported


def test_bpeconfig_layout_matches_reference():
    from shredword.cbase import BPEConfig
    assert ctypes.sizeof(BPEConfig) == 24
    assert [getattr(BPEConfig, f).offset for f in
            ("target_vocab_size", "unk_id", "character_coverage", "min_pair_freq")] == [0, 8, 12, 16]


def test_rejects_missing_corpus(tmp_path):
    """reference test/test_bpe.py:67-70"""
    from shredword.trainer import BPETrainer
    t = BPETrainer(vocab_size=10)
    with pytest.raises(IOError):
        t.load_corpus(str(tmp_path / "missing.txt"))
    t.destroy()
    t.destroy()  # idempotent


def test_context_manager_and_defaults():
    from shredword.trainer import BPETrainer
    with BPETrainer() as t:
        assert t.config.target_vocab_size == 8192 and t.config.unk_id == 0
        assert abs(t.config.character_coverage - 0.995) < 1e-6 and t.config.min_pair_freq == 2000
    assert t.trainer is None


def test_unigram_stub_fails_loudly():
    from shredword.trainer import UnigramTrainer
    with pytest.raises(RuntimeError):
        UnigramTrainer()


def test_train_without_gpu_fails_loudly(tmp_path):
    from shredword.cbase import lib
    from shredword.trainer import BPETrainer
    if lib.shred_device_count() > 0:
        pytest.skip("a GPU is present")
    p = tmp_path / "c.txt"
    p.write_text("ab ab ab abab\n" * 50)
    t = BPETrainer(vocab_size=300, min_pair_freq=2)
    t.load_corpus(str(p))  # host-side load works without a GPU
    with pytest.raises(RuntimeError):
        t.train()
    t.destroy()


CLI = os.path.join(PKG, "bin", "trainer")


def test_cli_usage_and_argument_errors(tmp_path):
    r = subprocess.run([CLI], capture_output=True, text=True)
    assert r.returncode == 0 and "Usage:" in r.stdout
    r = subprocess.run([CLI, "input=x", "model_type=bpe"], capture_output=True, text=True)
    assert r.returncode == 1 and "Missing required arguments" in r.stderr
    r = subprocess.run([CLI, "input=x", "model_type=wordpiece", "output_model=m", "output_vocab=v"],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "Invalid model_type" in r.stderr
    r = subprocess.run([CLI, f"input={tmp_path / 'missing.txt'}", "model_type=bpe", f"output_model={tmp_path}/m",
                        f"output_vocab={tmp_path}/v", "ignored", "unknown_key=1"], capture_output=True, text=True)
    assert r.returncode == 255 and "Failed to load corpus" in r.stderr


def test_encoder_without_gpu_fails_loudly(tmp_path):
    from shredword.cbase import lib
    from shredword.encoder import BPEEncoder
    if lib.shred_device_count() > 0:
        pytest.skip("a GPU is present")
    model = tmp_path / "m.model"
    model.write_bytes(b"")
    with pytest.raises(RuntimeError):
        BPEEncoder(str(model))
    with pytest.raises(RuntimeError):
        BPEEncoder.from_merges([[97, 98, 256]])


def test_failed_load_gather_fails_load_corpus(tmp_path):
    """A sharded load whose word-list all-gather fails (here: host_load_gather with no process
    group, so torch.distributed raises inside the callback) makes load_corpus fail instead of
    training every rank on a partial table."""
    import corpora
    from shredword import dist as sdist
    from shredword.trainer import BPETrainer
    corpus = str(tmp_path / "c.txt")
    corpora.write_small_corpus(corpus)
    t = BPETrainer(vocab_size=300, min_pair_freq=2)
    t.set_option("log", 0)
    t.set_load_gather(0, 2, sdist.host_load_gather())
    with pytest.raises(IOError):
        t.load_corpus(corpus)
    # a gather that returns NULL outright
    from shredword.cbase import GATHER_FN
    t.set_load_gather(1, 2, GATHER_FN(lambda ctx, send, n, out: None))
    with pytest.raises(IOError):
        t.load_corpus(corpus)
    # a gather is not usable with the stream layout: an error, not a silent whole-file load
    t.set_load_gather(0, 2, GATHER_FN(lambda ctx, send, n, out: None))
    t.set_option("layout", "stream")
    with pytest.raises(IOError):
        t.load_corpus(corpus)
    t.destroy()


def test_call_sequence_before_any_load(tmp_path):
    """The reference's trainer with no corpus (zero-initialised): a count adds nothing, a batch
    finds an empty heap, a train performs no merge, a save writes the 256 byte tokens -- no GPU
    is needed for any of that."""
    from shredword.cbase import lib
    from shredword.trainer import BPETrainer
    t = BPETrainer(vocab_size=300, min_pair_freq=2)
    t.set_option("log", 0)
    lib.bpe_count_bigrams(t.trainer)
    lib.bpe_init(t.trainer)
    assert lib.bpe_merge_batch(t.trainer, 5) == 0
    assert lib.bpe_train(t.trainer) == 0
    m, v = str(tmp_path / "e.model"), str(tmp_path / "e.vocab")
    t.save(m, v)
    t.destroy()
    assert os.path.getsize(m) == 0
    assert open(v, "rb").read().count(b"\n") == 257  # token 10 is itself a newline
