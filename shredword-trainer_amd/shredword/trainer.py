"""BPETrainer — the reference's Python surface (shredword/trainer.py:5-40) on the MI355X trainer.

Same constructor defaults, method names, argument meaning and errors as the reference:
``load_corpus`` raises IOError for a missing file or a failed load, ``train`` returns the merge
count (RuntimeError if negative) and prints ``Training completed: N merges performed.``,
``save`` creates parent directories, ``destroy`` is idempotent and runs from ``__exit__`` and
``__del__``.  Extensions: ``set_option``, ``reset``, ``stats``, ``tokens``.
"""
import ctypes
import os

from .cbase import BPEConfig, ShredStats, lib


class BPETrainer:
    def __init__(self, vocab_size=8192, unk_id=0, character_coverage=0.995, min_pair_freq=2000):
        self.config = BPEConfig(target_vocab_size=vocab_size, unk_id=unk_id,
                                character_coverage=character_coverage, min_pair_freq=min_pair_freq)
        self.trainer = lib.create_trainer(ctypes.byref(self.config))
        if not self.trainer:
            raise RuntimeError("Failed to create BPE trainer")
        self._load_corpus, self._train, self._save, self._destroy_fn = (
            lib.bpe_load_corpus, lib.bpe_train, lib.bpe_save, lib.bpe_trainer_destroy)

    def load_corpus(self, path: str):
        if not os.path.exists(path):
            raise IOError(f"Corpus file does not exist: {path}")
        result = self._load_corpus(self.trainer, path.encode("utf-8"))
        if result != 0:
            raise IOError(f"Failed to load corpus from {path} (code {int(result)})")

    def train(self) -> int:
        merges = self._train(self.trainer)
        if merges < 0:
            raise RuntimeError("Training failed")
        print(f"Training completed: {int(merges)} merges performed.")
        return int(merges)

    def save(self, model_path: str, vocab_path: str):
        model_dir, vocab_dir = os.path.dirname(model_path), os.path.dirname(vocab_path)
        if model_dir:
            os.makedirs(model_dir, exist_ok=True)
        if vocab_dir:
            os.makedirs(vocab_dir, exist_ok=True)
        self._save(self.trainer, model_path.encode("utf-8"), vocab_path.encode("utf-8"))
        print(f"Model saved to: {model_path}")
        print(f"Vocabulary saved to: {vocab_path}")

    # -- extensions ------------------------------------------------------------------------
    def set_option(self, key: str, value) -> None:
        if lib.shred_set_option(self.trainer, key.encode(), str(value).encode()) != 0:
            raise ValueError(f"bad option {key}={value}")

    def set_load_gather(self, rank: int, world: int, gather) -> None:
        """Later load_corpus calls count only byte range `rank` of `world` and merge every rank's
        word list through `gather` (a shred_gather_fn, e.g. shredword.dist.host_load_gather());
        the merge loop then runs on every rank (dist=replicate without RCCL)."""
        self._gather = gather  # the C side keeps the pointer: keep the callback alive
        if lib.shred_set_load_gather(self.trainer, rank, world, gather, None) != 0:
            raise ValueError(f"bad rank {rank} of {world}")

    def reset(self) -> None:
        """Restore the loaded corpus to its unmerged state (benchmark repeats)."""
        lib.shred_reset(self.trainer)

    def tokens(self):
        """The live device token stream (diagnostic): per entry a header INT32_MIN + rank, then
        its tokens, as a numpy int32 array."""
        import numpy as np
        n = lib.shred_debug_tokens(self.trainer, None, 0)
        if n < 0:
            raise RuntimeError("no device token stream")
        out = np.empty(n, dtype=np.int32)
        lib.shred_debug_tokens(self.trainer, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n)
        return out

    def index_trace(self):
        """Per-merge trace of the indexed merge loop (diagnostic, recorded while the 'timing'
        option is on): numpy uint32 array (merges, 37) of X, listed words, scanned words, changed
        words, occurrences, device ns command -> flag, lookup ns, scan ns, wave 0's stamps
        (ns after the command: pool entries loaded, first run loaded, first word merged, unused),
        device ns since the previous flag spent waiting for commands and undoing guesses, host ns
        from post to flag, then absolute clocks (low 32 bits): host post and flag seen (10 ns
        units), device command seen and wait begun (100 MHz ticks); then 16 phase stamps and counts that only
        a -DSHRED_WL_STAMPS build fills in (word_loop.hip, zeros otherwise); then the previous flag's
        release ticks and (stamps build) the device clock when the poller saw the command."""
        import numpy as np
        n = lib.shred_index_trace(self.trainer, None, 0)
        if n < 0:
            raise RuntimeError("no device")
        out = np.empty(n, dtype=np.uint32)
        lib.shred_index_trace(self.trainer, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n)
        return out.reshape(-1, 37)

    def stats(self) -> dict:
        s = ShredStats()
        lib.shred_get_stats(self.trainer, ctypes.byref(s))
        return {name: getattr(s, name) for name, _ in ShredStats._fields_}

    def destroy(self):
        if getattr(self, "trainer", None):
            try:
                self._destroy_fn(self.trainer)
            finally:
                self.trainer = None

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        self.destroy()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class UnigramTrainer:
    """Reference surface (trainer.py:43-82).  Unigram is outside this build's BPE scope: the
    native trainerCreate returns NULL, so construction raises RuntimeError as the reference
    does on that path."""

    def __init__(self, vocab_size=32000, character_coverage=0.9995, max_sentencepiece_length=16,
                 seed_size=1000000):
        self.vocab_size, self.character_coverage = vocab_size, character_coverage
        self.max_len, self.seed_size = max_sentencepiece_length, seed_size
        self.trainer = lib.trainerCreate(vocab_size, character_coverage, max_sentencepiece_length, seed_size)
        if not self.trainer:
            raise RuntimeError("Failed to create Unigram trainer")
        self.texts = []

    def destroy(self):
        if getattr(self, "trainer", None):
            try:
                lib.trainerDestroy(self.trainer)
            finally:
                self.trainer = None

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        self.destroy()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass
