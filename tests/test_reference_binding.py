"""The reference's own, unmodified Python layer (shredword/cbase.py + trainer.py, imported from a
temporary copy — never committed) binds our libtrainer.so: every symbol it binds at import exists
with a compatible signature, and BPETrainer drives load_corpus through it.  Needs
/root/reference, so it runs in the build container only (skipped elsewhere)."""
import os
import shutil
import subprocess
import sys
import textwrap

import pytest

from conftest import PKG

REF_PKG = "/root/reference/shredword"


@pytest.mark.skipif(not os.path.isdir(REF_PKG), reason="reference not mounted")
def test_reference_cbase_binds_our_library(tmp_path):
    dst = tmp_path / "shredword"
    shutil.copytree(REF_PKG, dst, ignore=shutil.ignore_patterns("csrc", "utils", "__pycache__"))
    shutil.copy(os.path.join(PKG, "shredword", "libtrainer.so"), dst / "libtrainer.so")
    corpus = tmp_path / "c.txt"
    corpus.write_text("abab abba baab\n" * 40)
    script = textwrap.dedent(f"""
        import sys; sys.path.insert(0, {str(tmp_path)!r})
        from shredword.trainer import BPETrainer
        from shredword import cbase
        assert cbase._lib_path.endswith("libtrainer.so"), cbase._lib_path
        t = BPETrainer(vocab_size=300, min_pair_freq=2)
        t.load_corpus({str(corpus)!r})
        try:
            t.load_corpus({str(tmp_path / 'missing.txt')!r})
        except IOError:
            print("IOERROR_OK")
        t.destroy()
        print("BOUND_OK")
    """)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "BOUND_OK" in r.stdout and "IOERROR_OK" in r.stdout
