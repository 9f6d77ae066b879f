"""Shared fixtures.  `-m "not gpu"` runs here (no GPU); `-m gpu` runs on an MI355X box."""
from __future__ import annotations

import gzip
import json
import os
import subprocess
import sys

import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(TESTS)
PKG = os.path.join(REPO, "shredword-trainer_amd")
GOLDEN = os.path.join(TESTS, "golden")
ORACLE = os.path.join(REPO, "oracle")
for p in (TESTS, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import corpora  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden_cases():
    return sorted(d for d in os.listdir(GOLDEN) if os.path.isfile(os.path.join(GOLDEN, d, "case.json")))


def load_case(name):
    d = os.path.join(GOLDEN, name)
    with open(os.path.join(d, "case.json")) as f:
        case = json.load(f)
    with open(os.path.join(d, "model.bin"), "rb") as f:
        case["model_bytes"] = f.read()
    with open(os.path.join(d, "vocab.txt"), "rb") as f:
        case["vocab_bytes"] = f.read()
    with gzip.open(os.path.join(d, "trace.txt.gz"), "rt") as f:
        case["trace"] = f.read()
    return case


def build_corpus(recipe, path):
    kind = recipe["kind"]
    if kind == "synthetic":
        corpora.gen_synthetic(path, recipe["bytes"], recipe["seed"], recipe["script"])
    elif kind == "adversarial":
        corpora.write_adversarial(path, recipe["seed"])
    elif kind == "small":
        corpora.write_small_corpus(path)
    else:
        raise ValueError(kind)


@pytest.fixture(scope="session")
def corpus_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("corpora"))


_CORPUS_CACHE = {}


@pytest.fixture(scope="session")
def case_corpus(corpus_dir):
    """Returns a function name -> (case dict, corpus path), corpora built once per session."""
    def get(name):
        case = load_case(name)
        key = json.dumps({k: v for k, v in case["corpus"].items() if k not in ("md5", "size")}, sort_keys=True)
        if key not in _CORPUS_CACHE:
            path = os.path.join(corpus_dir, f"corpus_{len(_CORPUS_CACHE)}.txt")
            build_corpus(case["corpus"], path)
            assert corpora.md5_file(path) == case["corpus"]["md5"], f"generator drift for {name}"
            _CORPUS_CACHE[key] = path
        return case, _CORPUS_CACHE[key]
    return get


SEQ = os.path.join(GOLDEN, "seq")


def seq_cases():
    """The stateful call-sequence goldens (tests/golden/seq, make_golden.py SEQ_CASES)."""
    return sorted(d for d in os.listdir(SEQ) if os.path.isfile(os.path.join(SEQ, d, "case.json")))


def load_seq_case(name):
    d = os.path.join(SEQ, name)
    with open(os.path.join(d, "case.json")) as f:
        case = json.load(f)
    case["outputs"] = []
    for i in range(len(case["saves"])):
        with open(os.path.join(d, f"model{i}.bin"), "rb") as fm, open(os.path.join(d, f"vocab{i}.txt"), "rb") as fv:
            case["outputs"].append((fm.read(), fv.read()))
    with gzip.open(os.path.join(d, "trace.txt.gz"), "rt") as f:
        case["trace"] = f.read()
    return case


@pytest.fixture(scope="session")
def seq_case(corpus_dir):
    """name -> (case, ops) with every load op's corpus built (md5-checked) and named by path."""
    def get(name):
        case = load_seq_case(name)
        ops = []
        for op in case["script"]:
            if op[0] == "load":
                recipe = op[1]
                key = json.dumps({k: v for k, v in recipe.items() if k not in ("md5", "size")}, sort_keys=True)
                if key not in _CORPUS_CACHE:
                    path = os.path.join(corpus_dir, f"corpus_{len(_CORPUS_CACHE)}.txt")
                    build_corpus(recipe, path)
                    assert corpora.md5_file(path) == recipe["md5"], f"generator drift for {name}"
                    _CORPUS_CACHE[key] = path
                ops.append(("load", _CORPUS_CACHE[key]))
            else:
                ops.append(tuple(op))
        return case, ops
    return get


@pytest.fixture(scope="session")
def oracle_bin():
    subprocess.run(["make", "-s", "-C", ORACLE, "port"], check=True)
    return os.path.join(ORACLE, "_build", "bpe_oracle")


def progress(msg):
    """A progress line for long GPU tests: appended to $SHREDWORD_HEARTBEAT_FILE when set (pytest
    captures fds 1 and 2, so a harness that kills silent commands watches a file instead)."""
    path = os.environ.get("SHREDWORD_HEARTBEAT_FILE")
    if path:
        with open(path, "a") as f:
            f.write(msg + "\n")


@pytest.fixture(autouse=True)
def _heartbeat(request):
    """Long GPU tests (full-size corpora: generation, load, training) write a progress line every
    30 s (see progress())."""
    if request.node.get_closest_marker("gpu") is None or not os.environ.get("SHREDWORD_HEARTBEAT_FILE"):
        yield
        return
    import threading
    import time
    done = threading.Event()
    t0 = time.time()

    def beat():
        while not done.wait(30.0):
            progress(f"[heartbeat] {request.node.nodeid} running {time.time() - t0:.0f} s")

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        yield
    finally:
        done.set()
        th.join(timeout=1.0)
