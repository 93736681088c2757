"""hm_scan_cpu (ABI 1.7): the product's host scan, SURVEY §8(b)'s liveness
path for a miner whose GPU is missing or failed.  It must equal the
reference scan (cmu440/bitcoin/miner/miner.go:46-59 over bitcoin.Hash,
cmu440/bitcoin/hash.go:13-17) exactly: checked here against the committed
golden scans and against the C oracle (test infrastructure) on edge cases
and random ranges, with both compressions (x86 SHA extensions and portable
C) and several thread counts.  No GPU needed."""
import os
import random

import pytest

from distributed_bitcoinminer_amd import _lib

MAXU64 = (1 << 64) - 1
PATHS = ["sha", "c"]


@pytest.fixture(params=PATHS)
def path(request, monkeypatch):
    """Run the test once with each compression of hm_scan_cpu."""
    if request.param == "c":
        monkeypatch.setenv("HM_CPU_NO_SHA", "1")
    else:
        monkeypatch.delenv("HM_CPU_NO_SHA", raising=False)
    return request.param


def test_golden_scans(golden, path):
    """Every committed golden range scan (the hashlib restatement's answers)."""
    kats = golden["scan_kats"]
    if path == "c":  # the portable compression on a subset (it is ~4x slower)
        kats = [k for k in kats if int(k["hi"]) - int(k["lo"]) <= 20000]
    for k in kats:
        m = bytes.fromhex(k["msg_hex"])
        lo, hi = int(k["lo"]), int(k["hi"])
        got = _lib.scan_cpu(m, lo, hi, threads=3)
        assert got == (int(k["hash"]), int(k["nonce"])), k.get("name")


def test_config1_answer(path):
    """configs[0]'s answer, SURVEY App. B: bradfitz [0, 10^7]."""
    assert _lib.scan_cpu(b"bradfitz", 0, 10**7, threads=8) == (356393768206, 7645578)


def test_edges(oracle_mod, path):
    """Empty range, the top of the u64 range (hi = 2^64-1 is scanned, the
    Upper+1 wrap belongs to callers), single nonces, digit-count edges, the
    empty message, and messages around every tail-block boundary."""
    assert _lib.scan_cpu(b"bradfitz", 5, 4) == (MAXU64, 0)
    assert _lib.scan_cpu(b"", 7, 7) == (oracle_mod.c_hash(b"", 7), 7)
    top = (MAXU64 - 3000, MAXU64)
    assert _lib.scan_cpu(b"bradfitz", *top, threads=4) == oracle_mod.c_scan(b"bradfitz", *top)
    assert _lib.scan_cpu(b"x", MAXU64, MAXU64) == (oracle_mod.c_hash(b"x", MAXU64), MAXU64)
    for lo, hi in ((0, 9), (0, 1000), (99990, 100009), (10**9 - 3000, 10**9 + 3000),
                   (10**19 - 2000, 10**19 + 2000)):
        assert _lib.scan_cpu(b"bradfitz", lo, hi, threads=5) == \
            oracle_mod.c_scan(b"bradfitz", lo, hi), (lo, hi)
    for n in (0, 1, 44, 45, 53, 54, 55, 56, 62, 63, 64, 118, 119, 120, 127, 128, 200):
        m = bytes((0x41 + i % 26) for i in range(n))
        for lo, hi in ((0, 150), (10**9 - 40, 10**9 + 40), (MAXU64 - 40, MAXU64)):
            assert _lib.scan_cpu(m, lo, hi, threads=2) == oracle_mod.c_scan(m, lo, hi), (n, lo)


def test_thread_counts_agree(oracle_mod, path):
    """The chunk split does not change the answer (lexicographic merge)."""
    lo, hi = 999_000, 1_201_000  # crosses 6 -> 7 digits
    want = oracle_mod.c_scan(b"thom yorke", lo, hi)
    for t in (1, 2, 3, 7, 16, 64, 0):
        assert _lib.scan_cpu(b"thom yorke", lo, hi, threads=t) == want, t


def test_random_ranges(oracle_mod, path):
    """200 random (message, range) draws: lengths 0..130, any byte, ranges
    up to 3000 nonces placed near digit-count changes and anywhere in u64."""
    rng = random.Random(5005 if path == "sha" else 5006)
    for _ in range(200):
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(131)))
        if rng.random() < 0.5:
            d = rng.randrange(1, 20)
            lo = max(0, 10**d - rng.randrange(1, 2000))
        else:
            lo = rng.randrange(MAXU64)
        hi = min(MAXU64, lo + rng.randrange(3000))
        assert _lib.scan_cpu(m, lo, hi, threads=rng.choice((1, 2, 4))) == \
            oracle_mod.c_scan(m, lo, hi), (m.hex(), lo, hi)


def test_invalid_arguments():
    import ctypes
    lib = _lib.load()
    out = _lib.hm_result()
    assert lib.hm_scan_cpu(None, 3, 0, 1, 1, ctypes.byref(out)) == _lib.HM_ERR_INVALID
    assert lib.hm_scan_cpu(b"x", 1, 0, 1, 1, None) == _lib.HM_ERR_INVALID
    assert lib.hm_scan_cpu(None, 0, 0, 1, 1, ctypes.byref(out)) == _lib.HM_OK


def test_no_oracle_in_the_product():
    """The host scan is the product's own code: nothing under csrc/ or the
    Makefile names, includes or links oracle/."""
    csrc = os.path.join(os.path.dirname(_lib.LIB_PATH), "csrc")
    for n in os.listdir(csrc):
        if not os.path.isfile(os.path.join(csrc, n)):
            continue
        with open(os.path.join(csrc, n), "rb") as f:
            assert b"oracle" not in f.read(), n
