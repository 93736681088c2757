"""The fast oracle (oracle/hm_oracle_fast.c: SHA extensions, midstate, ASCII
digit increments) against the plain one (oracle/hm_oracle.c) and the golden
fixtures.  The fast oracle only generates tests/golden/full_size.json in the
build container, so it must agree with the plain oracle on every layout
the full-size fixtures use: every message length across the 55/56/64-byte
padding boundaries, every digit-count change, and 2^64-1."""
import random

import pytest

from oracle import oracle as O

MAX = (1 << 64) - 1

pytestmark = pytest.mark.skipif(not O.fast_available(), reason="CPU lacks the SHA extensions")


def test_fast_vs_plain_layouts():
    rng = random.Random(20261016)
    for L in list(range(0, 131, 3)) + [44, 45, 54, 55, 56, 62, 63, 64, 118, 119, 120, 127, 128]:
        m = bytes(rng.randrange(256) for _ in range(L))
        d = rng.randrange(1, 21)
        c = 10 ** (d - 1) if d > 1 else 0
        for lo, hi in ((c, c + 1500), (max(0, c - 700), c + 700), (MAX - 900, MAX), (7, 7), (9, 8)):
            assert O.fast_scan_sum(m, lo, hi, threads=3) == O.c_scan_sum(m, lo, hi, threads=3), \
                (L, lo, hi)


def test_fast_vs_golden(golden):
    for case in golden["scan_kats"]:
        if "sum" not in case or int(case["hi"]) - int(case["lo"]) > 3_000_000:
            continue
        m = bytes.fromhex(case["msg_hex"])
        lo, hi = int(case["lo"]), int(case["hi"])
        exp = ((int(case["hash"]), int(case["nonce"])), int(case["sum"]), int(case["count"]))
        assert O.fast_scan_sum(m, lo, hi, threads=4) == exp, case["name"]


def test_fast_chunking_and_threads():
    """Chunk edges of the work queue (2^22 nonces) and thread counts."""
    m = b"jonny greenwood"
    lo, hi = (1 << 22) * 3 - 5, (1 << 22) * 5 + 17
    exp = O.c_scan_sum(m, lo, hi, threads=8)
    for th in (1, 2, 7):
        assert O.fast_scan_sum(m, lo, hi, threads=th) == exp


def test_fast_matches_large_fixture_slice():
    """A 2^24 slice of config 2's fixture range, both oracles."""
    lo, hi = 4_000_000_000, 4_000_000_000 + (1 << 24)
    assert O.fast_scan_sum(b"bradfitz", lo, hi) == O.c_scan_sum(b"bradfitz", lo, hi, threads=8)


def test_medium_fixtures_agree_with_plain_oracle():
    """The smallest cases of tests/golden/medium.json (written by the fast
    oracle) recomputed by the plain oracle."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "medium.json")) as f:
        cases = json.load(f)["cases"]
    small = sorted(cases, key=lambda c: int(c["count"]) * (1 + len(c["msg_hex"]) // 110))[:8]
    for c in small:
        m, lo, hi = bytes.fromhex(c["msg_hex"]), int(c["lo"]), int(c["hi"])
        exp = ((int(c["hash"]), int(c["nonce"])), int(c["sum"]), int(c["count"]))
        assert O.c_scan_sum(m, lo, hi, threads=8) == exp, c["name"]


def test_full_size_fixtures_agree_at_2p32():
    """Both oracles at the full 2^32 of configs[1] and configs[2]: the first
    weak-scaling piece of tests/golden/full_size.json (fast oracle) equals
    tests/golden/large.json (plain oracle, 8 threads) -- min, sum of all
    2^32 keys and count."""
    import json
    import os
    gold = os.path.join(os.path.dirname(__file__), "golden")
    with open(os.path.join(gold, "large.json")) as f:
        large = {c["msg_hex"]: c for c in json.load(f)}
    with open(os.path.join(gold, "full_size.json")) as f:
        weak = json.load(f)["weak"]
    assert len(weak) == 2
    for w in weak:
        p, c = w["pieces"][0], large[w["msg_hex"]]
        assert (p["lo"], p["hi"]) == (c["lo"], c["hi"]) == ("0", str(2**32 - 1))
        for k in ("hash", "nonce", "sum", "count"):
            assert p[k] == c[k], (w["name"], k)


def test_fast_oracle_long_messages(oracle_mod):
    """The fast oracle's midstate over many constant blocks (the long-message
    GPU tests' checker) against the per-nonce oracle, lengths up to 64 KiB."""
    import random
    if not oracle_mod.fast_available():
        import pytest
        pytest.skip("no SHA extensions on this host")
    for L in (255, 256, 1983, 4096, 65537):
        rng = random.Random(L)
        m = bytes(rng.randrange(256) for _ in range(L))
        for lo in (10**9 - 300, (1 << 64) - 400):
            hi = min((1 << 64) - 1, lo + 399)
            assert oracle_mod.fast_scan_sum(m, lo, hi, threads=2) == \
                oracle_mod.c_scan_sum(m, lo, hi), (L, lo)
