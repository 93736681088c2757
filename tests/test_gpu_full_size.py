"""BASELINE configs[3] and configs[4] at their full sizes on one GPU, pinned to
the oracle (tests/golden/full_size.json, written by tests/golden/gen_full.py
with the fast C oracle oracle/hm_oracle_fast.c, itself checked against
oracle/hm_oracle.c by tests/test_oracle_fast.py).

* config 4: [0, 2^40) of "bradfitz" as the shards of hm_partition for 8 GPUs
  (and 2 and 4), each through hm_scan_checked: per shard (min, sum of keys,
  count) equals the oracle's pieces merged, the shard counts add up to 2^40,
  and the shard minima merge to the oracle's whole-range answer, which one
  whole-range hm_scan also returns.  Windows around every shard edge match
  the independent generic kernel.
* config 5: every 20-digit miner chunk the reference server cuts from
  [2^64-1-2^34, 2^64-2] (server.go:165-205) for the four SURVEY messages,
  through hm_scan_checked, against the oracle's per-chunk triple.
"""
import json
import os

import pytest

from distributed_bitcoinminer_amd import _lib

pytestmark = pytest.mark.gpu
MAX = (1 << 64) - 1
_FIX = os.path.join(os.path.dirname(__file__), "golden", "full_size.json")


def _fixture():
    with open(_FIX) as f:
        return json.load(f)


def _triple(d):
    return (int(d["hash"]), int(d["nonce"])), int(d["sum"]), int(d["count"])


def _merge(triples):
    best = min((t[0] for t in triples), default=(MAX, 0))
    return best, sum(t[1] for t in triples) & MAX, sum(t[2] for t in triples)


def _generic(ctx, m, lo, hi):
    ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 1)
    try:
        return ctx.scan_checked(m, lo, hi)
    finally:
        ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 0)


def _shard_expect(pieces, lo, hi):
    """Oracle triple of [lo, hi] from the fixture's pieces (must align)."""
    inside = [p for p in pieces if int(p["lo"]) >= lo and int(p["hi"]) <= hi]
    assert inside and int(inside[0]["lo"]) == lo and int(inside[-1]["hi"]) == hi, \
        "shard does not align with the fixture's pieces: regenerate tests/golden/full_size.json"
    return _merge([_triple(p) for p in inside])


@pytest.mark.timeout(600)
def test_config4_full_range_shards(ctx):
    fx = _fixture()
    assert "cfg4" in fx, "tests/golden/full_size.json lacks cfg4 (run tests/golden/gen_full.py)"
    c4 = fx["cfg4"]
    m, lo, hi = bytes.fromhex(c4["msg_hex"]), int(c4["lo"]), int(c4["hi"])
    assert (lo, hi) == (0, (1 << 40) - 1)
    whole = _triple(c4["whole"])
    assert whole[2] == 1 << 40
    shards = _lib.partition(m, lo, hi, 8)
    got = []
    for a, b in shards:
        t = ctx.scan_checked(m, a, b)
        assert t == _shard_expect(c4["pieces"], a, b), (a, b)
        assert t[2] == b - a + 1
        got.append(t)
    assert _merge(got) == whole
    # the production kernels over the whole range
    assert ctx.scan(m, lo, hi) == whole[0]
    assert _lib.host_hash(m, whole[0][1]) == whole[0][0]
    # the 2- and 4-GPU cuts are unions of the 8-GPU pieces too
    for n in (2, 4):
        for a, b in _lib.partition(m, lo, hi, n):
            _shard_expect(c4["pieces"], a, b)
    # every internal 8-shard edge: fast kernels vs the generic kernel
    for (_, b), _ in zip(shards, shards[1:]):
        w = (b - 2_000_000, b + 2_000_001)
        assert ctx.scan_checked(m, *w) == _generic(ctx, m, *w), w


def test_config5_chunks_checked(ctx):
    fx = _fixture()
    for case in fx["cfg5"]:
        m = bytes.fromhex(case["msg_hex"])
        for ch in case["chunks"]:
            a, b = int(ch["lo"]), int(ch["hi"])
            if b == MAX:          # the miner's Upper+1 wraps (miner.go:52): nothing scanned
                assert _triple(ch) == ((MAX, 0), 0, 0)
                continue
            assert ctx.scan_checked(m, a, b) == _triple(ch), (case["name"], a, b)


def test_medium_random_fixtures(ctx):
    """153 random ranges of 10^6..2*10^8 nonces (every message length 0..130,
    digit-count changes, next to 2^64-1; tests/golden/gen_medium.py) through
    hm_scan_checked and hm_scan against the oracle's triples."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "medium.json")) as f:
        cases = json.load(f)["cases"]
    assert len(cases) >= 150
    for c in cases:
        m, lo, hi = bytes.fromhex(c["msg_hex"]), int(c["lo"]), int(c["hi"])
        exp = _triple(c)
        assert ctx.scan_checked(m, lo, hi) == exp, c["name"]
        assert ctx.scan(m, lo, hi) == exp[0], c["name"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["bradfitz", "long120"])
def test_weak_scaling_rank_shards(ctx, name):
    """bench.py's weak-scaling work at N = 8 (configs[1] / configs[2]): rank
    r scans [r*2^32, (r+1)*2^32).  Every rank's shard through hm_scan_checked
    equals the oracle's piece, so each rank's answer of the driver's 8-GPU run
    and their merge (what the all-gather produces) are pinned."""
    fx = _fixture()
    w = next(x for x in fx["weak"] if x["name"] == name)
    m = bytes.fromhex(w["msg_hex"])
    got = []
    for r, p in enumerate(w["pieces"]):
        lo, hi = r << 32, ((r + 1) << 32) - 1
        assert (int(p["lo"]), int(p["hi"])) == (lo, hi)
        t = ctx.scan_checked(m, lo, hi)
        assert t == _triple(p), (name, r)
        got.append(t)
    assert _merge(got)[2] == 8 << 32
