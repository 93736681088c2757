"""Coverage checksums on the GPU: hm_scan_checked vs the oracle and vs itself.

hm_scan_checked runs the checked variants of the production kernels (same
planner, tiles, lane/loop layout, guided task split, launch chunking and
multi-device shards) and returns, besides the (hash, nonce) minimum, the sum of
every key mod 2^64 and the number of nonces hashed.  A nonce skipped, hashed
twice or hashed over wrong bytes changes that pair, so these tests check that
every nonce of a range is hashed exactly once and correctly:

* against the golden fixtures (tests/golden/gen_golden.py, hashlib) and the C
  oracle (oracle/hm_oracle.c, oracle_scan_sum) at sizes the CPU finishes in
  seconds;
* against tests/golden/large.json at the full BASELINE sizes (2^32 nonces of
  configs[1] and configs[2], computed once by the 8-thread C oracle);
* beyond any CPU rescan, through size-independent properties: the sums of
  disjoint shards add up to the sum of their union, the counts are exact, and
  the independent generic kernel gives the same triple.
"""
import json
import os
import random

import pytest

from distributed_bitcoinminer_amd import _lib

pytestmark = pytest.mark.gpu
MAX = (1 << 64) - 1
M64 = MAX


def _add(parts):
    best = min(((h, n) for (h, n), _, _ in parts), default=(MAX, 0))
    return best, sum(s for _, s, _ in parts) & M64, sum(c for _, _, c in parts)


def _generic(ctx, m, lo, hi):
    ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 1)
    try:
        return ctx.scan_checked(m, lo, hi)
    finally:
        ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 0)


def test_checked_golden(ctx_paths, golden):
    n = 0
    for case in golden["scan_kats"]:
        if "sum" not in case:
            continue
        m = bytes.fromhex(case["msg_hex"])
        lo, hi = int(case["lo"]), int(case["hi"])
        exp = ((int(case["hash"]), int(case["nonce"])), int(case["sum"]), int(case["count"]))
        assert ctx_paths.scan_checked(m, lo, hi) == exp, (case["name"], lo, hi)
        n += 1
    assert n >= 390


def test_checked_min_equals_scan(ctx):
    for m, lo, hi in [(b"bradfitz", 0, 10**7), (b"x" * 57, 10**9 - 10**6, 10**9 + 10**6),
                      (b"bradfitz", MAX - 10**6, MAX)]:
        (best, _, cnt) = ctx.scan_checked(m, lo, hi)
        assert best == ctx.scan(m, lo, hi) and cnt == hi - lo + 1


def test_checked_layout_sweep_vs_oracle(ctx_paths, oracle_mod):
    """Every message length 0..130 x every digit count, both ends of each digit
    segment (partial tiles, surplus lanes, digit-count changes)."""
    rng = random.Random(5)
    for L in range(0, 131):
        m = bytes(rng.randrange(256) for _ in range(L))
        for d in range(1, 21):
            dlo = 0 if d == 1 else 10**(d - 1)
            dhi = min(10**d - 1, MAX)
            for lo, hi in ((dlo, min(dhi, dlo + 500)), (max(dlo, dhi - 400), min(MAX, dhi + 200))):
                assert ctx_paths.scan_checked(m, lo, hi) == oracle_mod.c_scan_sum(m, lo, hi), (L, d, lo, hi)


def test_checked_whole_tiles_vs_generic(ctx_paths):
    """Whole tiles of every fast layout (tiled / chained, W1, straddle, trailer,
    V) against the generic kernel's checked scan, including ranges large
    enough to use both whole and split (guided) tasks."""
    rng = random.Random(78)
    seen = set()
    for L in range(0, 131):
        m = bytes(rng.randrange(32, 127) for _ in range(L))
        for d in (7, 8, 10, 12, 16, 20):
            dlo, dhi = 10**(d - 1), min(10**d - 1, MAX)
            seg = _lib.debug_plan(m, dlo, dhi)[0]
            if seg["kind"] == _lib.HM_KIND_GENERIC:
                continue
            key = (seg["kind"], seg["W1"], seg["straddle"], seg["trailer"], seg["V"], seg["lane3"])
            if key in seen:
                continue
            seen.add(key)
            span = min(3 * 10**seg["V"] + 4321, 6 * 10**7, (dhi - dlo) // 2)
            lo = rng.randrange(dlo, dhi - span)
            fast = ctx_paths.scan_checked(m, lo, lo + span)
            assert fast == _generic(ctx_paths, m, lo, lo + span), (L, d, key)
            assert fast[2] == span + 1
    assert len(seen) >= 40, len(seen)


def test_checked_guided_split_boundaries(ctx):
    """bradfitz d=10: units of 6400 nonces; around one unit per wave of the
    grid the per-segment launch switches from whole units to tenths.  Ranges
    below, at and above that size, cut at arbitrary points, add up exactly.
    These ranges are small enough for the fused launch, so the per-segment
    kernels are forced (HM_OPT_FUSED=0); the fused answer must agree."""
    base = 3_000_000_000 + 12_345
    cuts = [base, base + 1, base + 6399, base + 20_000_000, base + 33_000_001,
            base + 64_000_000, base + 80_000_001]
    ctx.set_option(_lib.HM_OPT_FUSED, 0)
    try:
        whole = ctx.scan_checked(b"bradfitz", base, base + 80_000_000)
        assert ctx.stats()["dom_kind"] == _lib.HM_KIND_TILED
        parts = [ctx.scan_checked(b"bradfitz", a, b - 1) for a, b in zip(cuts, cuts[1:])]
    finally:
        ctx.set_option(_lib.HM_OPT_FUSED, 1)
    assert _add(parts) == whole
    assert whole == _generic(ctx, b"bradfitz", base, base + 80_000_000)
    assert whole == ctx.scan_checked(b"bradfitz", base, base + 80_000_000)  # fused


def _long120():
    rng = random.Random(440)
    return bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))


@pytest.mark.parametrize("msg", [b"bradfitz", _long120()], ids=["tiled", "chained"])
def test_checked_shard_edges_mid_tile(ctx, msg):
    """A weak-scaling shard of the bench (rank 3 of 8: [3*2^32, 4*2^32), d=11)
    starts and ends inside a tile (10^8 nonces for bradfitz).  The launch skips
    the lane chunks of its edge tiles that lie wholly outside the range; the
    count stays exact, cuts inside the first and last lane chunks and tiles add
    up, and windows at both edges match the generic kernel."""
    lo, hi = 3 << 32, (4 << 32) - 1
    seg = _lib.debug_plan(msg, lo, hi)[0]
    assert seg["kind"] in (_lib.HM_KIND_TILED, _lib.HM_KIND_CHAINED) and seg["d"] == 11
    whole = ctx.scan_checked(msg, lo, hi)
    assert whole[2] == hi - lo + 1
    P = 10 ** seg["V"]
    cuts = [lo, lo + 1, lo + 6399, lo + 6400 * 65 + 17, (lo // P + 1) * P, hi // P * P - 1,
            hi - 6400 * 3, hi, hi + 1]
    assert _add([ctx.scan_checked(msg, a, b - 1) for a, b in zip(cuts, cuts[1:])]) == whole
    for w_lo, w_hi in ((lo, lo + 3_000_000), (hi - 3_000_000, hi)):
        assert ctx.scan_checked(msg, w_lo, w_hi) == _generic(ctx, msg, w_lo, w_hi)


def _large():
    with open(os.path.join(os.path.dirname(__file__), "golden", "large.json")) as f:
        return [c for c in json.load(f) if "sum" in c]


@pytest.mark.parametrize("case", _large(), ids=lambda c: c["name"])
def test_checked_full_size_pinned(ctx, case):
    """BASELINE configs[1] and configs[2] at full size (2^32 nonces): minimum,
    sum of all 2^32 keys and count equal the C oracle's (tests/golden/large.json);
    uneven shards across digit and launch boundaries add up to the same."""
    m, lo, hi = bytes.fromhex(case["msg_hex"]), int(case["lo"]), int(case["hi"])
    exp = ((int(case["hash"]), int(case["nonce"])), int(case["sum"]), int(case["count"]))
    assert ctx.scan_checked(m, lo, hi) == exp
    cuts = [lo, 99_999_999, 10**9 - 3, 10**9 + 11, 2_147_483_648, 3_999_999_999, hi + 1]
    assert _add([ctx.scan_checked(m, a, b - 1) for a, b in zip(cuts, cuts[1:])]) == exp


def test_checked_beyond_cpu(ctx):
    """1.2e11 nonces at d=12 of a 56-B message (two-block tail with 5
    final-block digits: the chained kernel with a 10^5-row table since round
    3; the tiled kernel as two chunked launches of 2^20 tiles of 10^5 nonces
    when the chained layout is switched off -- both must give the same min,
    key sum and count), and 1.2e11 nonces of bradfitz at d=12 (three-word
    lanes, one launch): no CPU can rescan them, so the counts must be exact,
    shards split at the launch boundary and elsewhere must add up, and
    windows must match the generic kernel."""
    lo, hi = 10**11, 10**11 + 120_000_000_000
    ctx.set_option(_lib.HM_OPT_TABLE_DIGITS, -1)
    try:
        tiled = ctx.scan_checked(b"x" * 56, lo, hi)
        assert ctx.stats()["dom_kernel"].startswith("hm_tiled_csum_kernel<1, ")
    finally:
        ctx.set_option(_lib.HM_OPT_TABLE_DIGITS, 0)
    assert ctx.scan_checked(b"x" * 56, lo, hi) == tiled
    assert ctx.stats()["dom_kernel"] == "hm_chained_csum_kernel"
    for m in (b"x" * 56, b"bradfitz"):
        whole = ctx.scan_checked(m, lo, hi)
        assert whole[2] == hi - lo + 1
        boundary = (lo // 10**5 + (1 << 20)) * 10**5
        cuts = [lo, lo + 7_777_777_777, boundary - 3, boundary + 5, hi + 1]
        assert _add([ctx.scan_checked(m, a, b - 1) for a, b in zip(cuts, cuts[1:])]) == whole
        w_lo, w_hi = boundary - 20_000_000, boundary + 20_000_000
        assert ctx.scan_checked(m, w_lo, w_hi) == _generic(ctx, m, w_lo, w_hi)
        assert _lib.host_hash(m, whole[0][1]) == whole[0][0]


def test_checked_multi_device_and_streams(oracle_mod):
    """Shards over 2 and 3 'devices' (device 0 opened repeatedly) and 4 streams
    cover the range exactly once: same triple as one device and the oracle."""
    cases = [(b"a" * 45, 10**9 - 900_000, 10**9 + 300_000),
             (b"jonny greenwood", 10**8 - 2_000_000, 10**8 + 1_000_000),
             (b"bradfitz", MAX - 300_000, MAX)]
    exp = [oracle_mod.c_scan_sum(m, lo, hi) for m, lo, hi in cases]
    for devs, streams in (([0], 1), ([0], 4), ([0, 0], 1), ([0, 0, 0], 4)):
        with _lib.Context(devs) as c:
            c.set_option(_lib.HM_OPT_STREAMS, streams)
            for (m, lo, hi), e in zip(cases, exp):
                assert c.scan_checked(m, lo, hi) == e, (devs, streams, m, lo, hi)


def test_checked_empty_and_edges(ctx):
    assert ctx.scan_checked(b"bradfitz", 5, 4) == ((MAX, 0), 0, 0)
    assert ctx.scan_checked(b"bradfitz", MAX, MAX) == ((_lib.host_hash(b"bradfitz", MAX), MAX),
                                                        _lib.host_hash(b"bradfitz", MAX), 1)


@pytest.mark.parametrize("batch", [4, 32])
def test_queue_batch_checked(ctx, oracle_mod, batch):
    """HM_OPT_QUEUE_BATCH (round 6): a workgroup fetching 4 or 32 tasks per
    queue atomic still hashes every nonce once -- tiled (plain and straddle)
    and chained launches with their guided tails, checked against the
    oracle's (min, key sum, count).  The default (auto) takes 16 for
    launches of >= 10^11 nonces, which test_gpu_full_size covers."""
    ctx.set_option(_lib.HM_OPT_QUEUE_BATCH, batch)
    ctx.set_option(_lib.HM_OPT_FUSED, 0)
    try:
        for m, lo, hi in ((b"bradfitz", 0, 3 * 10**6), (b"thom yorke", 10**9 - 10**6, 10**9 + 10**6),
                          (b"z" * 120, 10**7 - 10**6, 10**7 + 10**6),
                          (b"q" * 60, 10**10, 10**10 + 2 * 10**6)):
            assert ctx.scan_checked(m, lo, hi) == oracle_mod.c_scan_sum(m, lo, hi), (batch, m, lo)
    finally:
        ctx.set_option(_lib.HM_OPT_QUEUE_BATCH, 0)
        ctx.set_option(_lib.HM_OPT_FUSED, 1)
