"""Chained layout for two-block tails with >= 5 final-block digits (round 3).

Lanes vary the last q digits of tail block 0, the final block's low fe digits
come from a K+W table (10^fe rows) and its high f - fe digits run as epochs,
one table and launch set each (plan.cpp consider_chained_epochs,
api.cpp enqueue_chained).  Every case goes through hm_scan_checked and is
compared with the SHA-extension CPU oracle's (min, key sum, count)
(oracle/hm_oracle_fast.c, itself checked against oracle/hm_oracle.c), so a
skipped, doubled or mis-hashed nonce fails.  The reference loop is
cmu440/bitcoin/miner/miner.go:46-59 over bitcoin.Hash (hash.go:13-17).
"""
import random

import pytest

from distributed_bitcoinminer_amd import _lib

pytestmark = pytest.mark.gpu
THREADS = 16  # the GPU box's CPU share


def _check(ctx, oracle_mod, m, lo, hi, kind=_lib.HM_KIND_CHAINED):
    seg = max(_lib.debug_plan(m, lo, hi), key=lambda s: s["hi"] - s["lo"])
    got = ctx.scan_checked(m, lo, hi)
    exp = oracle_mod.fast_scan_sum(m, lo, hi, threads=THREADS)
    assert got == exp, (len(m), lo, hi, seg)
    assert ctx.scan(m, lo, hi) == exp[0]
    return seg


@pytest.fixture()
def table_digits(ctx):
    yield lambda k: ctx.set_option(_lib.HM_OPT_TABLE_DIGITS, k)
    ctx.set_option(_lib.HM_OPT_TABLE_DIGITS, 0)


def test_f5_one_table(ctx, oracle_mod):
    """len 60 (3 digits in block 0), d = 8: f = 5, one 10^5-row table."""
    m = bytes(random.Random(60).randrange(33, 127) for _ in range(60))
    seg = _check(ctx, oracle_mod, m, 10**7, 10**8 - 1)
    assert seg["kind"] == _lib.HM_KIND_CHAINED and (seg["f"], seg["fe"]) == (5, 5)
    st = ctx.stats()
    assert st["dom_kernel"] == "hm_chained_kernel"
    assert 1.01 <= st["dom_compressions_eff"] <= 1.1  # block 0 once per <= 100 loop values


def test_epochs_small_tables(ctx, oracle_mod, table_digits):
    """The same segment with tables of 10^3 and 10^1 rows: 100 and 10^4 epochs."""
    m = bytes(random.Random(60).randrange(33, 127) for _ in range(60))
    exp = oracle_mod.fast_scan_sum(m, 10**7, 10**8 - 1, threads=THREADS)
    for k, nep in ((3, 100), (1, 10**4)):
        table_digits(k)
        assert ctx.scan_checked(m, 10**7, 10**8 - 1) == exp, k
        st = ctx.stats()
        assert st["dom_kernel"] == "hm_chained_csum_kernel" and st["dom_launches"] >= nep


def test_epoch_edges_and_partial_lanes(ctx, oracle_mod, table_digits):
    """Ranges that start and end inside lane chunks, epochs and tables:
    len 58 (5 digits in block 0) at d = 10 (f = 5) and d = 11 (f = 6), with
    the table capped to 10^2..10^4 rows; plus a request crossing 10^9."""
    m = bytes(random.Random(58).randrange(33, 127) for _ in range(58))
    rng = random.Random(5858)
    cases = [(10**9 + 4_321_987, 10**9 + 4_321_987 + 31_234_567),
             (10**10 + 77_777_777, 10**10 + 77_777_777 + 220_000_000),
             (10**9 - 3_000_000, 10**9 + 30_000_000)]
    for k in (2, 3, 4, 0):
        table_digits(k)
        for lo, hi in cases:
            seg = _check(ctx, oracle_mod, m, lo, hi)
            assert seg["kind"] == _lib.HM_KIND_CHAINED, (k, lo, hi, seg)
        lo = rng.randrange(10**9, 9 * 10**9)
        _check(ctx, oracle_mod, m, lo, lo + rng.randrange(26_000_000, 60_000_000))


def test_every_block0_digit_count(ctx, oracle_mod, table_digits):
    """Message lengths whose tail block 0 holds 3, 4 and 5 digits
    (r = 61, 60, 59 and 125..123), f = 5..7 final-block digits, tables capped
    to 10^3 rows so the ranges stay small for the CPU oracle."""
    table_digits(3)
    rng = random.Random(31)
    seen = set()
    for L in (58, 59, 60, 122, 123, 124):
        m = bytes(rng.randrange(256) for _ in range(L))
        r = (L + 1) % 64
        for f in (5, 6, 7):
            d = f + 64 - r
            S = 10**f                                  # nonces per lane value
            span = min(64 * S * 3, 10**d - 10**(d - 1) - 1)
            if span > 80_000_000:
                continue
            lo = 10**(d - 1) + rng.randrange(0, 64 * S)
            seg = _check(ctx, oracle_mod, m, lo, lo + span)
            if seg["kind"] == _lib.HM_KIND_CHAINED:
                seen.add((64 - r, f))
    assert {(5, 5), (4, 5), (3, 5)} <= seen, seen


def test_default_tables_config_size(ctx, oracle_mod, table_digits):
    """len 60 at d = 10 with the default 10^7-row table (f = 7, one launch)
    and a 10^6-row one (10 epochs);
    1.28e9 nonces, two lane chunks (6.4e8 nonces each) less a few at each
    end (the tiled kernel served this layout at 0.69 of the roofline)."""
    m = b"x" * 60
    lo = 2 * 640_000_000 + 123_456
    hi = 4 * 640_000_000 - 98_765
    seg = _check(ctx, oracle_mod, m, lo, hi)
    assert seg["kind"] == _lib.HM_KIND_CHAINED and (seg["f"], seg["fe"]) == (7, 7)
    assert ctx.stats()["dom_launches"] == 1
    table_digits(6)
    _check(ctx, oracle_mod, m, lo, hi)
    assert ctx.stats()["dom_launches"] == 10


def test_top_of_the_nonce_space(ctx, oracle_mod, table_digits):
    """20-digit nonces up to 2^64-1 (len 48: 15 digits in block 0, f = 5): the
    last tile is cut by 2^64-1, so lanes and epochs past it compute wrapped
    nonces that the range mask must drop.  One table, 10^2 and 10^1 rows."""
    MAX = (1 << 64) - 1
    m = bytes(random.Random(48).randrange(33, 127) for _ in range(48))
    for lo, hi in ((MAX - 30_000_000, MAX), (MAX - 25_123_457, MAX - 1_234_567)):
        exp = oracle_mod.fast_scan_sum(m, lo, hi, threads=THREADS)
        for k in (0, 2, 1):
            table_digits(k)
            seg = _lib.debug_plan(m, lo, hi)[0]
            assert seg["kind"] == _lib.HM_KIND_CHAINED and seg["f"] == 5
            assert ctx.scan_checked(m, lo, hi) == exp, (lo, hi, k)


def test_batches_streams_and_devices(oracle_mod):
    """Chained f >= 5 segments inside hm_scan_many batches: requests on four
    streams grow their K+W tables (10^5 and 10^6 rows) while other streams'
    work is in flight; then the same requests sharded over device 0 opened
    twice and three times (hm_partition shards, host merge)."""
    m58 = bytes(random.Random(58).randrange(33, 127) for _ in range(58))
    m60 = bytes(random.Random(60).randrange(33, 127) for _ in range(60))
    reqs = [(m58, 10**9 + 4_321_987, 10**9 + 4_321_987 + 31_234_567),     # f = 5, q = 5
            (m60, 10**7, 10**8 - 1),                                       # f = 5, q = 3
            (m58, 10**10 + 77_777_777, 10**10 + 77_777_777 + 220_000_000), # f = 6
            (b"bradfitz", 10**9, 10**9 + 10**7),                           # tiled
            (m60, 10**7 + 12_345, 10**7 + 12_345)]                         # one nonce
    assert sum(s["kind"] == _lib.HM_KIND_CHAINED and s["f"] >= 5
               for m, lo, hi in reqs for s in _lib.debug_plan(m, lo, hi)) >= 3
    exp = [oracle_mod.fast_scan_sum(m, lo, hi, threads=THREADS)[0] for m, lo, hi in reqs]
    for devs, streams in (([0], 4), ([0], 1), ([0, 0], 4), ([0, 0, 0], 4)):
        with _lib.Context(devs) as c:
            c.set_option(_lib.HM_OPT_STREAMS, streams)
            assert c.scan_many(reqs) == exp, (devs, streams)
            assert [c.scan(m, lo, hi) for m, lo, hi in reqs] == exp, (devs, streams)


def test_shards_cut_at_lane_chunks_checked(oracle_mod):
    """Multi-device contexts (GPU 0 opened 3 and 5 times) shard chained f >= 5
    ranges with hm_partition, whose cuts now fall on lane-chunk boundaries
    (plan.cpp partition_range): every shard re-plans as the chained layout and
    the per-device checked scans still cover the range exactly -- (min, key
    sum, count) equal the oracle's, so no nonce is lost or doubled at a cut."""
    m58 = bytes(random.Random(58).randrange(33, 127) for _ in range(58))
    m60 = bytes(random.Random(60).randrange(33, 127) for _ in range(60))
    cases = [(m58, 10**9 + 1_234_567, 10**9 + 71_234_567),      # f = 5, q = 5
             (m60, 10**7 + 5, 10**8 - 7),                        # f = 5, q = 3
             (m58, 10**10 + 3, 10**10 + 300_000_003)]            # f = 6
    for m, lo, hi in cases:
        exp = oracle_mod.fast_scan_sum(m, lo, hi, threads=THREADS)
        seg = _lib.debug_plan(m, lo, hi)[0]
        P, C = 10 ** seg["V"], 64 * 10 ** seg["f"]
        for n in (3, 5):
            cuts = [a for a, _ in _lib.partition(m, lo, hi, n)[1:]]
            assert all((a % P) % C == 0 for a in cuts), (n, cuts)
            with _lib.Context([0] * n) as c:
                assert c.scan_checked(m, lo, hi) == exp, (len(m), lo, hi, n)
                assert c.stats()["ndev"] == n
                assert c.scan(m, lo, hi) == exp[0]
                assert c.stats()["dom_kernel"] == "hm_chained_kernel"
