"""hm_partition: cost-weighted contiguous shards.  Host-only.

Properties: the shards are ascending, contiguous and cover [lo, hi] exactly
(so the merged per-shard minima equal the whole-range scan), and every shard
carries the same modelled cost up to one nonce's cost (seg_cost as the
planner reports it through hm_debug_plan)."""
import random

import pytest

from distributed_bitcoinminer_amd import _lib, parallel

MAX = (1 << 64) - 1


def _check_cover(shards, lo, hi):
    got = [s for s in shards if s is not None]
    if lo > hi:
        assert got == []
        return
    assert got[0][0] == lo and got[-1][1] == hi
    for a, b in zip(got, got[1:]):
        assert b[0] == a[1] + 1
    for a, b in got:
        assert a <= b


def _shard_cost(msg, shard):
    if shard is None:
        return 0
    return sum((s["hi"] - s["lo"] + 1) * s["cost"] for s in _lib.debug_plan(msg, *shard))


EDGE = [(b"bradfitz", 0, 0), (b"bradfitz", 0, 9), (b"bradfitz", 0, 2**32 - 1),
        (b"a" * 45, 0, 2**32 - 1), (b"a" * 54, 0, 10**12), (b"", MAX - 2, MAX),
        (b"x", 0, MAX), (b"x", 5, 4), (b"q", 7, 7), (bytes(range(120)), 0, 2**32 - 1),
        (b"jonny greenwood", 10**19 - 5, 10**19 + 5)]


@pytest.mark.parametrize("n", [1, 2, 3, 8, 64])
def test_partition_covers_exactly(n):
    for msg, lo, hi in EDGE:
        _check_cover(_lib.partition(msg, lo, hi, n), lo, hi)
    rng = random.Random(n)
    for _ in range(200):
        msg = bytes(rng.randrange(256) for _ in range(rng.randrange(130)))
        lo = rng.choice([0, rng.randrange(MAX), 10**rng.randrange(20)])
        hi = min(MAX, lo + rng.choice([0, 1, n - 1, rng.randrange(10**rng.randrange(1, 20))]))
        _check_cover(_lib.partition(msg, lo, hi, n), lo, hi)


@pytest.mark.parametrize("msg,lo,hi", [(b"a" * 45, 0, 2**32 - 1), (b"bradfitz", 0, 2**40 - 1),
                                       (bytes(range(120)), 0, 2**32 - 1), (b"a" * 50, 0, 10**15),
                                       (b"x", 0, MAX)])
def test_partition_balances_modelled_cost(msg, lo, hi):
    n = 8
    shards = _lib.partition(msg, lo, hi, n)
    costs = [_shard_cost(msg, s) for s in shards]
    worst_nonce = max(s["cost"] for s in _lib.debug_plan(msg, lo, hi))
    assert max(costs) - min(costs) <= 2 * worst_nonce + 1e-6 * max(costs), costs


def test_partition_weights_digit_segments():
    """m=45: 9-digit nonces fit one block (C=1), 10-digit ones need a trailer
    block (C=2): the shard holding [0, 10^9) must take more nonces."""
    segs = _lib.debug_plan(b"a" * 45, 0, 2**32 - 1)
    assert segs[-1]["trailer"] == 1 and segs[-2]["trailer"] == 0
    shards = _lib.partition(b"a" * 45, 0, 2**32 - 1, 8)
    sizes = [b - a + 1 for a, b in shards]
    assert sizes[0] > 1.5 * sizes[-1]
    ratio = segs[-1]["cost"] / segs[-2]["cost"]
    assert sizes[0] / sizes[-1] == pytest.approx(ratio, rel=1e-3)  # shard 0 also holds d<=8


def test_partition_uniform_segment_is_equal_counts():
    # one digit segment, one kernel: equal counts to within one nonce
    shards = _lib.partition(b"bradfitz", 10**9, 2 * 10**9 + 12344, 8)
    sizes = [b - a + 1 for a, b in shards]
    assert max(sizes) - min(sizes) <= 1


def test_partition_errors():
    lib = _lib.load()
    import ctypes
    buf = (ctypes.c_uint64 * 4)()
    assert lib.hm_partition(b"x", 1, 0, 9, 0, buf) == _lib.HM_ERR_INVALID
    assert lib.hm_partition(b"x", 1, 0, 9, 2, None) == _lib.HM_ERR_INVALID
    assert lib.hm_partition(None, 3, 0, 9, 2, buf) == _lib.HM_ERR_INVALID
    assert lib.hm_partition(None, 0, 0, 9, 2, buf) == _lib.HM_OK


def test_shard_range_with_msg_uses_partition():
    for r in range(8):
        assert parallel.shard_range(0, 2**32 - 1, 8, r, msg=b"a" * 45) == \
            _lib.partition(b"a" * 45, 0, 2**32 - 1, 8)[r]


def _chunk_bounds(seg):
    """Lane-chunk boundaries of a chained segment: tile t's chunk c starts at
    t*10^(q+f) + c*64*10^f (lanes vary block-0 digits, stride 10^f)."""
    P = 10 ** (seg["V"])
    C = 64 * 10 ** seg["f"]
    return P, C


@pytest.mark.parametrize("msg,lo,hi", [(b"x" * 60, 10**9, 10**10 - 1),
                                       (b"y" * 58, 10**10 + 77_777_777, 10**10 + 2_277_777_777)])
def test_partition_cuts_chained_f5_at_lane_chunks(msg, lo, hi):
    """A chained f >= 5 lane chunk spans 64*10^f nonces and is hashed whole by
    each shard that touches it, so hm_partition cuts such segments at lane
    chunk boundaries (plan.cpp partition_range): every internal cut is one,
    each shard still re-plans as the chained layout, and the shards' modelled
    costs (re-planned, edge lanes included) stay within one chunk of each
    other and add up to the whole range's."""
    seg = _lib.debug_plan(msg, lo, hi)[0]
    assert seg["kind"] == _lib.HM_KIND_CHAINED and seg["f"] >= 5
    P, C = _chunk_bounds(seg)
    chunk_cost = C * seg["cost"]  # one lane chunk's nonces x their per-nonce cost
    whole = _shard_cost(msg, (lo, hi))
    for n in (2, 4, 8):
        shards = _lib.partition(msg, lo, hi, n)
        _check_cover(shards, lo, hi)
        for a, _ in shards[1:]:
            assert (a % P) % C == 0, (n, a)
        # shards between two cuts hold whole chunks: the chained layout stays
        for s in shards[1:-1]:
            assert all(p["kind"] == _lib.HM_KIND_CHAINED for p in _lib.debug_plan(msg, *s)), s
        costs = [_shard_cost(msg, s) for s in shards]
        assert max(costs) - min(costs) <= 1.05 * chunk_cost, (n, costs, chunk_cost)
        assert sum(costs) <= 1.02 * whole, (n, sum(costs), whole)
