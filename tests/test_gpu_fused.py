"""The fused small-request launch (ABI 1.7, HM_KIND_FUSED) on the GPU.

A request of <= 2^27 nonces whose segments all fit runs as ONE planner
launch and ONE scan launch (fused_kernels.hip), each segment with its own
layout's task body.  Here: configs[0]'s Request (the client's [0, 10^7] plus
the server's +1, cmu440/bitcoin/server/server.go:169) is one launch; every
message length 0..130 (every tail layout: tiled with and without a trailer,
chained f <= 4, generic) is checked with the coverage checksum against the C
oracle, fused and per-segment; batches mix fused and per-segment requests;
and the edges (empty, single nonce, 2^64-1, forced generic) hold.  The
reference loop: cmu440/bitcoin/miner/miner.go:46-59 over bitcoin.Hash
(hash.go:13-17)."""
import random

import pytest

from distributed_bitcoinminer_amd import _lib

pytestmark = pytest.mark.gpu
MAX = (1 << 64) - 1


@pytest.fixture()
def fused_off(ctx):
    ctx.set_option(_lib.HM_OPT_FUSED, 0)
    yield ctx
    ctx.set_option(_lib.HM_OPT_FUSED, 1)


def test_config1_is_one_launch(ctx):
    assert ctx.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
    st = ctx.stats()
    assert st["launches"] == 1 and st["dom_kind"] == _lib.HM_KIND_FUSED, st
    assert st["dom_kernel"] == "hm_fused_kernel" and st["nonces"] == 10**7 + 2, st
    assert st["dom_compressions_eff"] == 1.0, st


def test_config1_per_segment_path_still_answers(fused_off):
    assert fused_off.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
    st = fused_off.stats()
    assert st["launches"] == 8 and st["dom_kind"] == _lib.HM_KIND_TILED, st


def test_every_layout_checked_vs_oracle(ctx, oracle_mod):
    """Every message length 0..130 over a range crossing a digit-count change:
    the fused launch's (min, key sum, count) equals the oracle's, and so does
    the per-segment path's."""
    rng = random.Random(505)
    kinds = set()
    for L in range(131):
        m = bytes(rng.randrange(32, 127) for _ in range(L))
        d = rng.randrange(2, 20)
        lo = max(0, 10**d - rng.randrange(1, 25_000))
        hi = min(MAX, 10**d + rng.randrange(0, 25_000))
        exp = oracle_mod.c_scan_sum(m, lo, hi)
        got = ctx.scan_checked(m, lo, hi)
        assert got == exp, (L, lo, hi)
        assert ctx.stats()["dom_kind"] == _lib.HM_KIND_FUSED
        kinds |= {s["kind"] for s in _lib.debug_plan(m, lo, hi)}
        ctx.set_option(_lib.HM_OPT_FUSED, 0)
        try:
            assert ctx.scan_checked(m, lo, hi) == exp, ("per-segment", L, lo, hi)
        finally:
            ctx.set_option(_lib.HM_OPT_FUSED, 1)
    assert kinds >= {_lib.HM_KIND_TILED, _lib.HM_KIND_CHAINED, _lib.HM_KIND_GENERIC}


def test_layouts_with_trailer_and_chained_segments(ctx, oracle_mod):
    """Messages whose segments use the trailer block (45-55 B at d = 10) and
    the chained layout (f = 1..4), several segments per request."""
    rng = random.Random(606)
    for L in (44, 45, 50, 54, 55, 56, 57, 60, 63, 64, 100, 119, 120, 127):
        m = bytes(rng.randrange(33, 127) for _ in range(L))
        for lo, hi in ((0, 2_000_000), (10**9 - 700_000, 10**9 + 700_000),
                       (10**11 - 300_000, 10**11 + 900_000)):
            assert ctx.scan_checked(m, lo, hi) == oracle_mod.c_scan_sum(m, lo, hi), (L, lo, hi)
            st = ctx.stats()
            assert st["launches"] == 1 and st["dom_kind"] == _lib.HM_KIND_FUSED, st


def test_random_requests_vs_oracle(ctx, oracle_mod):
    """200 random (message, range) draws of up to 2e5 nonces, anywhere in u64."""
    rng = random.Random(707)
    for _ in range(200):
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(131)))
        if rng.random() < 0.6:
            lo = max(0, 10**rng.randrange(1, 20) - rng.randrange(1, 100_000))
        else:
            lo = rng.randrange(MAX)
        hi = min(MAX, lo + rng.randrange(200_000))
        assert ctx.scan(m, lo, hi) == oracle_mod.c_scan(m, lo, hi), (m.hex(), lo, hi)


def test_edges(ctx, oracle_mod):
    assert ctx.scan(b"bradfitz", 5, 4) == (MAX, 0)
    for n in (0, 9, 10, 10**19, MAX):
        assert ctx.scan(b"x", n, n) == (oracle_mod.c_hash(b"x", n), n)
    lo = MAX - 150_000
    assert ctx.scan_checked(b"bradfitz", lo, MAX) == oracle_mod.c_scan_sum(b"bradfitz", lo, MAX)
    assert ctx.stats()["dom_kind"] == _lib.HM_KIND_FUSED
    ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 1)
    try:
        for m, lo, hi in ((b"bradfitz", 0, 200_000), (b"y" * 60, 10**9 - 5000, 10**9 + 5000)):
            assert ctx.scan_checked(m, lo, hi) == oracle_mod.c_scan_sum(m, lo, hi)
            st = ctx.stats()
            assert st["launches"] == 1 and st["dom_kind"] == _lib.HM_KIND_FUSED, st
    finally:
        ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 0)


def test_batch_mixes_fused_and_per_segment_requests(ctx, oracle_mod):
    """hm_scan_many: small requests go to fused launches on the stream
    round-robin, a large one to the per-segment path; all answers exact."""
    reqs = [(b"bradfitz", 0, 10**6), (b"thom yorke", 10**9 - 10**5, 10**9 + 10**5),
            (b"q" * 61, 10**12, 10**12 + 3 * 10**5), (b"bradfitz", 10**9, 10**9 + 3 * 10**8),
            (b"", 0, 99), (b"z" * 120, 10**7 - 10**5, 10**7 + 10**5)]
    exp = [oracle_mod.c_scan(m, lo, hi) for m, lo, hi in reqs]
    assert ctx.scan_many(reqs) == exp
    st = ctx.stats()
    assert st["launches"] >= 5 + 1, st


def test_multi_device_context_fuses_each_shard(oracle_mod):
    """Context([0, 0]): each device's shard of a small request is one fused
    launch; the merged answer equals the oracle's."""
    with _lib.Context([0, 0]) as c:
        m, lo, hi = b"bradfitz", 0, 3_000_000
        assert c.scan_checked(m, lo, hi) == oracle_mod.c_scan_sum(m, lo, hi)
        st = c.stats()
        assert st["launches"] == 2 and st["dom_kind"] == _lib.HM_KIND_FUSED, st


@pytest.mark.parametrize("parts", [2, 5, 10])
def test_split_tiled_tasks_checked(ctx, oracle_mod, parts):
    """HM_OPT_FUSED_PARTS: tiled tasks of the fused launch cut into `parts`
    pieces of the units loop; (min, key sum, count) over tiled layouts with
    and without trailer / straddle, several segments per request, still
    equal the oracle's."""
    rng = random.Random(808 + parts)
    ctx.set_option(_lib.HM_OPT_FUSED_PARTS, parts)
    try:
        assert ctx.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
        for L in (0, 8, 13, 30, 45, 50, 55, 61, 70, 110):
            m = bytes(rng.randrange(33, 127) for _ in range(L))
            lo = max(0, 10**rng.randrange(3, 19) - rng.randrange(1, 400_000))
            hi = lo + rng.randrange(1, 800_000)
            assert ctx.scan_checked(m, lo, hi) == oracle_mod.c_scan_sum(m, lo, hi), (L, lo, hi)
            assert ctx.stats()["dom_kind"] == _lib.HM_KIND_FUSED
    finally:
        ctx.set_option(_lib.HM_OPT_FUSED_PARTS, 1)


def test_fused_parts_option_validated(ctx):
    for bad in (0, 3, 4, 11, -1):
        with pytest.raises(_lib.HipMinerError):
            ctx.set_option(_lib.HM_OPT_FUSED_PARTS, bad)


@pytest.mark.parametrize("flags", [0, 2, 3, 4, 8, 9, 17, 25])
def test_task_dispensing_flags_checked(ctx, oracle_mod, flags):
    """HM_OPT_FUSED_FLAGS: every way the fused launch's waves get their tasks
    (queue, static first task, prefetch, static stride, LDS dispenser) hashes
    every nonce once: (min, key sum, count) equal the oracle's, over layouts
    with trailer, straddle, chained and generic segments."""
    rng = random.Random(909 + flags)
    ctx.set_option(_lib.HM_OPT_FUSED_FLAGS, flags)
    try:
        assert ctx.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
        for L in (0, 8, 45, 55, 60, 61, 100, 120):
            m = bytes(rng.randrange(33, 127) for _ in range(L))
            lo = max(0, 10**rng.randrange(3, 19) - rng.randrange(1, 400_000))
            hi = lo + rng.randrange(1, 1_500_000)
            assert ctx.scan_checked(m, lo, hi) == oracle_mod.c_scan_sum(m, lo, hi), (L, lo, hi)
            assert ctx.stats()["dom_kind"] == _lib.HM_KIND_FUSED
    finally:
        ctx.set_option(_lib.HM_OPT_FUSED_FLAGS, 1)


@pytest.mark.parametrize("tail", [1, 5, 10])
def test_guided_tail_pieces_checked(ctx, oracle_mod, tail):
    """HM_OPT_FUSED_TAIL (round 6; default 2, covered by every other test):
    the tasks of a fused launch's last partial wave-round run as up to `tail`
    pieces each -- tiled, trailer, chained and generic tasks alike, combined
    with split tiled tasks and every dispensing mode -- and every nonce is
    still hashed exactly once: (min, key sum, count) equal the oracle's."""
    rng = random.Random(1000 + tail)
    ctx.set_option(_lib.HM_OPT_FUSED_TAIL, tail)
    try:
        assert ctx.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
        for L in (0, 8, 45, 55, 57, 60, 61, 100, 120):
            m = bytes(rng.randrange(33, 127) for _ in range(L))
            for lo, hi in ((max(0, 10**rng.randrange(3, 19) - rng.randrange(1, 400_000)), None),
                           (0, 20_000), (10**15, 10**15 + 3)):
                hi = hi if hi is not None else lo + rng.randrange(1, 2_000_000)
                assert ctx.scan_checked(m, lo, hi) == oracle_mod.c_scan_sum(m, lo, hi), \
                    (tail, L, lo, hi)
                assert ctx.stats()["dom_kind"] == _lib.HM_KIND_FUSED
        for parts, flags in ((2, 1), (5, 9), (1, 4), (1, 2)):
            ctx.set_option(_lib.HM_OPT_FUSED_PARTS, parts)
            ctx.set_option(_lib.HM_OPT_FUSED_FLAGS, flags)
            m = b"thom yorke"
            assert ctx.scan_checked(m, 10**9 - 900_000, 10**9 + 900_000) == \
                oracle_mod.c_scan_sum(m, 10**9 - 900_000, 10**9 + 900_000), (parts, flags)
    finally:
        ctx.set_option(_lib.HM_OPT_FUSED_PARTS, 1)
        ctx.set_option(_lib.HM_OPT_FUSED_FLAGS, 1)
        ctx.set_option(_lib.HM_OPT_FUSED_TAIL, 2)


def test_fused_tail_option_validated(ctx):
    for bad in (0, 3, 4, 11, -1):
        with pytest.raises(_lib.HipMinerError):
            ctx.set_option(_lib.HM_OPT_FUSED_TAIL, bad)


def test_large_request_tail_segments_fused(ctx, oracle_mod):
    """HM_OPT_TAIL_FUSED (round 6, default on): a large request's segments off
    its dominant kernel (here d <= 8 of [0, 3*10^8], 10^8 nonces) run as ONE
    fused launch in the dominant launch's tail.  Checked against the oracle
    with the coverage sums, on 2 and 4 streams, and equal to the per-segment
    tail (option off); configs[1] and [2] keep their fixtures."""
    m, lo, hi = b"bradfitz", 0, 3 * 10**8
    exp = oracle_mod.fast_scan_sum(m, lo, hi) if oracle_mod.fast_available() else \
        oracle_mod.c_scan_sum(m, lo, hi)
    for streams in (2, 4):
        ctx.set_option(_lib.HM_OPT_STREAMS, streams)
        try:
            assert ctx.scan_checked(m, lo, hi) == exp, streams
            st = ctx.stats()
            assert st["dom_kind"] == _lib.HM_KIND_TILED, st
            # the dominant launch(es), then ONE fused launch for d = 1..8
            assert st["launches"] == st["dom_launches"] + 1, st
            ctx.set_option(_lib.HM_OPT_TAIL_FUSED, 0)
            assert ctx.scan_checked(m, lo, hi) == exp, streams
            assert ctx.stats()["launches"] == st["dom_launches"] + 8
        finally:
            ctx.set_option(_lib.HM_OPT_TAIL_FUSED, 1)
            ctx.set_option(_lib.HM_OPT_STREAMS, 4)
    assert ctx.scan(b"bradfitz", 0, 2**32 - 1) == (5256245051, 1626825724)
    import bench
    assert ctx.scan(bench.long120(), 0, 2**32 - 1) == (1410660608, 124104753)


def test_results_stored_to_host_or_copied_agree(oracle_mod):
    """HM_OPT_HOST_RESULT (round 6 experiment hook, default off): the call's
    last fold kernel stores the 16-B results in pinned host memory instead of
    the copy back.  Same answers on one device, a batch, a two-device host
    merge and the RCCL merge, fused requests and a tail-fused one included."""
    # the last request has tail segments (d <= 8) that run as one fused
    # launch on a tail stream beside its dominant d = 9 launch
    reqs = [(b"bradfitz", 0, 10**7 + 1), (b"thom yorke", 10**9, 10**9 + 2 * 10**8),
            (b"x" * 120, 0, 99_999), (b"", 5, 4), (b"jonny greenwood", 0, 2 * 10**8)]

    def oracle(m, a, b):
        if a > b:
            return (MAX, 0)
        if b - a > 10**7 and oracle_mod.fast_available():
            return tuple(oracle_mod.fast_scan_sum(m, a, b)[0])
        return oracle_mod.c_scan(m, a, b)
    exp = [oracle(m, a, b) for m, a, b in reqs]
    for devs, rccl in (([0], False), ([0, 0], False), ([0], True)):
        with _lib.Context(devs) as c:
            if rccl:
                c.set_option(_lib.HM_OPT_MERGE_RCCL, 1)
            for host in (1, 0, 1):
                c.set_option(_lib.HM_OPT_HOST_RESULT, host)
                assert c.scan_many(reqs) == exp, (devs, rccl, host)
                for (m, a, b), e in zip(reqs, exp):
                    assert c.scan(m, a, b) == e, (devs, rccl, host, m, a, b)


def test_fused_trace_diagnostics(oracle_mod):
    """HM_OPT_FUSED_TRACE (diagnostics, tools/fused_trace.py): every wave of the
    fused launch records its start, last-task and end times and its task
    count; the answers do not change and the waves' tasks cover the launch."""
    with _lib.Context([0]) as c:
        assert c.fused_trace() == []  # nothing traced yet
        c.set_option(_lib.HM_OPT_FUSED_TRACE, 1)
        assert c.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
        tr = c.fused_trace()
        st = c.stats()
        assert len(tr) == st["dom_grid"] * 4, (len(tr), st)
        assert all(t[0] <= t[1] <= t[2] for t in tr if t[3] > 0)
        # 10^7 + 2 nonces: >= 15,625 tiled tasks of 640 nonces, plus pieces
        assert sum(t[3] for t in tr) >= 15_625
        m = b"z" * 120
        assert c.scan(m, 0, 10**6) == oracle_mod.c_scan(m, 0, 10**6)
