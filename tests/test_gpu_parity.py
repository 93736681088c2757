"""GPU parity: hm_scan through the C ABI vs golden fixtures and the CPU oracle.

Bar: bit-exact (hash, nonce) -- this is integer/byte work.  Oracle-backed
cases use sizes the C oracle finishes in seconds; full-size ranges are checked
through size-independent properties (shard invariance, re-hash of the winner,
kernel-vs-kernel agreement).
"""
import random

import pytest

from distributed_bitcoinminer_amd import _lib

pytestmark = pytest.mark.gpu
MAX = (1 << 64) - 1


def test_golden_scans(ctx_paths, golden):
    for case in golden["scan_kats"]:
        m = bytes.fromhex(case["msg_hex"])
        lo, hi = int(case["lo"]), int(case["hi"])
        got = ctx_paths.scan(m, lo, hi)
        assert got == (int(case["hash"]), int(case["nonce"])), (case["name"], lo, hi)


def test_golden_scans_generic_kernel(ctx_paths, golden):
    ctx_paths.set_option(_lib.HM_OPT_FORCE_GENERIC, 1)
    try:
        for case in golden["scan_kats"][:60]:
            m = bytes.fromhex(case["msg_hex"])
            lo, hi = int(case["lo"]), int(case["hi"])
            if hi - lo > 2_000_000:
                continue
            assert ctx_paths.scan(m, lo, hi) == (int(case["hash"]), int(case["nonce"])), case["name"]
    finally:
        ctx_paths.set_option(_lib.HM_OPT_FORCE_GENERIC, 0)


def test_config1_answer(ctx):
    # client `bradfitz 10000000` -> the reference prints "Result 356393768206 7645578"
    assert ctx.scan(b"bradfitz", 0, 10**7) == (356393768206, 7645578)
    assert ctx.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)


def test_single_nonce_kats(ctx, golden):
    # lo == hi: the scan returns exactly (Hash(msg, n), n)
    for case in golden["hash_kats"][::7]:
        m = bytes.fromhex(case["msg_hex"])
        n = int(case["nonce"])
        assert ctx.scan(m, n, n) == (int(case["hash"]), n), (case["name"], n)


def test_empty_range(ctx):
    assert ctx.scan(b"bradfitz", 5, 4) == (MAX, 0)
    assert ctx.scan(b"", MAX, 0) == (MAX, 0)


def test_random_vs_oracle(ctx_paths, oracle_mod):
    """Random messages (0..130 B, every tail layout) x ranges across digit boundaries."""
    rng = random.Random(2026)
    for it in range(120):
        L = rng.randrange(0, 131)
        m = bytes(rng.randrange(256) for _ in range(L))
        k = rng.randrange(1, 20)
        c = 10 ** k
        lo = max(0, c - rng.randrange(0, 40000))
        hi = min(MAX, c + rng.randrange(0, 40000))
        assert ctx_paths.scan(m, lo, hi) == oracle_mod.c_scan(m, lo, hi), (L, lo, hi)


def test_tiles_vs_oracle_medium(ctx_paths, oracle_mod):
    """Ranges spanning whole tiles (10^5..10^8 nonces per tile) for assorted layouts."""
    rng = random.Random(7)
    for L in (0, 3, 8, 20, 44, 45, 50, 54, 55, 56, 60, 63, 64, 70, 100, 119, 120, 127):
        m = bytes(rng.randrange(32, 127) for _ in range(L))
        lo = rng.randrange(10**9, 10**12)
        hi = lo + 1_500_000
        assert ctx_paths.scan(m, lo, hi) == oracle_mod.c_scan(m, lo, hi), (L, lo, hi)


def test_chained_layouts_vs_oracle(ctx_paths, oracle_mod):
    """Two-block tails whose final block holds 1..4 digits (chained kernel)."""
    rng = random.Random(99)
    seen = set()
    for L in range(56, 130):
        m = bytes(rng.randrange(33, 127) for _ in range(L))
        r = (L + 1) % 64
        for d in range(8, 21):
            T = r + d
            if T < 65 or T - 64 > 4:
                continue
            dhi = min(10**d - 1, MAX)
            seg = _lib.debug_plan(m, 10**(d - 1), dhi)[0]
            if seg["kind"] != _lib.HM_KIND_CHAINED:
                continue
            seen.add((T - 64, seg["V"] - (T - 64)))
            base = rng.randrange(10**(d - 1), dhi - 300_000)
            lo, hi = base, base + rng.randrange(1, 250_000)
            assert ctx_paths.scan(m, lo, hi) == oracle_mod.c_scan(m, lo, hi), (L, d, lo, hi)
    assert {(1, 5), (2, 5), (3, 5), (4, 5)} <= seen


def test_long120_config3_slice(ctx, oracle_mod):
    rng = random.Random(440)
    m = bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))
    for lo, hi in [(10**9 - 1_000_000, 10**9 + 1_000_000), (3_000_000_000, 3_003_000_000)]:
        assert ctx.scan(m, lo, hi) == oracle_mod.c_scan(m, lo, hi), (lo, hi)


def test_full_2p32_range(ctx):
    """BASELINE configs[1] at full size: pinned by the C oracle (tests/golden/large.json),
    then size-independent checks: shard invariance across 7 uneven shards and the
    generic kernel on a 2^26 sub-range."""
    import json
    import os
    from distributed_bitcoinminer_amd.parallel import merge
    with open(os.path.join(os.path.dirname(__file__), "golden", "large.json")) as f:
        case = json.load(f)[0]
    m, lo, hi = bytes.fromhex(case["msg_hex"]), int(case["lo"]), int(case["hi"])
    full = ctx.scan(m, lo, hi)
    assert full == (int(case["hash"]), int(case["nonce"]))
    assert _lib.host_hash(m, full[1]) == full[0]
    cuts = [lo, 123_456_789, 10**9 - 1, 10**9 + 7, 2_000_000_001, 3_333_333_333, 4_000_000_000, hi + 1]
    parts = [ctx.scan(m, a, b - 1) for a, b in zip(cuts, cuts[1:])]
    assert merge(parts) == full


def test_generic_vs_tiled_large(ctx):
    lo, hi = 3 * 10**9, 3 * 10**9 + (1 << 26)
    tiled = ctx.scan(b"bradfitz", lo, hi)
    ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 1)
    try:
        generic = ctx.scan(b"bradfitz", lo, hi)
    finally:
        ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 0)
    assert tiled == generic


def test_options_streams_and_rccl_merge(oracle_mod):
    """Multi-stream segment overlap and the in-library RCCL merge of the 16-B
    per-device results (ncclCommInitAll + grouped ncclAllGather + the strided
    device-side fold over the gathered candidates, api.cpp rccl_merge) give
    the same answers as the oracle.  On this 1-GPU box the communicator has
    one rank; the merge path is the one an 8-device context takes, and
    hm_stats.merge records that it ran (server.go:273-276 merge semantics)."""
    lo, hi = 10**8 - 3_000_000, 10**8 + 3_000_000  # 8- and 9-digit segments
    exp = oracle_mod.c_scan(b"jonny greenwood", lo, hi)
    rng = random.Random(808)
    reqs = []
    for i in range(150):  # > kMaxBatch = 64: three batch chunks, strided fold per request
        L = rng.randrange(0, 130)
        m = bytes(rng.randrange(256) for _ in range(L))
        a = max(0, 10**rng.randrange(1, 20) - rng.randrange(0, 3000))
        reqs.append((m, a, a + rng.randrange(-3, 5000)))
    exp_many = [oracle_mod.c_scan(m, a, b) for m, a, b in reqs]
    ck_lo, ck_hi = 10**9 - 700_000, 10**9 + 500_000
    exp_ck = oracle_mod.c_scan_sum(b"a" * 45, ck_lo, ck_hi)
    with _lib.Context([0]) as c:
        c.set_option(_lib.HM_OPT_STREAMS, 4)
        assert c.scan(b"jonny greenwood", lo, hi) == exp
        assert c.stats()["merge"] == _lib.HM_MERGE_NONE
        c.set_option(_lib.HM_OPT_MERGE_RCCL, 1)
        assert c.scan(b"jonny greenwood", lo, hi) == exp
        assert c.stats()["merge"] == _lib.HM_MERGE_RCCL
        assert c.scan_many(reqs) == exp_many
        assert c.stats()["merge"] == _lib.HM_MERGE_RCCL
        assert c.scan_checked(b"a" * 45, ck_lo, ck_hi) == exp_ck
        assert c.stats()["merge"] == _lib.HM_MERGE_RCCL
        assert c.scan(b"bradfitz", 5, 4) == (MAX, 0)  # empty range through the merge
        c.set_option(_lib.HM_OPT_GRID_PER_CU, 1)
        assert c.scan(b"jonny greenwood", lo, hi) == exp
        c.set_option(_lib.HM_OPT_MERGE_RCCL, 0)
        assert c.scan(b"jonny greenwood", lo, hi) == exp
        assert c.stats()["merge"] == _lib.HM_MERGE_NONE
    with _lib.Context() as c:  # every visible device
        assert c.scan(b"jonny greenwood", lo, hi) == exp
    with _lib.Context([0, 0]) as c:  # one RCCL rank per device: duplicates are refused
        assert c.scan(b"jonny greenwood", lo, hi) == exp
        assert c.stats()["merge"] == _lib.HM_MERGE_HOST
        # refused where the option is set (ABI 1.5), before any scan work
        with pytest.raises(_lib.HipMinerError) as ei:
            c.set_option(_lib.HM_OPT_MERGE_RCCL, 1)
        assert ei.value.rc == _lib.HM_ERR_INVALID
        assert c.scan(b"jonny greenwood", lo, hi) == exp
        assert c.stats()["merge"] == _lib.HM_MERGE_HOST


def test_rccl_merge_distinct_devices(oracle_mod):
    """The in-library RCCL merge over DISTINCT device ordinals: ncclCommInitAll
    over every visible GPU, one rank per device, each scanning its
    hm_partition shard, then the grouped ncclAllGather of the 16-B results and
    the device-side fold (api.cpp rccl_merge; the multi-device form of
    server.go:273-276).  Needs >= 2 GPUs: the 1-GPU box skips it."""
    import torch
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip(f"{n} visible GPU(s): distinct-ordinal RCCL merge needs >= 2")
    lo, hi = 10**8 - 3_000_000, 10**8 + 3_000_000
    exp = oracle_mod.c_scan(b"jonny greenwood", lo, hi)
    ck_lo, ck_hi = 10**9 - 700_000, 10**9 + 500_000
    exp_ck = oracle_mod.c_scan_sum(b"a" * 45, ck_lo, ck_hi)
    reqs = [(b"bradfitz", 10**k - 999, 10**k + 4000) for k in range(3, 20)]
    exp_many = [oracle_mod.c_scan(m, a, b) for m, a, b in reqs]
    with _lib.Context(list(range(n))) as c:
        c.set_option(_lib.HM_OPT_MERGE_RCCL, 1)
        assert c.scan(b"jonny greenwood", lo, hi) == exp
        st = c.stats()
        assert st["merge"] == _lib.HM_MERGE_RCCL and st["ndev"] == n
        assert c.scan_many(reqs) == exp_many
        assert c.scan_checked(b"a" * 45, ck_lo, ck_hi) == exp_ck
        assert c.scan(b"bradfitz", 5, 4) == (MAX, 0)


def test_config4_single_process_rccl_all_gpus():
    """configs[3] through the process model SURVEY §8(e) prescribes for one
    miner driving every GPU: one context over all visible devices
    (ncclCommInitAll over distinct ordinals), "bradfitz" [0, 2^40) sharded by
    hm_partition, the 16-B results merged by the grouped RCCL all-gather and
    the device fold.  The answer is full_size.json's whole-range oracle answer;
    the devices ran concurrently (summed kernel busy time well above the wall
    time) and the host never waited mid-enqueue.  Needs >= 2 GPUs."""
    import json
    import os
    import torch
    n = min(torch.cuda.device_count(), 8)
    if n < 2:
        pytest.skip(f"{n} visible GPU(s): the single-process RCCL context needs >= 2")
    with open(os.path.join(os.path.dirname(__file__), "golden", "full_size.json")) as f:
        w = json.load(f)["cfg4"]["whole"]
    exp = (int(w["hash"]), int(w["nonce"]))
    with _lib.Context(list(range(n))) as c:
        c.set_option(_lib.HM_OPT_MERGE_RCCL, 1)
        assert c.scan(b"bradfitz", 0, (1 << 40) - 1) == exp
        st = c.stats()
        assert st["merge"] == _lib.HM_MERGE_RCCL and st["ndev"] == n, st
        assert st["mid_call_syncs"] == 0, st
        assert st["kernel_ms"] > 0.6 * n * st["wall_ms"], st  # devices overlapped
        print(f"cfg4 on {n} GPUs, one process: wall {st['wall_ms']:.1f} ms = "
              f"{(1 << 40) / st['wall_ms'] / 1e6:.1f} GH/s; kernel "
              f"{(1 << 40) / (st['kernel_ms'] / n) / 1e6:.1f} GH/s")


def test_miner_eval_request_on_gpu(ctx, golden):
    from distributed_bitcoinminer_amd import bitcoin, miner
    mnr = miner.Miner(ctx=ctx)
    for k in golden["miner_eval_kats"]:
        req = bitcoin.NewRequest(bytes.fromhex(k["msg_hex"]), int(k["lower"]), int(k["upper"]))
        out, err = bitcoin.unmarshal(mnr.eval_request(bitcoin.marshal(req)))
        assert err is None and (out.Hash, out.Nonce) == (int(k["hash"]), int(k["nonce"]))


def test_stats_accounting(ctx):
    ctx.scan(b"bradfitz", 0, 2**32 - 1)
    st = ctx.stats()
    assert st["nonces"] == 2**32
    assert st["dom_kernel"] == "hm_tiled_kernel<4, false, false>"
    assert st["dom_nonces"] == 900_000_000 + 2**32 - 10**9 and st["dom_launches"] == 2
    assert st["dom_compressions"] == 1 and st["dom_kind"] == _lib.HM_KIND_TILED
    assert st["dom_compressions_eff"] == 1.0
    assert 0 < st["dom_kernel_ms"] <= st["kernel_ms"] <= st["wall_ms"] * 1.5
    # config 3: two tail blocks (C = 2), the chained kernel hoists block 0 out
    # of its loop: 1 + 1/tch compressions per nonce (tch = 1000 for f = 3)
    rng = random.Random(440)
    long120 = bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))
    ctx.set_option(_lib.HM_OPT_FUSED, 0)  # 10^8 nonces: a fused launch by default
    try:
        ctx.scan(long120, 10**9, 10**9 + 10**8)
    finally:
        ctx.set_option(_lib.HM_OPT_FUSED, 1)
    st = ctx.stats()
    assert st["dom_kind"] == _lib.HM_KIND_CHAINED and st["dom_compressions"] == 2
    # counted exactly (ABI 1.5): one block-0 compression per task and lane;
    # whole units cost 1/1000 per loop value, guided-split ones 10/1000
    assert 1.001 <= st["dom_compressions_eff"] <= 1.01
    # the fused launch: chained tasks of 100 loop values (block 0 per 100),
    # plus one block 0 per piece of the guided tail's split tasks (the last
    # partial wave-round: 15625 mod 3072 tasks x 10 pieces on 256 CUs)
    ctx.scan(long120, 10**9, 10**9 + 10**8)
    st = ctx.stats()
    assert st["dom_kind"] == _lib.HM_KIND_FUSED and st["dom_compressions"] == 2
    assert 1.009 <= st["dom_compressions_eff"] <= 1.013
    # a scan_many batch over several chunks times every launch against one
    # origin: the union of launch intervals is positive and below the wall time
    ctx.scan_many([(b"bradfitz", 10**9 + 10**7 * i, 10**9 + 10**7 * (i + 1) - 1)
                   for i in range(130)])
    st = ctx.stats()
    assert st["launches"] >= 130 and 0 < st["kernel_ms"] <= st["wall_ms"] * 1.5


def test_server_model_end_to_end_gpu(ctx, oracle_mod):
    """Config-5 style: 8 GPU 'miners' (one context, eight chunk requests) under the
    server's chunking near 2^64-1; the last chunk ends at 2^64-1 and scans nothing."""
    from distributed_bitcoinminer_amd import miner, server_model as sm
    mnr = miner.Miner(ctx=ctx)
    for msg in (b"bradfitz", b"thom yorke", b"jonny greenwood"):
        lo, up = MAX - 1 - 4_000_000, MAX - 1
        got = sm.expected_client_result(msg, lo, up, 8, mnr.scan)
        chunks = sm.load_balance(lo, up, 8)
        assert chunks[-1][1] == MAX
        assert got == oracle_mod.c_scan(msg, lo, chunks[-1][0])


def test_layout_sweep_segment_edges(ctx_paths, oracle_mod):
    """Every message length 0..130 x every digit count: small ranges at both
    ends of each digit segment (partial tiles, masking, digit-count changes)."""
    import random as _r
    rng = _r.Random(31)
    for L in range(0, 131):
        m = bytes(rng.randrange(256) for _ in range(L))
        for d in range(1, 21):
            dlo = 0 if d == 1 else 10**(d - 1)
            dhi = min(10**d - 1, MAX)
            for lo, hi in ((dlo, min(dhi, dlo + 700)), (max(dlo, dhi - 700), min(MAX, dhi + 300))):
                assert ctx_paths.scan(m, lo, hi) == oracle_mod.c_scan(m, lo, hi), (L, d, lo, hi)


def test_layout_sweep_full_tiles_tiled_vs_generic(ctx_paths):
    """Whole tiles (10^5..10^8 nonces) of every layout the planner picks for
    lengths 0..130: fast kernels vs the independent generic kernel."""
    import random as _r
    rng = _r.Random(77)
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
            span = min(2 * 10**seg["V"] + 12345, 3 * 10**8, (dhi - dlo) // 2)
            lo = rng.randrange(dlo, dhi - span)
            fast = ctx_paths.scan(m, lo, lo + span)
            ctx_paths.set_option(_lib.HM_OPT_FORCE_GENERIC, 1)
            try:
                slow = ctx_paths.scan(m, lo, lo + span)
            finally:
                ctx_paths.set_option(_lib.HM_OPT_FORCE_GENERIC, 0)
            assert fast == slow, (L, d, key)
            assert _lib.host_hash(m, fast[1]) == fast[0]
    assert len(seen) >= 40, len(seen)


def test_multi_device_context_sharding(oracle_mod):
    """The in-process multi-device path (cost-weighted contiguous shards of
    hm_partition + merge of 16-B results) with device 0 opened as 2 and 3
    'devices' on this 1-GPU box.  The m=45 case crosses 9 -> 10 digits, where
    the trailer block doubles the per-nonce cost, so its shards are uneven."""
    cases = [(b"bradfitz", 0, 9999), (b"bradfitz", 5, 5), (b"bradfitz", 5, 6), (b"x", 5, 4),
             (b"jonny greenwood", 10**9 - 777_777, 10**9 + 123_456),
             (b"a" * 45, 10**9 - 900_000, 10**9 + 300_000),
             (b"bradfitz", MAX - 100_000, MAX)]
    for devs in ([0, 0], [0, 0, 0]):
        with _lib.Context(devs) as c:
            for m, lo, hi in cases:
                assert c.scan(m, lo, hi) == oracle_mod.c_scan(m, lo, hi), (devs, m, lo, hi)
            assert c.stats()["ndev"] == len(devs)


def test_scan_many_batches(oracle_mod):
    """hm_scan_many == per-request hm_scan, across batch chunks (> kMaxBatch =
    64 requests), empty requests, streams and multi-device contexts."""
    rng = random.Random(4242)
    reqs = []
    for i in range(150):
        L = rng.randrange(0, 130)
        m = bytes(rng.randrange(256) for _ in range(L))
        k = rng.randrange(1, 20)
        lo = max(0, 10**k - rng.randrange(0, 3000))
        hi = lo + rng.randrange(-5, 6000)
        reqs.append((m, lo, max(hi, 0) if i % 17 else lo - 1))  # some empty
    exp = [oracle_mod.c_scan(m, lo, hi) for m, lo, hi in reqs]
    for devs, streams in (([0], 1), ([0], 4), ([0, 0], 1)):
        with _lib.Context(devs) as c:
            c.set_option(_lib.HM_OPT_STREAMS, streams)
            assert c.scan_many(reqs) == exp, (devs, streams)
            assert c.scan_many([]) == []
    with _lib.Context([0]) as c:
        assert c.scan_many([(b"bradfitz", 0, 10**7), (b"bradfitz", 0, 9999)]) == \
            [(356393768206, 7645578), (1419516646206828, 9898)]


def test_chunked_tile_launches(ctx):
    """A segment with > 2^20 tiles is split into several launches.  A 56-B
    message at d=12 has a two-block tail whose last digit opens word 1 of
    block 1 (W1 = 1, no room for three-word lanes): V=5, 10^5-nonce tiles, so
    1.2e11 nonces = 1.2 M tiles -> 2 launches.  Checked by shard invariance
    across the launch boundary and the generic kernel on a window around it."""
    m = b"x" * 56
    lo, hi = 10**11, 10**11 + 120_000_000_000
    # the planner runs this layout chained (round 3, f = 5 final-block
    # digits) unless told otherwise; the two kernels must agree on all 1.2e11
    assert _lib.debug_plan(m, lo, hi)[0]["kind"] == _lib.HM_KIND_CHAINED
    ctx.set_option(_lib.HM_OPT_TABLE_DIGITS, -1)
    try:
        tiled = _chunked_tiled(ctx, m, lo, hi)
    finally:
        ctx.set_option(_lib.HM_OPT_TABLE_DIGITS, 0)
    assert ctx.scan(m, lo, hi) == tiled
    assert ctx.stats()["dom_kernel"] == "hm_chained_kernel"


def _chunked_tiled(ctx, m, lo, hi):
    from distributed_bitcoinminer_amd.parallel import merge
    whole = ctx.scan(m, lo, hi)
    st = ctx.stats()
    assert st["dom_kernel"].startswith("hm_tiled_kernel<1, "), st
    assert st["dom_launches"] >= 2
    boundary = (lo // 10**5 + (1 << 20)) * 10**5  # first nonce of the 2nd launch
    parts = [ctx.scan(m, lo, boundary - 7), ctx.scan(m, boundary - 6, hi)]
    assert merge(parts) == whole
    w_lo, w_hi = boundary - 30_000_000, boundary + 30_000_000
    fast = ctx.scan(m, w_lo, w_hi)
    ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 1)
    try:
        assert ctx.scan(m, w_lo, w_hi) == fast
    finally:
        ctx.set_option(_lib.HM_OPT_FORCE_GENERIC, 0)
    assert _lib.host_hash(m, whole[1]) == whole[0]
    return whole
