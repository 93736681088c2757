"""Randomised parity soak of the HIP path against the C oracle.

For HM_SOAK_SECONDS seconds (default 20 in the GPU suite; 300 for a soak
run), random (message, range) cases through hm_scan_checked,
each compared with oracle_scan_sum -- the min (hash, nonce) of the reference
loop (miner.go:46-59 over hash.go:13-17), the sum of every key mod 2^64 and
the count.  Messages are 0..200 random bytes (any value), ranges sit around
random digit-count boundaries or anywhere, from 1 to ~2*10^6 nonces, some
ending at 2^64-1.  One case in five is a two-block tail with 5 final-block
digits over 1.3-3.2*10^7 nonces (the chained layout with a K+W table, round 3)
under a random table cap HM_OPT_TABLE_DIGITS (1..5: 10^4..1 epochs).
A second soak (half the budget) sends random hm_scan_many batches to fresh
multi-"device" contexts under random stream counts and table-growth caps.
Since round 6 each case also draws the fused launch's guided-tail pieces
(HM_OPT_FUSED_TAIL 1/2/5/10) and the queue batch (HM_OPT_QUEUE_BATCH), and
one case in ten is a large request (1.4-3*10^8 nonces) whose tail segments
run as one fused launch beside the dominant kernel (HM_OPT_TAIL_FUSED on or
off), checked against the SHA-extension oracle.
HM_SOAK_SEED picks the sequence; a failure names its case.  HM_SOAK_FUSED=0
sends the small requests through the per-segment kernels instead of the fused
launch (HM_OPT_FUSED=0), which every request above 2^27 nonces takes.
Progress goes to stdout every ~10 s (run with -s).
"""
import os
import random
import time

import pytest

MAX = (1 << 64) - 1


def _epoch_case(rng):
    """Lengths whose tail block 0 holds 3..5 digits, f = 5 final-block digits."""
    L = rng.choice([58, 59, 60, 122, 123, 124])
    m = bytes(rng.randrange(256) for _ in range(L))
    d = 5 + 64 - (L + 1) % 64
    span = rng.randrange(13_000_000, 32_000_000)
    lo = 10 ** (d - 1) + rng.randrange(0, 9 * 10 ** (d - 1) - span)
    return m, lo, lo + span - 1, rng.randrange(0, 6)


def _large_case(rng):
    """A request above the fused size whose small digit segments form a tail
    (round 6: one fused launch on a tail stream)."""
    L = rng.randrange(0, 130)
    m = bytes(rng.randrange(256) for _ in range(L))
    c = 10 ** rng.randrange(8, 12)
    lo = c - rng.randrange(10**6, 10**8)
    return m, lo, lo + rng.randrange(140_000_000, 300_000_000)


def _case(rng):
    L = rng.choice([rng.randrange(0, 201), rng.randrange(40, 70), rng.randrange(110, 130)])
    m = bytes(rng.randrange(256) for _ in range(L))
    span = rng.choice([1, rng.randrange(1, 100), rng.randrange(100, 70_000),
                       rng.randrange(70_000, 2_000_000)])
    kind = rng.randrange(4)
    if kind == 0:  # across a digit-count boundary
        c = 10 ** rng.randrange(1, 20)
        lo = max(0, c - rng.randrange(0, span + 1))
    elif kind == 1:  # near the top of the nonce space
        lo = MAX - rng.randrange(0, span + 1)
    else:  # anywhere
        lo = rng.randrange(0, MAX)
    hi = min(MAX, lo + span - 1)
    return m, lo, hi


@pytest.mark.gpu
@pytest.mark.timeout(3600)
def test_random_soak_checked(ctx, oracle_mod):
    budget = float(os.environ.get("HM_SOAK_SECONDS", "20"))
    seed = int(os.environ.get("HM_SOAK_SEED", "355"))
    rng = random.Random(seed)
    t0 = last = time.time()
    n = nonces = 0
    from distributed_bitcoinminer_amd import _lib
    fused = os.environ.get("HM_SOAK_FUSED", "1") != "0"
    ctx.set_option(_lib.HM_OPT_FUSED, 1 if fused else 0)
    try:
        while time.time() - t0 < budget:
            table, large = 0, False
            if rng.randrange(5) == 0:
                m, lo, hi, table = _epoch_case(rng)
            elif rng.randrange(10) == 0:
                m, lo, hi = _large_case(rng)
                large = True
            else:
                m, lo, hi = _case(rng)
            opts = {_lib.HM_OPT_TABLE_DIGITS: table,
                    _lib.HM_OPT_FUSED_TAIL: rng.choice([1, 2, 2, 5, 10]),
                    _lib.HM_OPT_QUEUE_BATCH: rng.choice([0, 0, 4, 8, 16, 32]),
                    _lib.HM_OPT_TAIL_FUSED: rng.choice([1, 1, 0]),
                    _lib.HM_OPT_STREAMS: rng.choice([2, 2, 4, 1])}
            for o, v in opts.items():
                ctx.set_option(o, v)
            try:
                got = ctx.scan_checked(m, lo, hi)
            finally:
                for o, v in ((_lib.HM_OPT_TABLE_DIGITS, 0), (_lib.HM_OPT_FUSED_TAIL, 2),
                             (_lib.HM_OPT_QUEUE_BATCH, 0), (_lib.HM_OPT_TAIL_FUSED, 1),
                             (_lib.HM_OPT_STREAMS, 4)):
                    ctx.set_option(o, v)
            exp = oracle_mod.fast_scan_sum(m, lo, hi) if large and oracle_mod.fast_available() \
                else oracle_mod.c_scan_sum(m, lo, hi)
            assert (got[0], got[1], got[2]) == (tuple(exp[0]), exp[1], exp[2]), \
                (n, m.hex(), lo, hi, sorted(opts.items()))
            n += 1
            nonces += hi - lo + 1
            if time.time() - last > 10:
                last = time.time()
                print(f"soak: {n} cases, {nonces} nonces, {last - t0:.0f} s", flush=True)
    finally:
        ctx.set_option(_lib.HM_OPT_FUSED, 1)
    print(f"soak done: seed {seed}, fused {int(fused)}, {n} cases, {nonces} nonces, "
          "all equal to the oracle", flush=True)
    assert n > 0


@pytest.mark.gpu
@pytest.mark.timeout(3600)
def test_random_batches_fresh_contexts(oracle_mod):
    """Randomised hm_scan_many batches on fresh contexts (round 4): 1..3
    "devices" (GPU 0 opened repeatedly, so the batch is sharded and each shard
    grows its own K+W tables), 1 or 4 streams, a random HM_OPT_TABLE_ROWS_CAP
    (growth refused above 10^4 / 10^5 rows, as on a device out of memory) and
    2..6 requests (one batch in ten: 65..80, two hm_scan_many chunks) mixing
    the random cases with chained f = 5 cases.  Tables
    grow while earlier requests' work is in flight (the old ones are retired
    until the context closes); every answer equals the oracle's.  Runs for HM_SOAK_SECONDS / 2."""
    from distributed_bitcoinminer_amd import _lib
    budget = float(os.environ.get("HM_SOAK_SECONDS", "20")) / 2
    seed = int(os.environ.get("HM_SOAK_SEED", "355")) + 1
    rng = random.Random(seed)
    t0 = last = time.time()
    n = reqs_done = grows = 0
    while time.time() - t0 < budget:
        devs = [0] * rng.randrange(1, 4)
        streams = rng.choice([1, 2, 4])
        tail_fused = rng.choice([0, 1])
        cap = rng.choice([0, 0, 10**4, 10**5])
        reqs = []
        # one batch in ten spans two hm_scan_many chunks (> kMaxBatch = 64)
        for _ in range(rng.randrange(65, 81) if rng.randrange(10) == 0 else rng.randrange(2, 7)):
            if rng.randrange(3) == 0:
                m, lo, hi, _ = _epoch_case(rng)
            else:
                m, lo, hi = _case(rng)
            reqs.append((m, lo, hi))
        exp = [tuple(oracle_mod.fast_scan_sum(m, lo, hi, threads=16)[0]) for m, lo, hi in reqs]
        with _lib.Context(devs) as c:
            c.set_option(_lib.HM_OPT_FUSED, 0 if os.environ.get("HM_SOAK_FUSED", "1") == "0" else 1)
            c.set_option(_lib.HM_OPT_STREAMS, streams)
            c.set_option(_lib.HM_OPT_TAIL_FUSED, tail_fused)
            c.set_option(_lib.HM_OPT_TABLE_ROWS_CAP, cap)
            got = c.scan_many(reqs)
            st = c.stats()
        assert got == exp, (n, len(devs), streams, tail_fused, cap,
                            [(m.hex(), lo, hi) for m, lo, hi in reqs])
        assert st["mid_call_syncs"] == 0, (n, st)
        n += 1
        reqs_done += len(reqs)
        grows += st["table_grows"]
        if time.time() - last > 10:
            last = time.time()
            print(f"batch soak: {n} batches, {reqs_done} requests, {grows} table growths, "
                  f"{last - t0:.0f} s", flush=True)
    print(f"batch soak done: seed {seed}, {n} batches, {reqs_done} requests, {grows} table "
          f"growths, all equal to the oracle", flush=True)
    assert n > 0
