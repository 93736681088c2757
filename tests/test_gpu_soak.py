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
HM_SOAK_SEED picks the sequence; a failure names its case.
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
    while time.time() - t0 < budget:
        table = 0
        if rng.randrange(5) == 0:
            m, lo, hi, table = _epoch_case(rng)
        else:
            m, lo, hi = _case(rng)
        ctx.set_option(_lib.HM_OPT_TABLE_DIGITS, table)
        try:
            got = ctx.scan_checked(m, lo, hi)
        finally:
            ctx.set_option(_lib.HM_OPT_TABLE_DIGITS, 0)
        exp = oracle_mod.c_scan_sum(m, lo, hi)
        assert (got[0], got[1], got[2]) == (tuple(exp[0]), exp[1], exp[2]), (n, m.hex(), lo, hi, table)
        n += 1
        nonces += hi - lo + 1
        if time.time() - last > 10:
            last = time.time()
            print(f"soak: {n} cases, {nonces} nonces, {last - t0:.0f} s", flush=True)
    print(f"soak done: seed {seed}, {n} cases, {nonces} nonces, all equal to the oracle", flush=True)
    assert n > 0
