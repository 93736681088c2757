"""Every message length 0..200 (0..3 host-midstate blocks, every tail layout)
at three digit counts, through hm_scan_checked against the SHA-extension CPU
oracle's (min, key sum, count) over 10^6-nonce ranges: the tiled, trailer,
chained and generic kernels all meet the oracle on the same inputs.  The
reference loop is cmu440/bitcoin/miner/miner.go:46-59 over bitcoin.Hash
(hash.go:13-17)."""
import random

import pytest

pytestmark = pytest.mark.gpu
MAX = (1 << 64) - 1


def test_every_length_three_digit_counts(ctx, oracle_mod):
    rng = random.Random(200)
    for L in range(0, 201):
        m = bytes(rng.randrange(256) for _ in range(L))
        for lo in (10**9 - 400_000,                    # 9 -> 10 digits
                   rng.randrange(10**13, 10**14),      # 14 digits
                   MAX - 999_999):                     # 20 digits up to 2^64-1
            hi = min(MAX, lo + 999_999)
            exp = oracle_mod.fast_scan_sum(m, lo, hi, threads=16)
            assert ctx.scan_checked(m, lo, hi) == exp, (L, lo, hi)
