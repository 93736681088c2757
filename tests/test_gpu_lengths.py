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


def test_every_length_three_digit_counts(ctx_paths, oracle_mod):
    rng = random.Random(200)
    for L in range(0, 201):
        m = bytes(rng.randrange(256) for _ in range(L))
        for lo in (10**9 - 400_000,                    # 9 -> 10 digits
                   rng.randrange(10**13, 10**14),      # 14 digits
                   MAX - 999_999):                     # 20 digits up to 2^64-1
            hi = min(MAX, lo + 999_999)
            exp = oracle_mod.fast_scan_sum(m, lo, hi, threads=16)
            assert ctx_paths.scan_checked(m, lo, hi) == exp, (L, lo, hi)


@pytest.mark.parametrize("L", [255, 256, 1000, 1983, 4095, 4096, 65537])
def test_long_messages(ctx_paths, oracle_mod, L):
    """Messages far past the SURVEY lengths (up to 1025 host-midstate blocks;
    1983 B is the longest Data an LSP payload can carry in a 2000-B datagram
    with the JSON overhead, roughly): every tail layout at 9/10 and 20 digits,
    through hm_scan_checked and hm_scan against the oracle."""
    rng = random.Random(L)
    m = bytes(rng.randrange(256) for _ in range(L))
    for lo in (10**9 - 300_000, MAX - 700_000):
        hi = min(MAX, lo + 699_999)
        exp = oracle_mod.fast_scan_sum(m, lo, hi, threads=16)
        assert ctx_paths.scan_checked(m, lo, hi) == exp, (L, lo, hi)
        assert ctx_paths.scan(m, lo, hi) == exp[0]
    # the host hash of the winner agrees (hm_hash, bitcoin.Hash on the host)
    from distributed_bitcoinminer_amd import _lib
    assert _lib.host_hash(m, exp[0][1]) == exp[0][0]
