"""Concurrency of the C ABI (include/hipminer.h "Threading"): calls on one
context are serialised by its mutex and re-bind the device on every call, so
a Go miner may call from any OS thread; separate contexts on one GPU run
concurrently.  Python threads reach the ABI through ctypes, which releases
the GIL for the foreign call, so the calls really overlap.  Every answer must
equal the CPU oracle's (miner.go:46-59 over hash.go:13-17)."""
import random
import threading

import pytest

from distributed_bitcoinminer_amd import _lib

pytestmark = pytest.mark.gpu


def _requests(seed, n):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        L = rng.randrange(0, 130)
        m = bytes(rng.randrange(256) for _ in range(L))
        lo = max(0, 10 ** rng.randrange(1, 20) - rng.randrange(0, 50_000))
        out.append((m, lo, lo + rng.randrange(0, 400_000)))
    return out


def _run_threads(fns):
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001 -- reported below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts), "a scan thread hung"
    if errs:
        raise errs[0]


def test_one_context_many_threads(ctx, oracle_mod):
    """8 threads share one context: scans, checked scans, batches and stats
    interleave; each result is the oracle's."""
    reqs = [_requests(100 + i, 12) for i in range(8)]
    exp = [[oracle_mod.c_scan_sum(m, lo, hi) for m, lo, hi in r] for r in reqs]

    def worker(i):
        def f():
            for j, (m, lo, hi) in enumerate(reqs[i]):
                if (i + j) % 3 == 0:
                    assert ctx.scan_checked(m, lo, hi) == exp[i][j], (i, j)
                elif (i + j) % 3 == 1:
                    assert ctx.scan(m, lo, hi) == exp[i][j][0], (i, j)
                else:
                    assert ctx.scan_many([(m, lo, hi)] * 2) == [exp[i][j][0]] * 2, (i, j)
                st = ctx.stats()
                assert st["ndev"] == 1 and st["wall_ms"] > 0
        return f

    _run_threads([worker(i) for i in range(8)])


def test_contexts_per_thread(oracle_mod):
    """4 threads, one context each on GPU 0: their kernels run concurrently on
    the device; a 2^28-nonce scan per thread checks coverage under overlap."""
    big = [(b"bradfitz", 3_000_000_000 + k * (1 << 28), 3_000_000_000 + (k + 1) * (1 << 28) - 1)
           for k in range(4)]
    small = [_requests(200 + k, 6) for k in range(4)]
    exp_small = [[oracle_mod.c_scan(m, lo, hi) for m, lo, hi in r] for r in small]
    results = [None] * 4

    def worker(k):
        def f():
            with _lib.Context([0]) as c:
                m, lo, hi = big[k]
                results[k] = c.scan_checked(m, lo, hi)
                for j, (m2, lo2, hi2) in enumerate(small[k]):
                    assert c.scan(m2, lo2, hi2) == exp_small[k][j], (k, j)
        return f

    _run_threads([worker(k) for k in range(4)])
    with _lib.Context([0]) as c:
        for k in range(4):
            m, lo, hi = big[k]
            assert results[k][2] == hi - lo + 1
            assert results[k] == c.scan_checked(m, lo, hi), k  # the same triple alone
