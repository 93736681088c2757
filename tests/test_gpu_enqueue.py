"""The host never waits on the GPU while a call is still enqueuing (ABI 1.6).

Chained f >= 5 segments grow their stream's K+W table (10^5 .. 10^7 rows).
Work queued earlier may still read the old table, so it is retired (api.cpp
kw_table_rows; freed at hm_close -- ABI 1.7 freed it at the end of the call,
but hipFree waits for the whole device, other contexts' work included)
instead of freed, which would drain the device mid-enqueue: every device of a
context gets its work before the host waits on any of it (one
context drives all of a miner's GPUs).  hm_stats counts the waits issued while
enqueuing (mid_call_syncs), the tables grown (table_grows) and the host time
spent enqueuing (enqueue_ms); answers are compared with the oracle.  The
reference loop: cmu440/bitcoin/miner/miner.go:46-59 over bitcoin.Hash
(hash.go:13-17).
"""
import json
import os
import random

import pytest

from distributed_bitcoinminer_amd import _lib

pytestmark = pytest.mark.gpu
THREADS = 16  # the GPU box's CPU share
M58 = bytes(random.Random(58).randrange(33, 127) for _ in range(58))
F5 = (M58, 10**9 + 4_321_987, 10**9 + 4_321_987 + 31_234_567)        # f = 5: 10^5 rows
F6 = (M58, 10**10 + 77_777_777, 10**10 + 77_777_777 + 220_000_000)    # f = 6: 10^6 rows


def _weak_prefix(n_pieces):
    """Oracle answer of "bradfitz" over [0, n*2^32) from the full-size fixture."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "full_size.json")) as f:
        w = next(x for x in json.load(f)["weak"] if x["name"] == "bradfitz")
    return min((int(p["hash"]), int(p["nonce"])) for p in w["pieces"][:n_pieces])


def _chained_f(m, lo, hi):
    return {s["f"] for s in _lib.debug_plan(m, lo, hi) if s["kind"] == _lib.HM_KIND_CHAINED}


def test_table_growth_does_not_block_enqueue(oracle_mod):
    """Context([0, 0]) (two devices, one GPU): a 2^34-nonce request whose
    dominant launches run ~0.5 s, then two f >= 5 chained requests whose
    shards grow tables on both devices while that work is in flight.  No host
    wait before the last launch is queued, the whole batch is queued in a
    small fraction of the call, and every answer equals the oracle's."""
    assert 5 in _chained_f(*F5) and 6 in _chained_f(*F6)
    big = (b"bradfitz", 0, (4 << 32) - 1)
    reqs = [big, F5, F6]
    exp = [_weak_prefix(4)] + [oracle_mod.fast_scan_sum(m, lo, hi, threads=THREADS)[0]
                               for m, lo, hi in (F5, F6)]
    with _lib.Context([0, 0]) as c:
        assert c.scan_many(reqs) == exp
        st = c.stats()
        assert st["ndev"] == 2
        assert st["mid_call_syncs"] == 0, st
        # both devices' chained shards grow tables beyond the 10^4 rows of hm_open
        assert st["table_grows"] >= 2, st
        # ~0.5 s of kernels; enqueuing (planning, 10^5/10^6-row allocations,
        # launches) must not have waited for them
        assert st["kernel_ms"] > 200, st
        assert st["enqueue_ms"] < 0.25 * st["wall_ms"], st
        print("enqueue_ms", st["enqueue_ms"], "wall_ms", st["wall_ms"],
              "table_grows", st["table_grows"])
        # the grown tables stay: the same batch again grows none
        assert c.scan_many(reqs) == exp
        st = c.stats()
        assert st["table_grows"] == 0 and st["mid_call_syncs"] == 0, st


def test_single_device_growth_on_second_stream(oracle_mod):
    """One device: a large request keeps stream 0 busy while the chained
    requests grow K+W tables: F5 (small, round-robin stream) to 10^5 rows,
    then F6 (2.2e8 nonces: the dominant-stream order, stream 0) to 10^6 rows,
    which retires a table still in use if F5 went to stream 0 too."""
    reqs = [(b"bradfitz", 0, (2 << 32) - 1), F5, F6]
    exp = [_weak_prefix(2)] + [oracle_mod.fast_scan_sum(m, lo, hi, threads=THREADS)[0]
                               for m, lo, hi in (F5, F6)]
    with _lib.Context([0]) as c:
        assert c.scan_many(reqs) == exp
        st = c.stats()
        assert st["mid_call_syncs"] == 0 and st["table_grows"] >= 2, st
        assert st["enqueue_ms"] < 0.25 * st["wall_ms"], st


@pytest.mark.parametrize("cap,req,f", [(10**4, F5, 5), (10**5, F6, 6)])
def test_table_rows_cap_falls_back_to_epochs(oracle_mod, cap, req, f):
    """HM_OPT_TABLE_ROWS_CAP makes table growth fail as on a device out of
    memory: the chained layout falls back to a table of 10^(f-1) rows and 10
    epochs (enqueue_chained), and the answer and checksum are unchanged."""
    m, lo, hi = req
    exp = oracle_mod.fast_scan_sum(m, lo, hi, threads=THREADS)
    with _lib.Context([0]) as c:
        c.set_option(_lib.HM_OPT_TABLE_ROWS_CAP, cap)
        assert c.scan_checked(m, lo, hi) == exp
        st = c.stats()
        assert st["dom_kernel"] == "hm_chained_csum_kernel", st
        assert st["table_grows"] == (0 if cap == 10**4 else 1), st  # 10^4 rows at hm_open
        assert st["dom_launches"] >= 10, st   # >= 10 epochs of one table each
        assert c.scan(m, lo, hi) == exp[0]
        # lifting the cap grows the table to the planned 10^f rows: fewer launches
        n_capped = st["dom_launches"]
        c.set_option(_lib.HM_OPT_TABLE_ROWS_CAP, 0)
        assert c.scan_checked(m, lo, hi) == exp
        st = c.stats()
        assert st["table_grows"] >= 1 and st["dom_launches"] < n_capped, st
    assert f in _chained_f(m, lo, hi)


def test_mid_call_sync_counter_counts(oracle_mod):
    """hm_stats.mid_call_syncs is live: the test hook HM_OPT_TEST_MID_SYNC puts
    a host wait into each device's enqueue, and the counter sees one per
    device (0 without the hook); the answers do not change."""
    m, lo, hi = b"bradfitz", 10**9, 10**9 + 50_000_000
    exp = oracle_mod.fast_scan_sum(m, lo, hi, threads=THREADS)[0]
    with _lib.Context([0, 0]) as c:
        assert c.scan(m, lo, hi) == exp
        assert c.stats()["mid_call_syncs"] == 0
        c.set_option(_lib.HM_OPT_TEST_MID_SYNC, 1)
        assert c.scan(m, lo, hi) == exp
        assert c.stats()["mid_call_syncs"] == 2, c.stats()
        c.set_option(_lib.HM_OPT_TEST_MID_SYNC, 0)
        assert c.scan(m, lo, hi) == exp
        assert c.stats()["mid_call_syncs"] == 0


def test_streams_are_made_on_first_use(oracle_mod):
    """ABI 1.8 (hardware-queue headroom of the N = 8 line): hm_open
    makes stream 0 only; fused requests stay on it; a multi-segment request
    makes the tail streams up to HM_OPT_STREAMS and no more; answers equal
    the fixture throughout."""
    from distributed_bitcoinminer_amd import _lib
    with _lib.Context([0]) as c:
        assert c.streams_made() == 1
        assert c.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)  # fused
        assert c.scan_many([(b"x", 0, 999), (b"y", 5, 50_000)]) == \
            [oracle_mod.c_scan(b"x", 0, 999), oracle_mod.c_scan(b"y", 5, 50_000)]
        assert c.streams_made() == 2  # two fused requests of a batch: two streams
        c.set_option(_lib.HM_OPT_STREAMS, 2)
        # one digit segment, far above the fused size: stream 0 alone
        lo = 10**11
        assert c.scan(b"bradfitz", lo, lo + 10**9) == oracle_mod.fast_scan_sum(
            b"bradfitz", lo, lo + 10**9)[0]
        assert c.streams_made() == 2
        assert c.scan(b"bradfitz", 0, 2**32 - 1) == (5256245051, 1626825724)
        assert c.streams_made() == 2
        c.set_option(_lib.HM_OPT_STREAMS, 4)
        # the tail segments (d <= 8) run as one fused launch: 2 streams suffice
        assert c.scan(b"bradfitz", 0, 2**32 - 1) == (5256245051, 1626825724)
        assert c.streams_made() == 2
        c.set_option(_lib.HM_OPT_TAIL_FUSED, 0)  # one launch per tail segment
        assert c.scan(b"bradfitz", 0, 2**32 - 1) == (5256245051, 1626825724)
        assert c.streams_made() == 4
    with _lib.Context([0]) as c:
        c.set_option(_lib.HM_OPT_STREAMS, 1)
        assert c.scan(b"bradfitz", 0, 2**32 - 1) == (5256245051, 1626825724)
        assert c.streams_made() == 1
