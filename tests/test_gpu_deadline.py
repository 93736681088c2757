"""SURVEY §8(b) liveness on the GPU (ABI 1.8): a GPU scan that misses its
deadline returns HM_ERR_TIMEOUT instead of blocking, abandons its context,
and the miner answers that Request on the host and later ones too.

Why: the native LSP client heartbeats on its own thread (lsp_client.cpp), so
a miner blocked in a hung hm_scan is never dropped, and the unchanged server
reassigns only dropped miners' chunks (server.go:326-376): without a
deadline the client would never get its Result (miner.go:60-62 always writes
one).  A 1-ms deadline on a 10^9-nonce Request (≈ 27 ms of kernel) stands in
for the hung GPU, without hanging one."""
import os
import subprocess
import time

import pytest

from distributed_bitcoinminer_amd import _lib, bitcoin
from tests import lsp_harness as H

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MINER = os.path.join(ROOT, "distributed_bitcoinminer_amd", "hm_miner")
ENV = dict(os.environ, HM_LSP_EPOCH_MS="100", HM_LSP_EPOCH_LIMIT="50", HIPMINER_DEVICES="0")
LO, HI = 10**9, 2 * 10**9 - 1  # the [10^9, 2*10^9) Request


def _expected(oracle_mod, msg, lo, hi):
    if oracle_mod.fast_available():
        return oracle_mod.fast_scan_sum(msg, lo, hi)[0]
    return oracle_mod.c_scan(msg, lo, hi)


def test_deadline_timeout_abandons_the_context(oracle_mod):
    c = _lib.Context([0])
    c.scan(b"bradfitz", 0, 10**6)  # module loaded, first launches done
    c.set_option(_lib.HM_OPT_DEADLINE_MS, 1)
    t = time.perf_counter()
    with pytest.raises(_lib.HipMinerError) as ei:
        c.scan(b"bradfitz", LO, HI)
    assert ei.value.rc == _lib.HM_ERR_TIMEOUT
    assert time.perf_counter() - t < 1.0
    # abandoned: every later call fails at once, without touching the device
    for call in (lambda: c.scan(b"bradfitz", 0, 9), lambda: c.scan_many([(b"x", 0, 9)]),
                 lambda: c.scan_checked(b"x", 0, 9),
                 lambda: c.set_option(_lib.HM_OPT_DEADLINE_MS, 0)):
        t = time.perf_counter()
        with pytest.raises(_lib.HipMinerError) as ei:
            call()
        assert ei.value.rc == _lib.HM_ERR_TIMEOUT
        assert time.perf_counter() - t < 0.05
    t = time.perf_counter()
    c.close()  # host memory only
    assert time.perf_counter() - t < 0.05
    # a new context on the same GPU works (the abandoned work drains beside it)
    with _lib.Context([0]) as c2:
        assert c2.scan(b"bradfitz", 0, 9999) == (1419516646206828, 9898)
        assert c2.scan(b"bradfitz", LO, HI) == _expected(oracle_mod, b"bradfitz", LO, HI)


def test_auto_deadline_is_modelled_and_harmless(ctx, oracle_mod):
    """HM_OPT_DEADLINE_MS = -1: 2 s + 8x the modelled kernel time; the polled
    wait returns the same answers as the blocking one, on the fused, the
    per-segment and the multi-request paths."""
    ctx.set_option(_lib.HM_OPT_DEADLINE_MS, -1)
    try:
        assert ctx.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
        d_small = ctx.stats()["deadline_ms"]
        assert 2000 <= d_small < 2100, d_small
        got = ctx.scan(b"bradfitz", 0, (1 << 32) - 1)
        assert got == (5256245051, 1626825724)  # tests/golden/large.json
        st = ctx.stats()
        # ~0.11 s modelled for 2^32 nonces at C = 1
        assert 2500 < st["deadline_ms"] < 4000, st
        assert st["wall_ms"] < st["deadline_ms"]
        reqs = [(b"thom yorke", 19970000, 19971000), (b"x" * 120, 0, 99_999)]
        assert ctx.scan_many(reqs) == [oracle_mod.c_scan(m, a, b) for m, a, b in reqs]
        ctx.set_option(_lib.HM_OPT_DEADLINE_MS, 60_000)
        ctx.scan(b"bradfitz", 0, 10**6)
        assert ctx.stats()["deadline_ms"] == 60_000
    finally:
        ctx.set_option(_lib.HM_OPT_DEADLINE_MS, 0)
    ctx.scan(b"bradfitz", 0, 10**6)
    assert ctx.stats()["deadline_ms"] == 0


def _ask(srv, cid, data, lower, upper):
    srv.write(cid, bitcoin.marshal(bitcoin.NewRequest(data, lower, upper)))
    res, err = bitcoin.unmarshal(srv.read(cid, timeout=120))
    assert err is None and res.Type == bitcoin.Result
    return res.Hash, res.Nonce


def test_miner_answers_a_timed_out_request_on_the_host(oracle_mod):
    """hm_miner with a 1-ms scan deadline: the [10^9, 2*10^9) Request times out
    on the GPU, is answered on the host with the oracle's Result, the miner
    answers later Requests (GPU retried after HM_MINER_RETRY_MS), and the
    process exits 0."""
    assert os.path.exists(MINER), "build hm_miner first (__graft_entry__.build())"
    exp = _expected(oracle_mod, b"bradfitz", LO, HI)
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=50)
    env = dict(ENV, HM_SCAN_DEADLINE_MS="1", HM_MINER_RETRY_MS="0", HM_CPU_THREADS="16",
               HM_MINER_VERBOSE="1")
    p = subprocess.Popen([MINER, srv.hostport], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        cid = srv.accept(timeout=120)
        assert srv.read(cid, timeout=60) == bitcoin.marshal(bitcoin.NewJoin())
        assert _ask(srv, cid, "bradfitz", LO, HI) == exp
        assert _ask(srv, cid, "bradfitz", 0, 9999) == (1419516646206828, 9898)
        m = "thom yorke".encode()
        assert _ask(srv, cid, m, 19970000, 19971000) == oracle_mod.c_scan(m, 19970000, 19971000)
    finally:
        srv.close()
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    err = p.stderr.read()
    assert p.returncode == 0, err
    assert "GPU scan FAILED" in err and "deadline" in err and "hm_scan_cpu" in err, err
    assert f"Request [{LO}, {HI}] on host" in err, err
    assert "GPU (re)opened" in err, err


def test_miner_uses_the_gpu_again_after_one_failure(oracle_mod):
    """one failed GPU scan (HM_MINER_TEST_FAIL_AFTER=1) sends that
    Request to the host, and the next Request runs on a reopened GPU context
    instead of staying on the host for good."""
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=50)
    env = dict(ENV, HM_MINER_TEST_FAIL_AFTER="1", HM_MINER_RETRY_MS="0", HM_CPU_THREADS="8",
               HM_MINER_VERBOSE="1")
    p = subprocess.Popen([MINER, srv.hostport], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        cid = srv.accept(timeout=120)
        assert srv.read(cid, timeout=60) == bitcoin.marshal(bitcoin.NewJoin())
        assert _ask(srv, cid, "bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
        m = "thom yorke".encode()
        assert _ask(srv, cid, m, 19970000, 19971000) == oracle_mod.c_scan(m, 19970000, 19971000)
        assert _ask(srv, cid, "bradfitz", 0, 10**8) == _expected(oracle_mod, b"bradfitz", 0, 10**8)
    finally:
        srv.close()
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    err = p.stderr.read()
    assert p.returncode == 0, err
    lines = [l for l in err.splitlines() if "on gpu" in l or "on host" in l]
    assert [l.rsplit(" in ", 1)[0].split(" on ")[1] for l in lines] == ["gpu", "host", "gpu"], err
    assert "GPU (re)opened" in err, err


def test_miner_with_an_invisible_ordinal_falls_back(oracle_mod):
    """HIPMINER_DEVICES naming a GPU the box does not have makes
    hm_open fail with HM_ERR_INVALID; the miner treats it like no GPU and
    answers on the host (only a malformed list is fatal)."""
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=50)
    env = dict(ENV, HIPMINER_DEVICES="63", HM_CPU_THREADS="8")
    p = subprocess.Popen([MINER, srv.hostport], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        cid = srv.accept(timeout=120)
        assert srv.read(cid, timeout=60) == bitcoin.marshal(bitcoin.NewJoin())
        assert _ask(srv, cid, "bradfitz", 0, 9999) == (1419516646206828, 9898)
    finally:
        srv.close()
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    err = p.stderr.read()
    assert p.returncode == 0, err
    assert "NO GPU" in err and "invalid argument" in err, err


def test_deadline_on_a_two_device_context_and_checked_scans(oracle_mod):
    """The deadline covers every device of a context (Context([0, 0]): two
    shards, both polled) and hm_scan_checked; a generous deadline changes no
    answer, a 1-ms one abandons the context, whose close does not wait."""
    with _lib.Context([0, 0]) as c:
        c.set_option(_lib.HM_OPT_DEADLINE_MS, 60_000)
        m = b"thom yorke"
        assert c.scan_checked(m, 10**9 - 10**6, 10**9 + 10**6) == \
            oracle_mod.c_scan_sum(m, 10**9 - 10**6, 10**9 + 10**6)
        assert c.scan(b"bradfitz", 0, 2**32 - 1) == (5256245051, 1626825724)
        assert c.stats()["deadline_ms"] == 60_000
        c.set_option(_lib.HM_OPT_DEADLINE_MS, 1)
        with pytest.raises(_lib.HipMinerError) as ei:
            c.scan_checked(b"bradfitz", LO, HI)
        assert ei.value.rc == _lib.HM_ERR_TIMEOUT
        t = time.perf_counter()
    assert time.perf_counter() - t < 0.05  # hm_close of the abandoned context
