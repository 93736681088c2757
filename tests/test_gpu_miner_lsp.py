"""End to end on the GPU: native hm_miner processes join an LSP server and
answer Requests, as the staff `mtest` checks a miner (p1/README.md:139-141),
and several miners under the reference server's chunking/merge model
(server.go:165-205, 273-276; config-5 style, near 2^64-1)."""
import os
import subprocess

import pytest

from distributed_bitcoinminer_amd import bitcoin, server_model as sm
from tests import lsp_harness as H

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MINER = os.path.join(ROOT, "distributed_bitcoinminer_amd", "hm_miner")
MAX = (1 << 64) - 1
ENV = dict(os.environ, HM_LSP_EPOCH_MS="100", HM_LSP_EPOCH_LIMIT="50", HIPMINER_DEVICES="0")


def _spawn(srv):
    assert os.path.exists(MINER), "build hm_miner first (__graft_entry__.build())"
    return subprocess.Popen([MINER, srv.hostport], env=ENV, stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)


def _ask(srv, cid, data, lower, upper):
    srv.write(cid, bitcoin.marshal(bitcoin.NewRequest(data, lower, upper)))
    res, err = bitcoin.unmarshal(srv.read(cid, timeout=120))
    assert err is None and res.Type == bitcoin.Result
    return res.Hash, res.Nonce


def test_miner_join_and_requests(oracle_mod, golden):
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=50)
    p = _spawn(srv)
    try:
        cid = srv.accept(timeout=120)
        assert srv.read(cid, timeout=60) == bitcoin.marshal(bitcoin.NewJoin())
        # config 1 through the server: client maxNonce 10^7 -> miner Request [0, 10^7+1]
        assert _ask(srv, cid, "bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
        for k in golden["miner_eval_kats"]:
            exp = (int(k["hash"]), int(k["nonce"]))
            assert _ask(srv, cid, bytes.fromhex(k["msg_hex"]), int(k["lower"]), int(k["upper"])) == exp
        m = "thom yorke".encode()
        assert _ask(srv, cid, m, 19970000, 19971000) == oracle_mod.c_scan(m, 19970000, 19971000)
        weird = 'a<b>&"é '.encode()
        assert _ask(srv, cid, weird, 5, 5000) == oracle_mod.c_scan(weird, 5, 5000)
        # malformed Requests: decode errors are ignored (miner.go:45), so the
        # miner scans the zero Request [0, 0] of "" or the fields that decoded
        for payload, exp in [(b"garbage", (oracle_mod.c_hash(b"", 0), 0)),
                             (b'{"Data":"abc","Lower":5,"Upper":"x"}', (MAX, 0)),
                             (b'{"Data":"abc","Lower":5,"Upper":7,"Type":"?"}',
                              oracle_mod.c_scan(b"abc", 5, 7))]:
            srv.write(cid, payload)
            res, err = bitcoin.unmarshal(srv.read(cid, timeout=120))
            assert err is None and (res.Hash, res.Nonce) == exp, payload
    finally:
        srv.close()
        try:
            p.wait(timeout=60)  # loses the server after EpochLimit epochs and exits
        except subprocess.TimeoutExpired:
            p.kill()
    assert p.returncode == 0, p.stderr.read() if p.stderr else ""


def test_three_miners_under_server_model(oracle_mod):
    """Three GPU miner processes; the fake server splits each client request the
    way server.go:165-205 does and merges in arrival order (:273-276)."""
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=50)
    procs = [_spawn(srv) for _ in range(3)]
    try:
        cids = [srv.accept(timeout=120) for _ in procs]
        for c in cids:
            assert srv.read(c, timeout=60) == bitcoin.marshal(bitcoin.NewJoin())
        reqs = [(b"bradfitz", MAX - 1 - 3_000_000, MAX - 1),
                (b"jonny greenwood", 0, 9999),
                (b"thom yorke", 10**19, 10**19 + 2_000_000)]
        for data, lo, up in reqs:
            chunks = sm.load_balance(lo, up, len(cids))
            for c, (a, b) in zip(cids, chunks):
                srv.write(c, bitcoin.marshal(bitcoin.NewRequest(data, a, b)))
            results = []
            for c, _ in zip(cids, chunks):
                r, _ = bitcoin.unmarshal(srv.read(c, timeout=120))
                results.append((r.Hash, r.Nonce))
            got = sm.merge_in_arrival_order(results)
            # expected: the union of what the miners scan (the last chunk of the
            # near-2^64 request ends at 2^64-1 and scans nothing)
            exp = sm.expected_client_result(
                data, lo, up, len(cids),
                lambda d, a, b: oracle_mod.c_miner_eval(d, a, b))
            assert got == exp, (data, lo, up)
    finally:
        srv.close()
        for p in procs:
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                p.kill()


def test_config5_eight_miners_near_max():
    """Config 5 at the SURVEY width: 8 GPU miner processes, the four SURVEY
    messages as queued client requests [2^64-1-2^34, 2^64-2] (20-digit
    nonces).  Each request is split as server.go:165-205 splits it; every
    miner's Result and the merged answer (server.go:273-276) must equal the
    oracle's (tests/golden/full_size.json, tests/golden/gen_full.py)."""
    import json
    from distributed_bitcoinminer_amd import _lib
    with open(os.path.join(ROOT, "tests", "golden", "full_size.json")) as f:
        cases = json.load(f)["cfg5"]
    assert len(cases) == 4
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=100)
    procs = [_spawn(srv) for _ in range(8)]
    try:
        cids = [srv.accept(timeout=180) for _ in procs]
        for c in cids:
            assert srv.read(c, timeout=120) == bitcoin.marshal(bitcoin.NewJoin())
        for case in cases:                    # FIFO: one client request at a time
            data = bytes.fromhex(case["msg_hex"])
            lo, up = int(case["lower"]), int(case["upper"])
            assert (lo, up) == (MAX - 1 - (1 << 34), MAX - 1)
            chunks = sm.load_balance(lo, up, len(cids))
            assert [(int(c["lo"]), int(c["hi"])) for c in case["chunks"]] == chunks
            assert chunks[-1][1] == MAX
            for c, (a, b) in zip(cids, chunks):
                srv.write(c, bitcoin.marshal(bitcoin.NewRequest(data, a, b)))
            got = []
            for c in cids:
                r, _ = bitcoin.unmarshal(srv.read(c, timeout=300))
                got.append((r.Hash, r.Nonce))
            exp = [(int(c["hash"]), int(c["nonce"])) for c in case["chunks"]]
            assert got == exp, case["name"]   # exp[-1] == (MAX, 0): the wrap (miner.go:52)
            res = case["client_result"]
            merged = sm.merge_in_arrival_order(got)
            assert merged == (int(res["hash"]), int(res["nonce"]))
            assert _lib.host_hash(data, merged[1]) == merged[0]
    finally:
        srv.close()
        for p in procs:
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                p.kill()


def test_server_sim_reassigns_a_killed_miner(oracle_mod):
    """The server's whole event loop (ServerSim, server.go:207-400) over the
    fake LSP transport with 3 GPU miner processes.  One miner is killed before
    its chunk arrives: the LSP layer reports it lost after EpochLimit silent
    epochs (-> the server's drop path, :326-376), its chunk is re-sent to a
    surviving miner, and the client's Result equals the A-inv-7 model."""
    import signal
    import time
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=20)
    procs = [_spawn(srv) for _ in range(3)]
    client = 10_000                       # the client's conn id (not an LSP peer here)
    data, lo, up = b"jonny greenwood", 10**9, 10**9 + 30_000_000
    try:
        cids = [srv.accept(timeout=180) for _ in procs]
        sim = sm.ServerSim()
        for c in cids:
            assert srv.read(c, timeout=120) == bitcoin.marshal(bitcoin.NewJoin())
            assert sim.miner_join(c) == []
        # accept order need not follow spawn order, so the killed miner's conn
        # is identified by its loss, not assumed
        procs[1].send_signal(signal.SIGKILL)
        procs[1].wait(timeout=30)
        pending = list(sim.client_request(client, data, lo, up))
        answers, final, dropped = [], None, set()
        deadline = time.monotonic() + 120
        while final is None and time.monotonic() < deadline:
            for c, msg in pending:
                if c == client:
                    final = (msg.Hash, msg.Nonce)
                else:
                    srv.write(c, bitcoin.marshal(msg))
            pending = []
            for c in cids:
                if c in dropped:
                    continue
                if srv.is_lost(c):
                    dropped.add(c)
                    pending += sim.drop(c)
                    continue
                try:
                    raw = srv.by_id[c].ready.get(timeout=0.05)
                except Exception:
                    continue
                res, err = bitcoin.unmarshal(raw)
                assert err is None and res.Type == bitcoin.Result
                answers.append((c, (res.Hash, res.Nonce)))
                pending += sim.miner_result(c, res.Hash, res.Nonce)
        assert final is not None, ("no Result within the deadline", answers, dropped,
                                   sim.curr and (sim.curr.responsible, sim.curr.responses),
                                   [(m.miner_id, m.available) for m in sim.miners],
                                   [m.miner_id for m in sim.dropped],
                                   {c: srv.is_lost(c) for c in cids}, pending,
                                   [p.poll() for p in procs])
        assert len(dropped) == 1              # exactly the killed miner
        assert len(answers) == 3              # two own chunks + the reassigned one
        assert final == sm.merge_in_arrival_order([r for _, r in answers])
        exp = sm.expected_client_result(data, lo, up, 3,
                                        lambda d, a, b: oracle_mod.c_miner_eval(d, a, b))
        assert final == exp
    finally:
        srv.close()
        for p in procs:
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                p.kill()


def test_miner_falls_back_to_host_after_a_failed_gpu_scan(oracle_mod):
    """SURVEY §8(b) liveness, mid-run: the GPU answers the first Request, the
    second GPU scan fails (HM_MINER_TEST_FAIL_AFTER=1 injects HM_ERR_HIP), and
    that Request is answered on the host (hm_scan_cpu) and every later one
    too (on the host until the 1-s retry backoff passes, then on a reopened
    GPU context), with the oracle's Results; the miner says so on stderr."""
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=50)
    env = dict(ENV, HM_MINER_TEST_FAIL_AFTER="1", HM_CPU_THREADS="8")
    p = subprocess.Popen([MINER, srv.hostport], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        cid = srv.accept(timeout=120)
        assert srv.read(cid, timeout=60) == bitcoin.marshal(bitcoin.NewJoin())
        assert _ask(srv, cid, "bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)  # GPU
        m = "thom yorke".encode()
        assert _ask(srv, cid, m, 19970000, 19971000) == oracle_mod.c_scan(m, 19970000, 19971000)
        assert _ask(srv, cid, b"x" * 120, MAX - 5000, MAX - 1) == \
            oracle_mod.c_scan(b"x" * 120, MAX - 5000, MAX - 1)
        assert _ask(srv, cid, "bradfitz", 0, MAX) == (MAX, 0)  # Upper+1 wraps: no scan
    finally:
        srv.close()
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    err = p.stderr.read()
    assert p.returncode == 0, err
    assert "GPU scan FAILED" in err and "hm_scan_cpu" in err, err
    assert "NO GPU" not in err, err
