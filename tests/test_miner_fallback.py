"""hm_miner without a GPU (SURVEY §8(b) liveness): the native miner joins the
(fake) LSP server and still answers every Request correctly, scanning on
the host through hm_scan_cpu, and says so loudly on stderr.  The reference
miner always writes a Result (cmu440/bitcoin/miner/miner.go:60-62); without
this the unchanged server would wait out its 10-s drop timer and reassign
the chunk (server.go:326-376).  Runs on CPU: HIP_VISIBLE_DEVICES=-1 hides
any GPU."""
import os
import subprocess

from distributed_bitcoinminer_amd import bitcoin
from tests import lsp_harness as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MINER = os.path.join(ROOT, "distributed_bitcoinminer_amd", "hm_miner")
MAX = (1 << 64) - 1


def _ask(srv, cid, data, lower, upper):
    srv.write(cid, bitcoin.marshal(bitcoin.NewRequest(data, lower, upper)))
    res, err = bitcoin.unmarshal(srv.read(cid, timeout=120))
    assert err is None and res.Type == bitcoin.Result
    return res.Hash, res.Nonce


def test_miner_without_gpu_answers_on_the_host(oracle_mod, golden):
    assert os.path.exists(MINER), "build hm_miner first (__graft_entry__.build())"
    env = dict(os.environ, HM_LSP_EPOCH_MS="100", HM_LSP_EPOCH_LIMIT="50",
               HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1", HM_CPU_THREADS="4")
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=50)
    p = subprocess.Popen([MINER, srv.hostport], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        cid = srv.accept(timeout=60)
        assert srv.read(cid, timeout=60) == bitcoin.marshal(bitcoin.NewJoin())
        # config 1 through the server: client maxNonce 10^7 -> Request [0, 10^7+1]
        assert _ask(srv, cid, "bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
        for k in golden["miner_eval_kats"]:  # incl. the Upper = 2^64-1 wrap
            exp = (int(k["hash"]), int(k["nonce"]))
            assert _ask(srv, cid, bytes.fromhex(k["msg_hex"]), int(k["lower"]),
                        int(k["upper"])) == exp
        m = "thom yorke".encode()
        assert _ask(srv, cid, m, 19970000, 19971000) == oracle_mod.c_scan(m, 19970000, 19971000)
        assert _ask(srv, cid, b"x" * 120, MAX - 5000, MAX - 1) == \
            oracle_mod.c_scan(b"x" * 120, MAX - 5000, MAX - 1)
    finally:
        srv.close()
        try:
            p.wait(timeout=60)  # loses the server after EpochLimit epochs and exits
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    err = p.stderr.read()
    assert p.returncode == 0, err
    assert "NO GPU" in err and "hm_scan_cpu" in err, err


def _run_miner(env_extra, timeout=60):
    env = dict(os.environ, HM_LSP_EPOCH_MS="100", HM_LSP_EPOCH_LIMIT="20",
               HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1", HM_CPU_THREADS="2",
               **env_extra)
    srv = H.FakeLspServer(epoch_ms=100, epoch_limit=20)
    p = subprocess.Popen([MINER, srv.hostport], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    got = None
    try:
        if p.poll() is None:
            try:
                cid = srv.accept(timeout=10)
                assert srv.read(cid, timeout=60) == bitcoin.marshal(bitcoin.NewJoin())
                got = _ask(srv, cid, "bradfitz", 0, 9999)
            except Exception:  # the miner exited before joining
                pass
    finally:
        srv.close()
        try:
            p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return p.returncode, got, p.stderr.read()


def test_miner_device_list_parse_errors_are_fatal_the_rest_falls_back():
    """only a malformed HIPMINER_DEVICES ends hm_miner (exit 1,
    before it joins); a well-formed list naming a GPU that is not there --
    here none is visible -- falls back to the host scan like no GPU at all."""
    assert os.path.exists(MINER), "build hm_miner first (__graft_entry__.build())"
    for bad in ("x", "0,a", "-1", "1.5"):
        rc, got, err = _run_miner({"HIPMINER_DEVICES": bad})
        assert rc == 1 and got is None, (bad, rc, err)
        assert "bad HIPMINER_DEVICES" in err, err
    for ok in ("7", " 0 , 3 ", "63,"):
        rc, got, err = _run_miner({"HIPMINER_DEVICES": ok})
        assert rc == 0 and got == (1419516646206828, 9898), (ok, rc, err)
        assert "NO GPU" in err, err
