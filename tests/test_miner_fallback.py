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
