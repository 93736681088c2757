"""Native LSP client (csrc/lsp_client.cpp) and wire codec (csrc/wire.cpp):
byte parity with the reference's formats and protocol behaviour against a
fake LSP server (tests/lsp_harness.py), including datagram loss.  CPU only."""
import os
import random
import subprocess

import pytest

from distributed_bitcoinminer_amd import bitcoin
from tests import lsp_harness as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "build", "hipminer", "hm_lsp_tool")


@pytest.fixture(scope="module")
def tool():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "distributed_bitcoinminer_amd", "csrc"),
                    "tools"], check=True)
    return TOOL


def run(tool, *args, env=None):
    return subprocess.run([tool, *args], capture_output=True, text=True, check=True,
                          env=env, timeout=120).stdout.strip()


def test_checksum_matches_restatement(tool):
    rng = random.Random(5)
    for _ in range(60):
        n = rng.randrange(0, 90)
        p = bytes(rng.randrange(256) for _ in range(n))
        conn, seq = rng.randrange(0, 1 << 31), rng.randrange(0, 1 << 31)
        assert int(run(tool, "checksum", str(conn), str(seq), p.hex() or "-")) == \
            H.checksum(conn, seq, n, p)


def test_encode_decode_parity(tool):
    payload = b'{"Type":0,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}'
    assert run(tool, "encode", "1", "7", "3", payload.hex()).encode() == H.encode(1, 7, 3, payload)
    assert run(tool, "encode", "2", "7", "3", "-").encode() == H.encode(2, 7, 3, None)
    assert run(tool, "encode", "0", "0", "0", "-").encode() == H.encode(0, 0, 0, None)
    good = H.encode(1, 9, 4, b"abcde").decode()
    assert run(tool, "decode", good) == f"1 9 4 5 {H.checksum(9, 4, 5, b'abcde')} 1 {b'abcde'.hex()}"
    # over-long payload is truncated to Size; short or corrupted ones fail integrity
    long = good.replace('"Size":5', '"Size":3').replace(
        f'"Checksum":{H.checksum(9, 4, 5, b"abcde")}', f'"Checksum":{H.checksum(9, 4, 3, b"abc")}')
    assert run(tool, "decode", long).endswith(f"1 {b'abc'.hex()}")
    assert run(tool, "decode", good.replace('"Size":5', '"Size":6')).split()[5] == "0"
    assert run(tool, "decode", good.replace('"SeqNum":4', '"SeqNum":5')).split()[5] == "0"


def test_json_string_matches_python_mirror(tool):
    rng = random.Random(8)
    samples = [b"", b"bradfitz", b'<&>"\\\n\r\t\x00\x1f\x7f', "é中  ".encode(),
               b"\xff\xfe\xc3", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xe2\x82"]
    samples += [bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40))) for _ in range(80)]
    for s in samples:
        assert run(tool, "jsonstr", s.hex() or "-") == bitcoin._go_json_string(s), s


def test_bitcoin_codec_roundtrip(tool):
    for m in [bitcoin.NewRequest("bradfitz", 0, 9999), bitcoin.NewResult(2**64 - 1, 0),
              bitcoin.NewJoin(), bitcoin.NewRequest("a<b>& é", 2**64 - 6, 2**64 - 1)]:
        js = bitcoin.marshal(m).decode()
        assert run(tool, "bitcoin", js) == "1 " + js
    # case-insensitive keys, unknown and nested keys ignored, bad fields left zero
    out = run(tool, "bitcoin", '{"type":1,"DATA":"x","lower":-1,"Upper":1.5,"z":{"a":[1,2]},"Nonce":7}')
    assert out == '1 {"Type":1,"Data":"x","Lower":0,"Upper":0,"Hash":0,"Nonce":7}'


@pytest.mark.parametrize("window,drop", [(1, 0.0), (4, 0.0), (1, 0.2), (3, 0.25)])
def test_echo_client_against_fake_server(tool, window, drop):
    srv = H.FakeLspServer(epoch_ms=50, epoch_limit=20, window=window, drop_send=drop,
                          drop_recv=drop, seed=window)
    env = dict(os.environ, HM_LSP_EPOCH_MS="50", HM_LSP_EPOCH_LIMIT="20", HM_LSP_WINDOW=str(window))
    p = subprocess.Popen([tool, "echo", srv.hostport], stdout=subprocess.PIPE, text=True, env=env)
    try:
        cid = srv.accept(timeout=30)
        assert srv.read(cid, timeout=30) == b"hello"
        msgs = [f"m{i}-".encode() * (i % 7 + 1) for i in range(25)]
        for m in msgs:
            srv.write(cid, m)
        got = [srv.read(cid, timeout=60) for _ in msgs]
        assert got == msgs  # in order, exactly once, despite loss
        srv.write(cid, b"quit")
        out, _ = p.communicate(timeout=60)
        assert p.returncode == 0 and "echoed 25" in out
    finally:
        if p.poll() is None:
            p.kill()
        srv.close()


def test_connect_fails_without_server(tool):
    import socket
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))  # a port nobody answers on
    port = s.getsockname()[1]
    env = dict(os.environ, HM_LSP_EPOCH_MS="30", HM_LSP_EPOCH_LIMIT="3")
    r = subprocess.run([tool, "echo", f"127.0.0.1:{port}"], capture_output=True, text=True,
                       env=env, timeout=30)
    s.close()
    assert r.returncode == 3 and "connect failed" in r.stdout


def test_client_detects_lost_server(tool):
    srv = H.FakeLspServer(epoch_ms=40, epoch_limit=4)
    env = dict(os.environ, HM_LSP_EPOCH_MS="40", HM_LSP_EPOCH_LIMIT="4")
    p = subprocess.Popen([tool, "echo", srv.hostport], stdout=subprocess.PIPE, text=True, env=env)
    try:
        cid = srv.accept(timeout=30)
        assert srv.read(cid, timeout=30) == b"hello"
        srv.close()  # server vanishes: the client must give up after EpochLimit epochs
        out, _ = p.communicate(timeout=30)
        assert p.returncode == 0 and "echoed 0" in out
    finally:
        if p.poll() is None:
            p.kill()


# "spec" servers beat at epoch ticks only when idle, so their gaps reach two
# epochs: EpochLimit 2 is borderline there for any client (the reference's
# 2-epoch drop timer included), hence 3.
@pytest.mark.parametrize("heartbeat,limit", [("reference", 5), ("reference", 2), ("spec", 5),
                                             ("spec", 3)])
def test_idle_connection_stays_alive(tool, heartbeat, limit):
    """An idle miner waits between client requests for as long as the server is
    quiet.  Against the reference server's timers (reminder only after a
    silent epoch, every message resets them) a client that beat every epoch
    would keep the server silent and drop it; both sides must survive many
    EpochLimits of idleness."""
    import time
    # 80-ms epochs: an EpochLimit-2 drop timer of 160 ms leaves room for the
    # scheduling jitter of a loaded host (40-ms epochs flaked under pytest -n)
    epoch = 80
    srv = H.FakeLspServer(epoch_ms=epoch, epoch_limit=limit, heartbeat=heartbeat)
    env = dict(os.environ, HM_LSP_EPOCH_MS=str(epoch), HM_LSP_EPOCH_LIMIT=str(limit))
    p = subprocess.Popen([tool, "echo", srv.hostport], stdout=subprocess.PIPE, text=True, env=env)
    try:
        cid = srv.accept(timeout=30)
        assert srv.read(cid, timeout=30) == b"hello"
        time.sleep(25 * epoch / 1000)                    # 25 idle epochs
        assert p.poll() is None and not srv.is_lost(cid)
        srv.write(cid, b"ping")
        assert srv.read(cid, timeout=30) == b"ping"
        srv.write(cid, b"quit")
        out, _ = p.communicate(timeout=30)
        assert p.returncode == 0 and "echoed 1" in out
    finally:
        if p.poll() is None:
            p.kill()
        srv.close()


def test_bitcoin_codec_go_error_semantics(tool):
    # syntax error: Go decodes nothing (checkValid runs first)
    assert run(tool, "bitcoin", '{"Type":1,"Data":"x","Lower":5') == \
        '0 {"Type":0,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}'
    assert run(tool, "bitcoin", 'garbage') == \
        '0 {"Type":0,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}'
    # type error: the other fields still decode
    assert run(tool, "bitcoin", '{"Data":"abc","Lower":5,"Upper":"x"}') == \
        '1 {"Type":0,"Data":"abc","Lower":5,"Upper":0,"Hash":0,"Nonce":0}'
    # the Python mirror agrees
    m, err = bitcoin.unmarshal(b'{"Type":1,"Data":"x","Lower":5')
    assert err is not None and m == bitcoin.Message()
    m, err = bitcoin.unmarshal(b'{"Data":"abc","Lower":5,"Upper":"x"}')
    assert err is not None and (m.Data, m.Lower, m.Upper) == (b"abc", 5, 0)
