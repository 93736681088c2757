"""Config 1 end to end (BASELINE configs[0]), timed: one GPU miner process
behind LSP, as the reference client -> server -> miner chain drives it.

The client's `bradfitz 10000000` reaches the miner as Request [0, 10^7+1]
(server.go:169 adds one; miner.go:52 scans inclusively).  A fake LSP server
(tests/lsp_harness.py, the role of the reference server / staff mtest) sends
that Request to a native `hm_miner` process (csrc/miner_main.cpp) and times
Request-write -> Result-read, i.e. JSON + LSP framing both ways over
localhost UDP plus the whole hm_scan.  Beside it: the same miner Request on
the host, one thread of the C restatement of the reference loop
(oracle/hm_oracle.c), which stands in for one Go miner (no Go toolchain;
SURVEY §8(c)).  Prints one JSON line.

usage: python tools/e2e_cfg1.py [--reps 20]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoinminer_amd import bitcoin  # noqa: E402
from tests import lsp_harness as H  # noqa: E402

MINER = os.path.join(ROOT, "distributed_bitcoinminer_amd", "hm_miner")
EXPECT = (356393768206, 7645578)  # SURVEY App. B; tests/golden/golden.json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    env = dict(os.environ, HIPMINER_DEVICES="0")
    srv = H.FakeLspServer(epoch_ms=2000, epoch_limit=5)  # lsp.Params defaults (params.go:8-13)
    p = subprocess.Popen([MINER, srv.hostport], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    lat = []
    try:
        t = time.perf_counter()
        cid = srv.accept(timeout=120)
        assert srv.read(cid, timeout=120) == bitcoin.marshal(bitcoin.NewJoin())
        join_s = time.perf_counter() - t
        req = bitcoin.marshal(bitcoin.NewRequest("bradfitz", 0, 10**7 + 1))
        for i in range(a.reps + 1):
            t = time.perf_counter()
            srv.write(cid, req)
            res, err = bitcoin.unmarshal(srv.read(cid, timeout=120))
            dt = time.perf_counter() - t
            assert err is None and (res.Hash, res.Nonce) == EXPECT, (res, err)
            if i:  # the first Request loads the scan code object: reported apart
                lat.append(dt)
            else:
                first = dt
    finally:
        srv.close()
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    lat.sort()
    from oracle import oracle
    oracle.build()
    t = time.perf_counter()
    cpu = oracle.c_miner_eval(b"bradfitz", 0, 10**7 + 1, threads=1)
    cpu_s = time.perf_counter() - t
    assert cpu == EXPECT, cpu
    med = lat[len(lat) // 2]
    print(json.dumps({
        "config": "cfg1: client 'bradfitz' maxNonce 10^7 -> miner Request [0, 10^7+1] over LSP",
        "result": {"hash": EXPECT[0], "nonce": EXPECT[1]},
        "gpu_miner_request_ms": {"median": round(med * 1e3, 3), "min": round(lat[0] * 1e3, 3),
                                 "max": round(lat[-1] * 1e3, 3), "reps": len(lat),
                                 "first_request_ms": round(first * 1e3, 3),
                                 "join_ms": round(join_s * 1e3, 3)},
        "cpu_miner_request_ms": round(cpu_s * 1e3, 1),
        "cpu_miner": "oracle/hm_oracle.c, 1 thread (one reference miner's per-nonce work)",
        "speedup_median": round(cpu_s / med, 1),
    }), flush=True)


if __name__ == "__main__":
    main()
