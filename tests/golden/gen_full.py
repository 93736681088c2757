#!/usr/bin/env python3
"""Full-size fixtures for BASELINE configs[3] and configs[4], computed in the
build container by the fast C oracle (oracle/hm_oracle_fast.c: SHA extensions,
midstate; checked against oracle/hm_oracle.c by tests/test_oracle_fast.py).

* cfg4: "bradfitz" over [0, 2^40).  The range is cut at every bound of
  hm_partition(msg, 0, 2^40-1, n) for n = 1..8 and at every multiple of 2^34;
  each piece records (min hash, nonce, sum of keys mod 2^64, count).  Any
  shard made of whole pieces -- in particular every rank's shard of a 1..8-GPU
  run -- is pinned by merging its pieces.  About 3 h on 8 cores.
* weak: bench.py's weak-scaling ranges: rank r of N scans [r*2^32,
  (r+1)*2^32) of configs[1]'s "bradfitz" and configs[2]'s 120-B message, so
  the whole job of an N-GPU run is [0, N*2^32); one piece per 2^32 for
  r = 0..7 pins N = 1..8.  About 20 min.
* cfg5: the four SURVEY messages, each as a client Request
  [2^64-1-2^34, 2^64-2] split by the reference server into 8 miner chunks
  (server.go:165-205, restated in server_model.load_balance); every chunk's
  miner result (miner.go:46-59 incl. the Upper+1 wrap, :52) and the client's
  merged answer (server.go:140-141, 273-276).

Progress is appended to build/gen_full.progress.jsonl so an interrupted run
resumes; the result is tests/golden/full_size.json.

Usage: python tests/golden/gen_full.py [--threads N]
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
MAX = (1 << 64) - 1
PROGRESS = os.path.join(ROOT, "build", "gen_full.progress.jsonl")
OUT = os.path.join(ROOT, "tests", "golden", "full_size.json")


def long120() -> bytes:
    rng = random.Random(440)
    return bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))


CFG5_MSGS = [("bradfitz", b"bradfitz"), ("thom_yorke", b"thom yorke"),
             ("long120", long120()), ("jonny_greenwood", b"jonny greenwood")]
CFG5_LO, CFG5_UP, CFG5_MINERS = MAX - 1 - (1 << 34), MAX - 1, 8
CFG4_MSG, CFG4_LO, CFG4_HI = b"bradfitz", 0, (1 << 40) - 1


def cfg4_pieces():
    from distributed_bitcoinminer_amd import _lib
    cuts = {CFG4_LO, CFG4_HI + 1}
    for n in range(1, 9):
        for sh in _lib.partition(CFG4_MSG, CFG4_LO, CFG4_HI, n):
            if sh is not None:
                cuts.add(sh[0])
                cuts.add(sh[1] + 1)
    cuts |= set(range(CFG4_LO, CFG4_HI + 1, 1 << 34))
    cuts = sorted(cuts)
    return [(a, b - 1) for a, b in zip(cuts, cuts[1:])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--cfg5-only", action="store_true",
                    help="write full_size.json with the cfg5 section only (keeps an existing cfg4)")
    args = ap.parse_args()
    from oracle import oracle
    from distributed_bitcoinminer_amd import server_model as sm
    oracle.build()
    assert oracle.fast_available(), "needs the x86 SHA extensions"
    os.makedirs(os.path.dirname(PROGRESS), exist_ok=True)
    done = {}
    if os.path.exists(PROGRESS):
        for line in open(PROGRESS):
            r = json.loads(line)
            done[r["key"]] = r

    def piece(key, msg, lo, hi):
        if key in done:
            return done[key]
        t = time.time()
        (h, n), s, c = oracle.fast_scan_sum(msg, lo, hi, threads=args.threads)
        r = {"key": key, "lo": str(lo), "hi": str(hi), "hash": str(h), "nonce": str(n),
             "sum": str(s), "count": str(c), "seconds": round(time.time() - t, 1)}
        with open(PROGRESS, "a") as f:
            f.write(json.dumps(r) + "\n")
        done[key] = r
        print(key, r["seconds"], "s", flush=True)
        return r

    out = {"generator": "tests/golden/gen_full.py (oracle/hm_oracle_fast.c)"}
    # cfg5 first (minutes), then cfg4 (hours)
    cfg5 = []
    for name, msg in CFG5_MSGS:
        chunks = sm.load_balance(CFG5_LO, CFG5_UP, CFG5_MINERS)
        res = []
        for i, (a, b) in enumerate(chunks):
            up = (b + 1) & MAX                      # miner.go:52
            if not a < up:
                r = {"lo": str(a), "hi": str(b), "hash": str(MAX), "nonce": "0",
                     "sum": "0", "count": "0"}
            else:
                r = dict(piece(f"cfg5:{name}:{i}", msg, a, up - 1))
                r.pop("key")
                r["lo"], r["hi"] = str(a), str(b)   # the Request as sent
            res.append(r)
        merged = sm.merge_in_arrival_order([(int(r["hash"]), int(r["nonce"])) for r in res])
        cfg5.append({"name": name, "msg_hex": msg.hex(), "lower": str(CFG5_LO),
                     "upper": str(CFG5_UP), "miners": CFG5_MINERS, "chunks": res,
                     "client_result": {"hash": str(merged[0]), "nonce": str(merged[1])}})
    out["cfg5"] = cfg5
    if not args.cfg5_only:
        weak = []
        for name, msg in (("bradfitz", CFG4_MSG), ("long120", long120())):
            pcs = []
            for r in range(8):
                p = dict(piece(f"weak:{name}:{r}", msg, r << 32, ((r + 1) << 32) - 1))
                p.pop("key")
                pcs.append(p)
            weak.append({"name": name, "msg_hex": msg.hex(), "pieces": pcs})
        out["weak"] = weak
    if args.cfg5_only:
        if os.path.exists(OUT):
            with open(OUT) as f:
                old = json.load(f)
            if "cfg4" in old:
                out["cfg4"] = old["cfg4"]
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1)
        print("wrote", OUT, "(cfg5)")
        return
    pieces = []
    for a, b in cfg4_pieces():
        r = dict(piece(f"cfg4:{a}", CFG4_MSG, a, b))
        r.pop("key")
        pieces.append(r)
    best = min((int(p["hash"]), int(p["nonce"])) for p in pieces)
    out["cfg4"] = {"msg_hex": CFG4_MSG.hex(), "lo": str(CFG4_LO), "hi": str(CFG4_HI),
                   "pieces": pieces,
                   "whole": {"hash": str(best[0]), "nonce": str(best[1]),
                             "sum": str(sum(int(p["sum"]) for p in pieces) & MAX),
                             "count": str(sum(int(p["count"]) for p in pieces))}}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT, out["cfg4"]["whole"])


if __name__ == "__main__":
    main()
