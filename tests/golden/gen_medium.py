#!/usr/bin/env python3
"""Medium-size random fixtures (10^6..2*10^8 nonces per case) from the fast C
oracle (oracle/hm_oracle_fast.c, checked against oracle/hm_oracle.c by
tests/test_oracle_fast.py), computed in the build container.

Cases: for every message length 0..130 (so every tail layout the planner
picks: tiled W1 = 1..15 with and without straddle and trailer, chained f =
1..4, generic), one random range inside a random digit segment, plus ranges
across digit-count changes and next to 2^64-1.  Each records the scan result
and the coverage checksum (sum of keys mod 2^64, count) of hm_scan_checked.

Usage: python tests/golden/gen_medium.py [--threads N]  -> tests/golden/medium.json
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
OUT = os.path.join(ROOT, "tests", "golden", "medium.json")


def cases():
    rng = random.Random(0x5EED)
    out = []
    for L in range(0, 131):
        m = bytes(rng.randrange(256) for _ in range(L))
        d = rng.randrange(6, 21)
        dlo, dhi = 10 ** (d - 1), min(10 ** d - 1, MAX)
        w = min(int(10 ** rng.uniform(6, 7.7)), (dhi - dlo) // 2)
        lo = rng.randrange(dlo, dhi - w)
        out.append((f"len{L}_d{d}", m, lo, lo + w))
    for k in range(6, 20):  # digit-count changes
        L = rng.randrange(0, 131)
        m = bytes(rng.randrange(32, 127) for _ in range(L))
        w = int(10 ** rng.uniform(6, 7.3))
        c = 10 ** k
        a = rng.randrange(0, w)
        out.append((f"cross10^{k}_len{L}", m, c - a, c - a + w))
    for L in (0, 8, 45, 57, 120, 127):  # next to 2^64-1
        m = bytes(rng.randrange(32, 127) for _ in range(L))
        w = int(10 ** rng.uniform(6, 7.5))
        out.append((f"max_len{L}", m, MAX - w, MAX))
    big = bytes(rng.randrange(32, 127) for _ in range(8))  # a few large ones
    out.append(("big_d12", big, 123_456_789_012, 123_456_789_012 + 200_000_000))
    out.append(("big_d16", big, 5_432_109_876_543_210, 5_432_109_876_543_210 + 150_000_000))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    from oracle import oracle
    oracle.build()
    assert oracle.fast_available(), "needs the x86 SHA extensions"
    res = []
    t0 = time.time()
    for name, m, lo, hi in cases():
        (h, n), s, c = oracle.fast_scan_sum(m, lo, hi, threads=args.threads)
        res.append({"name": name, "msg_hex": m.hex(), "lo": str(lo), "hi": str(hi),
                    "hash": str(h), "nonce": str(n), "sum": str(s), "count": str(c)})
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/gen_medium.py (oracle/hm_oracle_fast.c)",
                   "cases": res}, f, indent=0)
    print(f"wrote {OUT}: {len(res)} cases, {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
