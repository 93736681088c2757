#!/usr/bin/env python3
"""Large-range fixtures, computed with the multi-threaded C oracle
(oracle/hm_oracle.c) in the build container (minutes on 8 cores).

  bradfitz [0, 2^32-1] -> (5256245051, 1626825724)   (249 s, 8 threads)

Usage: python tests/golden/gen_large.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CASES = [("bradfitz", b"bradfitz", 0, 2**32 - 1)]


def main():
    from oracle import oracle
    oracle.build()
    out = []
    for name, m, lo, hi in CASES:
        t = time.time()
        h, n = oracle.c_scan(m, lo, hi, threads=os.cpu_count() or 1)
        out.append({"name": name, "msg_hex": m.hex(), "lo": str(lo), "hi": str(hi),
                    "hash": str(h), "nonce": str(n), "oracle_seconds": round(time.time() - t, 1)})
    with open(os.path.join(ROOT, "tests", "golden", "large.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
