#!/usr/bin/env python3
"""Large-range fixtures, computed with the multi-threaded C oracle
(oracle/hm_oracle.c) in the build container (minutes on 8 cores).

  bradfitz [0, 2^32-1] -> (5256245051, 1626825724)   (249 s, 8 threads)
  BASELINE configs[2] 120-B message [0, 2^32-1]      (3 compressions per nonce)

Each case also records the coverage checksum of hm_scan_checked: the sum of
every key mod 2^64 and the count of nonces.

Usage: python tests/golden/gen_large.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

def long120() -> bytes:
    import random
    rng = random.Random(440)
    return bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))


CASES = [("bradfitz", b"bradfitz", 0, 2**32 - 1),
         ("cfg3_long120", long120(), 0, 2**32 - 1)]


def main():
    from oracle import oracle
    oracle.build()
    out = []
    for name, m, lo, hi in CASES:
        t = time.time()
        (h, n), sm, cnt = oracle.c_scan_sum(m, lo, hi, threads=os.cpu_count() or 1)
        out.append({"name": name, "msg_hex": m.hex(), "lo": str(lo), "hi": str(hi),
                    "hash": str(h), "nonce": str(n), "sum": str(sm), "count": str(cnt),
                    "oracle_seconds": round(time.time() - t, 1)})
        print(out[-1], flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "large.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
