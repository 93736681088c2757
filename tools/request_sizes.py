"""Wall rate of hm_scan against the request size (dev tool, GPU box): the
client's `[0, maxNonce]` for maxNonce = 10^3 .. 2^32 (bradfitz and the 120-B
message), median of 7 calls after one warm-up; small requests are latency-
bound (launches and their tails), large ones run at the kernel rate."""
import json
import random
import statistics
import sys
import time

sys.path.insert(0, ".")
from distributed_bitcoinminer_amd import _lib  # noqa: E402

rng = random.Random(440)
long120 = bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))
c = _lib.Context([0])
for name, m in (("bradfitz", b"bradfitz"), ("long120", long120)):
    for hi in (10**3, 10**4, 10**5, 10**6, 10**7, 10**8, 10**9, 2**32 - 1):
        c.scan(m, 0, hi)
        ts = []
        for _ in range(7):
            t = time.perf_counter()
            c.scan(m, 0, hi)
            ts.append(time.perf_counter() - t)
        st = c.stats()
        med = statistics.median(ts)
        print(json.dumps({"msg": name, "maxNonce": hi, "median_ms": round(med * 1e3, 4),
                          "GHs": round((hi + 1) / med / 1e9, 3), "launches": st["launches"],
                          "kernel_ms": round(st["kernel_ms"], 4)}), flush=True)
