"""Interleaved A/B of fused-launch settings on small requests (dev tool, GPU box).

For every (HM_OPT_FUSED_FLAGS, HM_OPT_GRID_PER_CU, HM_OPT_FUSED_PARTS)
setting and every request,
the calls are interleaved round-robin so clock drift hits all settings
alike; prints the median hm_scan wall time and kernel time per pair and
request (one JSON line each).
usage: fused_ab.py REPS flags_list per_cu_list [parts_list]"""
import json
import random
import statistics
import sys
import time

sys.path.insert(0, ".")
from distributed_bitcoinminer_amd import _lib  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
FLAGS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2,3").split(",")]
PER_CU = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "2,3").split(",")]
PARTS = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "1").split(",")]
rng = random.Random(440)
long120 = bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))
REQS = [("cfg1", b"bradfitz", 0, 10**7 + 1), ("bf_1e6", b"bradfitz", 0, 10**6),
        ("d8", b"bradfitz", 10**7, 10**8 - 1), ("l120_1e7", long120, 0, 10**7),
        ("l120_1e8", long120, 0, 10**8)]
c = _lib.Context([0])
settings = [(f, p, n) for f in FLAGS for p in PER_CU for n in PARTS]
res = {(s, r[0]): ([], []) for s in settings for r in REQS}
ref = {}
for rep in range(REPS + 1):
    for s in settings:
        c.set_option(_lib.HM_OPT_FUSED_FLAGS, s[0])
        c.set_option(_lib.HM_OPT_GRID_PER_CU, s[1])
        c.set_option(_lib.HM_OPT_FUSED_PARTS, s[2])
        for name, m, lo, hi in REQS:
            t = time.perf_counter()
            out = c.scan(m, lo, hi)
            dt = time.perf_counter() - t
            assert ref.setdefault(name, out) == out, (name, s, out)
            if rep:
                st = c.stats()
                res[(s, name)][0].append(dt * 1e3)
                res[(s, name)][1].append(st["kernel_ms"])
for (s, name), (w, k) in res.items():
    print(json.dumps({"req": name, "flags": s[0], "per_cu": s[1], "parts": s[2],
                      "wall_ms": round(statistics.median(w), 4),
                      "kernel_ms": round(statistics.median(k), 4)}), flush=True)
