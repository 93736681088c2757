"""Whole-call sweep of the persistent grid (workgroups per CU) and the
segment stream count: wall GH/s of hm_scan and the dominant kernel's GH/s.
Dev tool (runs on the GPU box)."""
import json
import os
import random
import sys
import time

sys.path.insert(0, '.')
from distributed_bitcoinminer_amd import _lib

rng = random.Random(440)
m120 = bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))
WL = {"cfg2": (b"bradfitz", 0, 2**32 - 1), "cfg3": (m120, 0, 2**32 - 1),
      "d12": (b"bradfitz", 10**11, 10**11 + 2**34 - 1)}
c = _lib.Context([0])
for name, (msg, lo, hi) in WL.items():
    ref = None
    for per_cu in [int(x) for x in os.environ.get("HM_SWEEP_PER_CU", "2,3,4,0").split(",")]:
        for streams in [int(x) for x in os.environ.get("HM_SWEEP_STREAMS", "1,4").split(",")]:
            c.set_option(_lib.HM_OPT_GRID_PER_CU, per_cu)
            c.set_option(_lib.HM_OPT_STREAMS, streams)
            walls = []
            for _ in range(4):
                t = time.perf_counter()
                r = c.scan(msg, lo, hi)
                walls.append(time.perf_counter() - t)
                ref = ref or r
                assert r == ref, (r, ref)
            st = c.stats()
            w = sorted(walls[1:])[1]
            print(json.dumps({"wl": name, "per_cu": per_cu, "streams": streams,
                              "wall_GHs": round((hi - lo + 1) / w / 1e9, 3),
                              "dom_GHs": round(st["dom_nonces"] / st["dom_kernel_ms"] / 1e6, 3),
                              "grid": st["dom_grid"]}), flush=True)
