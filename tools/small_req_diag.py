"""Where a small request's time goes (dev tool, GPU box; round 5).

configs[0]'s Request is the client's [0, 10^7] plus the server's +1
(server.go:169): eight digit segments, the 7-digit one holding 90 % of the
nonces.  For that request, and for its 7-digit segment alone, print the
median hm_scan wall time, the kernel union and the dominant kernel's summed
time, per stream count and persistent-grid size, with the fused launch
(HM_OPT_FUSED) on or off.  One JSON line per case.
usage: small_req_diag.py REPS [fused list] [streams list] [grid_per_cu list]"""
import json
import statistics
import sys
import time

sys.path.insert(0, ".")
from distributed_bitcoinminer_amd import _lib  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 15
CASES = [("cfg1", 0, 10**7 + 1), ("d7", 10**6, 10**7 - 1), ("d8", 10**7, 10**8 - 1)]
c = _lib.Context([0])
m = b"bradfitz"
FUSED = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0").split(",")]
STREAMS = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "4,1").split(",")]
PER_CU = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "0,2,4,8").split(",")]
for fused in FUSED:
  c.set_option(_lib.HM_OPT_FUSED, fused)
  for streams in STREAMS:
    c.set_option(_lib.HM_OPT_STREAMS, streams)
    for per_cu in PER_CU:
        c.set_option(_lib.HM_OPT_GRID_PER_CU, per_cu)
        for name, lo, hi in CASES:
            c.scan(m, lo, hi)
            ts, ks, ds = [], [], []
            for _ in range(REPS):
                t = time.perf_counter()
                c.scan(m, lo, hi)
                ts.append(time.perf_counter() - t)
                st = c.stats()
                ks.append(st["kernel_ms"])
                ds.append(st["dom_kernel_ms"])
            med = statistics.median(ts)
            print(json.dumps({"case": name, "fused": fused, "streams": streams, "grid_per_cu": per_cu,
                              "median_ms": round(med * 1e3, 4),
                              "GHs": round((hi - lo + 1) / med / 1e9, 3),
                              "kernel_ms": round(statistics.median(ks), 4),
                              "dom_kernel_ms": round(statistics.median(ds), 4),
                              "launches": st["launches"], "dom_grid": st["dom_grid"],
                              "dom_kernel": st["dom_kernel"],
                              "enqueue_ms": round(st["enqueue_ms"], 4)}), flush=True)
