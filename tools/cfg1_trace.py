"""Config 1's Request [0, 10^7+1] through hm_scan, 20 times after a warm-up
(dev tool, GPU box): run under rocprofv3 --kernel-trace (and --memory-copy-trace)
to see the fused launch's planner, scan, fold and readback on the timeline."""
import sys
import time

sys.path.insert(0, ".")
from distributed_bitcoinminer_amd import _lib  # noqa: E402

c = _lib.Context([0])
for i in range(21):
    t = time.perf_counter()
    assert c.scan(b"bradfitz", 0, 10**7 + 1) == (356393768206, 7645578)
    if i:
        print(f"{(time.perf_counter() - t) * 1e3:.4f} ms", flush=True)
c.close()
