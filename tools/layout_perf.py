"""Throughput of the scan kernels across message lengths (dev tool, GPU box).
For each length L, 2^31 ten-digit nonces [10^9, 10^9 + 2^31): the layout the
planner picks (kind, W1, straddle, trailer), kernel GH/s and the nominal
roofline fraction 1552 * C * GH/s / 78.64 T (frac: C before hoisting; frac_eff: the
compressions the kernel executes, as bench.py prices them)."""
import json
import sys

sys.path.insert(0, '.')
from distributed_bitcoinminer_amd import _lib

PEAK = 256 * 4 * 32 * 2.4e9
c = _lib.Context([0])
lo, hi = 10**9, 10**9 + 2**31 - 1
for L in list(range(0, 131, 4)) + [45, 46, 47, 53, 54, 55, 57, 63, 119, 120, 121]:
    m = bytes(0x61 + (i % 26) for i in range(L))
    seg = _lib.debug_plan(m, lo, hi)[0]
    c.scan(m, lo, hi)
    r = c.scan(m, lo, hi)
    st = c.stats()
    gh = st["dom_nonces"] / st["dom_kernel_ms"] / 1e6
    print(json.dumps({"len": L, "kind": seg["kind"], "W1": seg["W1"], "straddle": seg["straddle"],
                      "trailer": seg["trailer"], "C": st["dom_compressions"], "kernel": st["dom_kernel"],
                      "kernel_GHs": round(gh, 2),
                      "frac": round(gh * 1e9 * 1552 * st["dom_compressions"] / PEAK, 3),
                      "frac_eff": round(gh * 1e9 * 1552 * st["dom_compressions_eff"] / PEAK, 3)}),
          flush=True)
