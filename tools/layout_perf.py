"""Throughput of the scan kernels across message lengths (dev tool, GPU box).

usage: python tools/layout_perf.py [d] [--all]
For each length L, 2^31 d-digit nonces [10^(d-1), 10^(d-1) + 2^31) (default
d = 10; --all: every length 0..127, else every 4th plus the boundary
lengths): the layout the planner picks (kind, W1, straddle, trailer; f / fe
for chained), kernel GH/s and the nominal roofline fraction 1552 * C * GH/s
/ 78.64 T (frac: C before hoisting; frac_eff: the compressions the kernel
executes, as bench.py prices them).  Where the planner picks the chained
layout for >= 5 final-block digits (round 3), the tiled kernel it replaced
is timed beside it (HM_OPT_TABLE_DIGITS = -1) as `tiled_GHs`."""
import json
import sys

sys.path.insert(0, '.')
from distributed_bitcoinminer_amd import _lib

PEAK = 256 * 4 * 32 * 2.4e9
args = [a for a in sys.argv[1:] if not a.startswith("--")]
d = int(args[0]) if args else 10
c = _lib.Context([0])
lo = 10**(d - 1)
hi = lo + 2**31 - 1
lengths = list(range(0, 128)) if "--all" in sys.argv else \
    list(range(0, 131, 4)) + [45, 46, 47, 53, 54, 55, 57, 58, 59, 63, 119, 120, 121, 122, 123]


def timed(m):
    c.scan(m, lo, hi)
    c.scan(m, lo, hi)
    st = c.stats()
    return st, st["dom_nonces"] / st["dom_kernel_ms"] / 1e6


for L in lengths:
    m = bytes(0x61 + (i % 26) for i in range(L))
    seg = max(_lib.debug_plan(m, lo, hi), key=lambda s: s["hi"] - s["lo"])
    st, gh = timed(m)
    row = {"len": L, "d": d, "kind": seg["kind"], "W1": seg["W1"], "straddle": seg["straddle"],
           "trailer": seg["trailer"], "f": seg["f"], "fe": seg["fe"], "C": st["dom_compressions"],
           "kernel": st["dom_kernel"], "kernel_GHs": round(gh, 2),
           "frac": round(gh * 1e9 * 1552 * st["dom_compressions"] / PEAK, 3),
           "frac_eff": round(gh * 1e9 * 1552 * st["dom_compressions_eff"] / PEAK, 3)}
    if seg["kind"] == _lib.HM_KIND_CHAINED and seg["f"] >= 5:
        c.set_option(_lib.HM_OPT_TABLE_DIGITS, -1)
        st2, gh2 = timed(m)
        c.set_option(_lib.HM_OPT_TABLE_DIGITS, 0)
        row.update(tiled_kernel=st2["dom_kernel"], tiled_GHs=round(gh2, 2))
    print(json.dumps(row), flush=True)
