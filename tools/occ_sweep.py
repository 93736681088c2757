"""Occupancy sweep of the scan kernels with one binary: the persistent grid
is k workgroups (= k waves/SIMD) per CU.  Dev tool."""
import sys, json
sys.path.insert(0, '.')
from distributed_bitcoinminer_amd import _lib
msg = sys.argv[1].encode() if len(sys.argv) > 1 else b"bradfitz"
lo, hi = 10**9, 2**32 - 1
c = _lib.Context([0])
ref = None
for rnd in range(3):
    for k in [1, 2, 3, 4, 5, 6, 7, 8, 0]:
        c.set_option(_lib.HM_OPT_GRID_PER_CU, k)
        r = c.scan(msg, lo, hi)
        ref = ref or r
        assert r == ref
        st = c.stats()
        if rnd == 2:
            print(json.dumps({"per_cu": k, "kernel_GHs": st["dom_nonces"] / st["dom_kernel_ms"] / 1e6,
                              "grid": st["dom_grid"], "kernel": st["dom_kernel"]}), flush=True)
