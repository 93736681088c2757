"""Chained layouts with >= 5 final-block digits (dev tool, GPU box): kernel
and wall GH/s against the K+W table size (HM_OPT_TABLE_DIGITS: 10^k rows per
table, the remaining final-block digits as epochs; -1 = the tiled kernel)."""
import json
import sys

sys.path.insert(0, ".")
from distributed_bitcoinminer_amd import _lib  # noqa: E402

c = _lib.Context([0])
cases = [("len60_d10_2chunks", b"x" * 60, 2 * 640_000_000, 4 * 640_000_000 - 1),
         ("len58_d10", b"y" * 58, 10**9, 10**9 + 2**32 - 1),
         ("len60_d8_full", b"x" * 60, 10**7, 10**8 - 1)]
for name, m, lo, hi in cases:
    for k in (-1, 7, 6, 5, 4):
        c.set_option(_lib.HM_OPT_TABLE_DIGITS, k)
        c.scan(m, lo, hi)
        res = c.scan(m, lo, hi)
        st = c.stats()
        print(json.dumps({"case": name, "table_digits": k, "res": list(res),
                          "kernel": st["dom_kernel"], "launches": st["dom_launches"],
                          "kernel_GHs": round(st["dom_nonces"] / st["dom_kernel_ms"] / 1e6, 3),
                          "wall_GHs": round((hi - lo + 1) / st["wall_ms"] / 1e6, 3),
                          "busy_GHs": round((hi - lo + 1) / st["kernel_ms"] / 1e6, 3),
                          "c_eff": round(st["dom_compressions_eff"], 4)}), flush=True)
