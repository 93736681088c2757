"""Quick timing of hm_scan on the GPU box (dev tool, not the bench contract)."""
import sys, time, json
sys.path.insert(0, '.')
from distributed_bitcoinminer_amd import _lib
if "--lib" in sys.argv:  # an experiment build (tools/build_variant.sh)
    i = sys.argv.index("--lib")
    _lib.LIB_PATH = sys.argv[i + 1]
    del sys.argv[i:i + 2]
c = _lib.Context([0])
if "--opt" in sys.argv:  # --opt NAME=VALUE (an HM_OPT_* suffix), repeatable
    while "--opt" in sys.argv:
        i = sys.argv.index("--opt")
        k, _, v = sys.argv[i + 1].partition("=")
        c.set_option(getattr(_lib, "HM_OPT_" + k), int(v))
        del sys.argv[i:i + 2]
msg = sys.argv[1].encode() if len(sys.argv) > 1 else b"bradfitz"
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = int(sys.argv[3]) if len(sys.argv) > 3 else 2**32 - 1
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
for i in range(reps):
    t = time.perf_counter(); r = c.scan(msg, lo, hi); dt = time.perf_counter() - t
    st = c.stats()
    n = hi - lo + 1
    print(json.dumps({"res": r, "wall_s": dt, "GHs": n / dt / 1e9,
                      "dom_GHs": st["dom_nonces"] / (st["dom_kernel_ms"] * 1e-3) / 1e9 if st["dom_kernel_ms"] else None,
                      **st}), flush=True)
