"""Round-3 experiment (dev tool): one work queue per XCD vs one device-wide
queue (HM_OPT_QUEUES 8 vs 1), interleaved in one process, kernel GH/s of the
dominant kernel (hm_stats HIP events); plus the correctness of both modes and
of the last-wave drain path (HM_OPT_QUEUE_MASK 3: queues 4..7 have no serving
wave) by hm_scan_checked (min, key sum, count) against mode 1.
usage: python tools/ab_queues.py [rounds] > out.jsonl"""
import json
import random
import sys

sys.path.insert(0, ".")
from distributed_bitcoinminer_amd import _lib  # noqa: E402

rng = random.Random(440)
long120 = bytes(rng.choice(range(0x21, 0x7F)) for _ in range(120))
WL = {"cfg2": (b"bradfitz", 0, 2**32 - 1), "cfg3": (long120, 0, 2**32 - 1),
      "d12": (b"bradfitz", 10**11, 10**11 + 2**34 - 1)}
c = _lib.Context([0])
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6

# correctness: every mode gives the same checked triple
for name, (m, lo, hi) in [("cfg2_slice", (b"bradfitz", 10**9 - 5 * 10**7, 10**9 + 10**8)),
                          ("cfg3_slice", (long120, 10**9 - 10**7, 10**9 + 10**8)),
                          ("d12_slice", (b"bradfitz", 10**11, 10**11 + 3 * 10**8))]:
    got = {}
    for mode, mask in ((1, 7), (8, 7), (8, 3), (8, 0)):
        c.set_option(_lib.HM_OPT_QUEUES, mode)
        c.set_option(_lib.HM_OPT_QUEUE_MASK, mask)
        got[f"{mode}/{mask}"] = c.scan_checked(m, lo, hi)
    c.set_option(_lib.HM_OPT_QUEUE_MASK, 7)
    ok = len({v for v in got.values()}) == 1 and got["1/7"][2] == hi - lo + 1
    print(json.dumps({"check": name, "ok": ok, "got": {k: [list(v[0]), v[1], v[2]]
                                                        for k, v in got.items()}}), flush=True)

for r in range(rounds):
    for name, (m, lo, hi) in WL.items():
        order = (1, 8) if r % 2 == 0 else (8, 1)
        for mode in order:
            c.set_option(_lib.HM_OPT_QUEUES, mode)
            res = c.scan(m, lo, hi)
            st = c.stats()
            print(json.dumps({"round": r, "wl": name, "mode": mode, "res": list(res),
                              "kernel_GHs": st["dom_nonces"] / (st["dom_kernel_ms"] * 1e-3) / 1e9,
                              "wall_GHs": (hi - lo + 1) / (st["wall_ms"] * 1e-3) / 1e9}),
                  flush=True)
