"""Interleaved A/B of hipminer context OPTIONS in ONE process (dev tool, GPU box).

usage: python tools/ab_opts.py ROUNDS VARIANT [VARIANT ...] [--no-check] [-- msg lo hi]
  VARIANT = name:opt=value,opt=value   (opt: a number or an HM_OPT_* suffix,
            e.g. base:  s2:STREAMS=2  f0:FUSED=0)
  msg "long120" = BASELINE configs[2]'s message (random.Random(440)).

Every variant gets its own context on GPU 0; each round scans the range once
per variant, in turn, so clock and thermal drift hit all variants alike.
Prints one JSON line per variant: median wall GH/s (whole hm_scan), median
dominant-kernel GH/s, median wall ms, and the answers must agree (unless
--no-check)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_bitcoinminer_amd import _lib  # noqa: E402


def parse_variant(v):
    name, _, opts = v.partition(":")
    out = []
    for kv in filter(None, opts.split(",")):
        k, _, val = kv.partition("=")
        opt = int(k) if k.isdigit() else getattr(_lib, "HM_OPT_" + k)
        out.append((opt, int(val)))
    return name, out


def main():
    args = sys.argv[1:]
    check = "--no-check" not in args
    args = [a for a in args if a != "--no-check"]
    msg, lo, hi = b"bradfitz", 0, 2**32 - 1
    if "--" in args:
        i = args.index("--")
        msg, lo, hi = args[i + 1].encode(), int(args[i + 2]), int(args[i + 3])
        args = args[:i]
        if msg == b"long120":
            import random
            r = random.Random(440)
            msg = bytes(r.choice(range(0x21, 0x7F)) for _ in range(120))
    rounds = int(args[0])
    variants = [parse_variant(v) for v in args[1:]]
    ctxs = []
    for name, opts in variants:
        c = _lib.Context([0])
        for o, v in opts:
            c.set_option(o, v)
        c.scan(msg, lo, min(hi, lo + 10**6))  # warm: module, streams
        ctxs.append((name, c))
    res = {n: [] for n, _ in ctxs}
    ref = None
    for _ in range(rounds):
        for name, c in ctxs:
            t = time.perf_counter()
            got = c.scan(msg, lo, hi)
            dt = time.perf_counter() - t
            st = c.stats()
            ref = ref or got
            assert not check or got == ref, (name, got, ref)
            res[name].append((dt, st["dom_nonces"] / st["dom_kernel_ms"] / 1e6, st["launches"]))
    n = hi - lo + 1
    for name, _ in ctxs:
        walls = sorted(x[0] for x in res[name][1:] or res[name])
        kern = sorted(x[1] for x in res[name][1:] or res[name])
        print(json.dumps({"variant": name, "msg_len": len(msg), "lo": lo, "hi": hi,
                          "rounds": rounds, "median_wall_GHs": round(n / walls[len(walls) // 2] / 1e9, 3),
                          "median_wall_ms": round(walls[len(walls) // 2] * 1e3, 4),
                          "min_wall_ms": round(walls[0] * 1e3, 4),
                          "median_dom_GHs": round(kern[len(kern) // 2], 3),
                          "launches": res[name][-1][2], "answer": list(ref)}), flush=True)
    for _, c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
