"""Per-rank shard timing of the weak-scaling bench on ONE GPU (dev tool).

The driver's N-GPU bench gives rank r the nonces [r*2^32, (r+1)*2^32) and
reports N*2^32 / (max over ranks).  This times each rank's shard alone on
GPU 0 (median of `reps` hm_scan calls, wall clock incl. planning and the
readback) so the slowest rank -- the one that sets the N-GPU value -- is
known before the 8-GPU run.  With `--partition` it also times the
cost-weighted hm_partition shards of [0, N*2^32).  `--workload cfg4` times
the strong-scaling split of bench.py --workload cfg4: for N = 1, 2, 4, 8 the
hm_partition shards of [0, 2^40), predicted N-GPU GH/s = 2^40 / slowest rank.

usage: python tools/rank_sweep.py [--workload cfg2|cfg3|cfg4] [--ranks 8] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_bitcoinminer_amd import _lib  # noqa: E402

PER_GPU = 1 << 32


def long120() -> bytes:
    import random
    r = random.Random(440)
    return bytes(r.choice(range(0x21, 0x7F)) for _ in range(120))


def time_shard(ctx, msg, lo, hi, reps):
    if hi - lo < (1 << 36):  # warm (module load, tables); huge shards warm themselves
        ctx.scan(msg, lo, hi)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        ctx.scan(msg, lo, hi)
        ts.append(time.perf_counter() - t)
    ts.sort()
    st = ctx.stats()
    return ts[len(ts) // 2], st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2", choices=["cfg2", "cfg3", "cfg4"])
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--partition", action="store_true")
    a = ap.parse_args()
    msg = long120() if a.workload == "cfg3" else b"bradfitz"
    ctx = _lib.Context([0])
    if a.workload == "cfg4":
        shards = {f"cfg4_n{n}": _lib.partition(msg, 0, (1 << 40) - 1, n) for n in (1, 2, 4, 8)}
    else:
        shards = {"equal": [(r * PER_GPU, (r + 1) * PER_GPU - 1) for r in range(a.ranks)]}
    if a.partition and a.workload != "cfg4":
        shards["partition"] = _lib.partition(msg, 0, a.ranks * PER_GPU - 1, a.ranks)
    for name, sh in shards.items():
        worst = 0.0
        times = []
        for r, (lo, hi) in enumerate(sh):
            dt, st = time_shard(ctx, msg, lo, hi, a.reps)
            worst = max(worst, dt)
            times.append(dt)
            segs = [(s["d"], s["kind"]) for s in _lib.debug_plan(msg, lo, hi)]
            print(json.dumps({"split": name, "rank": r, "lo": lo, "hi": hi, "ms": round(dt * 1e3, 3),
                              "GHs": round((hi - lo + 1) / dt / 1e9, 3),
                              "dom_kernel": st["dom_kernel"], "segments": segs}), flush=True)
        if name == "equal":  # weak scaling: the job of N ranks is ranks 0..N-1
            for n in (1, 2, 4, 8):
                if n <= len(times):
                    print(json.dumps({"split": name, "n_gpus": n,
                                      "worst_ms": round(max(times[:n]) * 1e3, 3),
                                      "predicted_GHs": round(n * PER_GPU / max(times[:n]) / 1e9, 3)}),
                          flush=True)
        total = sh[-1][1] - sh[0][0] + 1
        print(json.dumps({"split": name, "ranks": len(sh), "worst_ms": round(worst * 1e3, 3),
                          "predicted_GHs": round(total / worst / 1e9, 3)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
