"""Timeline of the fused small-request launch (dev tool, GPU box).

usage: python tools/fused_trace.py [msg lo hi] [--runs N] [--opt NAME=VALUE ...]

Runs one request N times (after a warm-up) with HM_OPT_FUSED_TRACE, so every
wave of the fused launch records the wall clock (wall_clock64, 100 MHz) at
its start, when it takes its last task, and at its end, plus its task count.
Prints one JSON line per run: the launch's span (first wave start to last
wave end) against hm_stats' kernel time, the ramp (wave starts after the
first), the tail (wave ends before the last), the share of wave-time lost to
each, and the tasks per wave -- where a small request's time beyond its
layouts' rate goes (DESIGN §5 "Request size")."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_bitcoinminer_amd import _lib  # noqa: E402

TICK_US = 0.01  # wall_clock64 runs at 100 MHz on MI355X (hipDeviceAttributeWallClockRate)


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(p / 100 * len(xs)))]


def main():
    args = sys.argv[1:]
    runs = 5
    opts = []
    while "--runs" in args:
        i = args.index("--runs")
        runs = int(args[i + 1])
        del args[i:i + 2]
    while "--opt" in args:
        i = args.index("--opt")
        k, _, v = args[i + 1].partition("=")
        opts.append((getattr(_lib, "HM_OPT_" + k), int(v)))
        del args[i:i + 2]
    msg, lo, hi = b"bradfitz", 0, 10**7 + 1
    if args:
        msg, lo, hi = args[0].encode(), int(args[1]), int(args[2])
        if msg == b"long120":
            import random
            r = random.Random(440)
            msg = bytes(r.choice(range(0x21, 0x7F)) for _ in range(120))
    with _lib.Context([0]) as c:
        for o, v in opts:
            c.set_option(o, v)
        c.set_option(_lib.HM_OPT_FUSED_TRACE, 1)
        for _ in range(3):
            c.scan(msg, lo, hi)  # warm-up
        for run in range(runs):
            c.scan(msg, lo, hi)
            st = c.stats()
            tr = [t for t in c.fused_trace() if t[2] > 0]
            t0 = min(t[0] for t in tr)
            t_end = max(t[2] for t in tr)
            span = (t_end - t0) * TICK_US
            starts = [(t[0] - t0) * TICK_US for t in tr]
            ends = [(t[2] - t0) * TICK_US for t in tr]
            lasts = [(t[1] - t0) * TICK_US for t in tr if t[3] > 0]
            tasks = [t[3] for t in tr]
            n = len(tr)
            ramp_loss = sum(starts) / (n * span)
            tail_loss = sum(span - e for e in ends) / (n * span)
            print(json.dumps({
                "run": run, "msg_len": len(msg), "lo": lo, "hi": hi, "waves": n,
                "kernel_ms_events": round(st["kernel_ms"], 4), "wall_ms": round(st["wall_ms"], 4),
                "span_us": round(span, 1),
                "start_us": {"p50": round(pct(starts, 50), 1), "p90": round(pct(starts, 90), 1),
                             "max": round(max(starts), 1)},
                "last_task_start_us": {"p10": round(pct(lasts, 10), 1),
                                       "p50": round(pct(lasts, 50), 1),
                                       "max": round(max(lasts), 1)} if lasts else None,
                "end_us": {"min": round(min(ends), 1), "p10": round(pct(ends, 10), 1),
                           "p50": round(pct(ends, 50), 1), "p90": round(pct(ends, 90), 1)},
                "ramp_loss": round(ramp_loss, 4), "tail_loss": round(tail_loss, 4),
                "tasks_per_wave": {"min": min(tasks), "median": statistics.median(tasks),
                                   "max": max(tasks), "total": sum(tasks)},
                "options": [[o, v] for o, v in opts]}), flush=True)


if __name__ == "__main__":
    main()
