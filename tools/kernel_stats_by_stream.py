#!/usr/bin/env python3
"""Per-(kernel, stream) time attribution of a rocprofv3 kernel trace.

rocprofv3 --stats sums each dispatch's [start, end].  For a kernel queued on
a low-priority stream behind the persistent scan launch that interval
includes its wait for workgroup slots (DESIGN.md §3 "Tail filling"), so the
7-us fold kernels there show averages of tens of ms and a large share of the
summed time.  This tool groups the dispatches by (kernel, stream) and adds
each dispatch's EXCLUSIVE time: the part of its interval during which no
other dispatch was in flight.  Exclusive time sums to at most the wall time
of the trace, and the share column uses it.

usage: python tools/kernel_stats_by_stream.py <run_kernel_trace.csv> [out.csv]
"""
import csv
import sys


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").replace("hm::", "")


def main(src, dst=None):
    rows = []
    for r in csv.DictReader(open(src)):
        rows.append((short(r["Kernel_Name"]), int(r["Stream_Id"]),
                     int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    # exclusive time: subtract the union of the other dispatches' overlaps
    rows.sort(key=lambda x: x[2])
    excl = []
    for i, (_, _, a, b) in enumerate(rows):
        cover = []
        for j, (_, _, c, d) in enumerate(rows):
            if j != i and c < b and d > a:
                cover.append((max(a, c), min(b, d)))
        cover.sort()
        covered, cur_a, cur_b = 0, None, None
        for x, y in cover:
            if cur_b is None or x > cur_b:
                if cur_b is not None:
                    covered += cur_b - cur_a
                cur_a, cur_b = x, y
            else:
                cur_b = max(cur_b, y)
        if cur_b is not None:
            covered += cur_b - cur_a
        excl.append((b - a) - covered)
    groups = {}
    for (name, stream, a, b), e in zip(rows, excl):
        g = groups.setdefault((name, stream), [0, 0, 0])
        g[0] += 1
        g[1] += b - a
        g[2] += e
    tot_excl = sum(g[2] for g in groups.values()) or 1
    out = [["Kernel", "Stream_Id", "Calls", "TotalMs", "AvgMs", "ExclusiveMs",
            "ExclusiveAvgMs", "ExclusivePct"]]
    for (name, stream), (n, t, e) in sorted(groups.items(), key=lambda kv: -kv[1][2]):
        out.append([name, stream, n, f"{t / 1e6:.4f}", f"{t / n / 1e6:.4f}", f"{e / 1e6:.4f}",
                    f"{e / n / 1e6:.4f}", f"{100.0 * e / tot_excl:.2f}"])
    f = open(dst, "w", newline="") if dst else sys.stdout
    csv.writer(f).writerows(out)
    if dst:
        f.close()


if __name__ == "__main__":
    main(*sys.argv[1:])
