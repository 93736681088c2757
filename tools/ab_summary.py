"""Summarise tools/gpu_ab_shapes.sh / gpu_pad_ab.sh output: per request shape,
the mean over runs and variants (build/<group>/<k>/libhipminer.so) of the
median kernel GH/s and wall GH/s of each group.  Dev tool.
usage: python tools/ab_summary.py <outdir>"""
import collections
import glob
import json
import os
import statistics as S
import sys

d = sys.argv[1]
shapes = sorted({os.path.basename(f)[3:].rsplit("_", 1)[0] for f in glob.glob(f"{d}/ab_*_*.txt")})
for w in shapes:
    dom, wall = collections.defaultdict(list), collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/ab_{w}_*.txt")):
        for line in open(f):
            if line.startswith("{"):
                r = json.loads(line)
                parts = r["lib"].split("/")
                # build/<group>/<k>/lib.so (offset variants) or build/ab_flags/<name>/lib.so
                g = parts[-3] if parts[-2].isdigit() else parts[-2]
                dom[g].append(r["median_dom_GHs"])
                wall[g].append(r["median_wall_GHs"])
    groups = sorted(dom)
    base = groups[0]
    out = [f"{w:9s}"]
    for g in groups:
        rel = f" ({100 * (S.mean(wall[g]) / S.mean(wall[base]) - 1):+.2f} %)" if g != base else ""
        out.append(f"{g}: kernel {S.mean(dom[g]):.3f} wall {S.mean(wall[g]):.3f}{rel}")
    print("  ".join(out))
