"""Summarise a rocprofv3 run directory (from tools/profile_rNN.sh) into
profiles/<round>/pmc_summary.json.  Dev tool.

Per scan kernel: launches, total nonces (from the bench's own accounting is not
available here, so the quick_scan workload bradfitz [0, 2^32) is assumed),
SQ_INSTS_VALU per 64-nonce wave-iteration, effective clock
(GRBM_GUI_ACTIVE / 8 / duration, MI355X_MICROARCH.md 'DVFS give-back'),
and HBM bytes per launch: FETCH_SIZE x 2 (gfx950 reports half of wide reads,
MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KB.
Each entry records the sha256 (16 hex) of the scan code object it was measured
on (build/hipminer/hipminer_scan.hsaco); bench.py uses an entry only for that
same build.
usage: python tools/summarize_profile.py gpurun_out/r01 profiles/r01
"""
import collections
import csv
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
merge_into = os.path.join(dst, "pmc_summary.json")
# segment nonces of bradfitz [0, 2^32) by kernel (planner: d=9 and d=10 share W1=4)
NONCES = {"hm_tiled_kernel<4, false, false>": 900_000_000 + (2**32 - 10**9),
          "hm_tiled_kernel<4, true, false>": 90_000_000,
          "hm_tiled_kernel<3, false, false>": 9_990_000,
          # cfg3 (120-B message): d = 8, 9, 10 are chained
          "hm_chained_kernel": 2**32 - 10**7,
          # cfg4's dominant segment (bradfitz d = 12): [10^11, 3*10^11) since
          # round 6 (a launch of >= 10^11 nonces, which fetches 16 tasks per
          # queue atomic, as the bench's 9*10^11-nonce launch does)
          "hm_tiled_kernel<5, true, false>": 200_000_000_000}


def per_dispatch(path):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("void hm::", "").replace("hm::", ""))
        d[k][r["Counter_Name"]] = d[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d[k]["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return d


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import code_object_sha16  # noqa: E402

SHA = code_object_sha16()
out = {}
valu = per_dispatch(os.path.join(src, "pmc_valu", "run_counter_collection.csv"))
fetch = per_dispatch(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
write = per_dispatch(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
for name, nonces in NONCES.items():
    vs = [v for (i, n), v in valu.items() if n == name]
    fs = [v for (i, n), v in fetch.items() if n == name]
    ws = [v for (i, n), v in write.items() if n == name]
    if not vs:
        continue
    insts = sum(v["SQ_INSTS_VALU"] for v in vs)
    dur = sum(v["dur_ns"] for v in vs)
    grbm = sum(v["GRBM_GUI_ACTIVE"] for v in vs)
    big = max(vs, key=lambda v: v["dur_ns"])
    n_l = len(vs)
    fetch_kb = sum(v["FETCH_SIZE"] for v in fs)
    write_kb = sum(v["WRITE_SIZE"] for v in ws)
    out[name] = {
        "launches": n_l, "nonces": nonces, "duration_ms": dur / 1e6,
        "valu_insts_per_wave_iteration_64_nonces": insts / (nonces / 64),
        "f_eff_ghz_largest_dispatch": big["GRBM_GUI_ACTIVE"] / 8 / big["dur_ns"],
        "f_eff_ghz_all": grbm / 8 / dur,
        "cycles_per_wave_inst": (dur * 1e-9 * grbm / 8 / dur * 1e9) / (insts / 1024) if insts else None,
        "fetch_kb_raw": fetch_kb, "write_kb": write_kb,
        "hbm_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024 / n_l,
        "code_object_sha16": SHA,
    }
os.makedirs(dst, exist_ok=True)
if os.path.exists(merge_into):  # keep kernels summarised from other runs
    with open(merge_into) as f:
        prev = json.load(f)
    prev.update(out)
    out = prev
with open(merge_into, "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
