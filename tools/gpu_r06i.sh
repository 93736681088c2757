#!/bin/bash
# Round-6 run i: issue profile of the fused launch on configs[0]'s request
# against a 10^8-nonce fused launch (same kernel, 10x the tasks per wave):
# SQ wait / active cycles per wave, to tell stalls (I-cache, scalar loads,
# queue atomics) from issue-bound time.  Also lists the box's counters.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06i}
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
P="timeout -s KILL 90 rocprofv3 --kernel-trace"
C="--pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES"
$P $C -d $O/cfg1 -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 10000001 20 > $O/cfg1.log 2>&1 &&
$P $C -d $O/e8 -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 99999999 5 > $O/e8.log 2>&1 &&
$P $C -d $O/cfg2 -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/cfg2.log 2>&1
rc=$?
python3 - <<PY
import csv, collections
for run in ("cfg1", "e8", "cfg2"):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open("$O/%s/run_counter_collection.csv" % run)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in d.items():
        if "fused_kernel" in k or "tiled_kernel" in k:
            wc = v["SQ_WAVE_CYCLES"] or 1
            print(run, k, {c: round(x) for c, x in v.items()},
                  "wait_any %.3f wait_inst %.3f active %.3f" % (v["SQ_WAIT_ANY"] / wc, v["SQ_WAIT_INST_ANY"] / wc, v["SQ_ACTIVE_INST_ANY"] / wc))
PY
grep -i "ifetch\|icache\|SQC_" $O/counters_list.txt | head -20
echo "final rc=$rc"
exit $rc
