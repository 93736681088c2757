#!/bin/bash
# Round-6 run j: instruction- and scalar-cache counters of the fused launch on
# configs[0]'s request vs a 10^8-nonce fused launch (cold-start cost per wave).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06j}
mkdir -p $O
P="timeout -s KILL 90 rocprofv3 --kernel-trace"
for w in "cfg1 0 10000001 20" "e8 0 99999999 5"; do
  set -- $w
  $P --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES -d $O/$1_ic -o run --output-format csv -- python tools/quick_scan.py bradfitz $2 $3 $4 > $O/$1_ic.log 2>&1 || exit $?
  $P --pmc SQC_DCACHE_REQ SQC_DCACHE_MISSES -d $O/$1_dc -o run --output-format csv -- python tools/quick_scan.py bradfitz $2 $3 $4 > $O/$1_dc.log 2>&1 || exit $?
done
python3 - <<PY
import csv, collections
for run in ("cfg1_ic", "cfg1_dc", "e8_ic", "e8_dc"):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open("$O/%s/run_counter_collection.csv" % run)):
        k = r["Kernel_Name"].split("(")[0][-30:]
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    for k, v in d.items():
        if "fused_kernel" in k:
            print(run, k, {c: round(x) for c, x in v.items()}, "dispatch-samples", max(n[(k, c)] for c in v))
PY
echo "final rc=0"
