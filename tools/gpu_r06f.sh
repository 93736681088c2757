#!/bin/bash
# Round-6 run f: repeat the FETCH_SIZE / WRITE_SIZE passes of the d = 12
# launch (2*10^11 nonces) three times, to see how much of cfg4's PMC traffic
# is run-to-run noise (FETCH 7.2 MB in r06final, 76.5 MB in r06final_b).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06f}
mkdir -p $O
P="timeout -s KILL 90 rocprofv3 --kernel-trace"
for i in 1 2 3; do
  $P --pmc FETCH_SIZE -d $O/fetch_$i -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 299999999999 1 > $O/fetch_$i.log 2>&1 || exit $?
  $P --pmc WRITE_SIZE -d $O/write_$i -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 299999999999 1 > $O/write_$i.log 2>&1 || exit $?
done
$P --pmc FETCH_SIZE -d $O/fetch_cfg2 -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/fetch_cfg2.log 2>&1
rc=$?
for f in $O/fetch_* $O/write_*; do [ -d $f ] && python3 -c "
import csv,sys
t={}
for r in csv.DictReader(open('$f/run_counter_collection.csv')):
    k=r['Kernel_Name'][:40]; t[k]=t.get(k,0)+float(r['Counter_Value'])
print('$f', {k:round(v) for k,v in t.items() if 'tiled' in k})"; done
echo "final rc=$rc"
exit $rc
