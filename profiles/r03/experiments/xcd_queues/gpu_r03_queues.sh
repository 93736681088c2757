#!/bin/bash
# Round-3 per-XCD work-queue experiment: interleaved A/B + PMC WRITE_SIZE /
# FETCH_SIZE of cfg2's two dominant launches in each queue mode.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03q}
mkdir -p $O
P="timeout -s KILL 90 rocprofv3 --kernel-trace"
timeout -k 10 200 python tools/ab_queues.py 6 > $O/ab.jsonl 2> $O/ab.err &&
for q in 1 8; do
  HM_QUEUES=$q $P --pmc WRITE_SIZE -d $O/q$q/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/q$q.write.log 2>&1 &&
  HM_QUEUES=$q $P --pmc FETCH_SIZE -d $O/q$q/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/q$q.fetch.log 2>&1 || exit 1
done
rc=$?
echo "rc=$rc"; grep check $O/ab.jsonl | cut -c1-200
exit $rc
