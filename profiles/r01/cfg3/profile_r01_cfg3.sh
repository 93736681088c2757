#!/bin/bash
# cfg3 (120-B message, chained kernel) kernel trace + bench (run under gpurun).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r01_cfg3
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --workload cfg3 --steps 5 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
rc=$?
grep -h '"metric"' $O/trace.log > $O/bench_under_rocprof.json
cat $O/bench_under_rocprof.json
exit $rc
