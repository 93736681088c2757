#!/bin/bash
# GPU-box recipe (round 2, final profiles): rocprofv3 kernel traces + stats of
# the bench command, in two launch modes.
#  * serial (HM_BENCH_STREAMS=1): every launch in order on one stream, so each
#    dispatch's [start, end] is its own execution time and the stats attribute
#    time exactly.  Committed as bench_kernel_stats.csv.
#  * default (4 streams): the small segments queue on low-priority streams
#    behind the persistent dominant launch and rocprofv3 counts that wait as
#    their duration (a 5-us fold kernel shows tens of ms).  Committed raw as
#    bench_kernel_stats_concurrent_raw.csv, beside the per-(kernel, stream)
#    exclusive-time view of the same trace (kernel_stats_by_stream.csv).
# Each run's bench JSON line is kept, so the dominant kernel's rocprof average
# can be compared with the live HIP-event average (roofline.avg_launch_ms).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r02prof}
mkdir -p $O
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary"
HM_BENCH_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv -- $B > $O/bench_serial.json 2> $O/serial.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/concurrent -o run --output-format csv -- $B > $O/bench_concurrent.json 2> $O/concurrent.log &&
python tools/kernel_stats_by_stream.py $O/concurrent/run_kernel_trace.csv $O/kernel_stats_by_stream.csv &&
HM_BENCH_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cfg3_serial -o run --output-format csv -- $B --workload cfg3 > $O/bench_cfg3_serial.json 2> $O/cfg3_serial.log
rc=$?
head -4 $O/serial/run_kernel_stats.csv $O/cfg3_serial/run_kernel_stats.csv
echo "profile rc=$rc"
exit $rc
