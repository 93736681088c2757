#!/bin/bash
# GPU-box recipe: PMC passes (tools/profile_r02.sh) and the bench lines
# (cfg2 default with secondary cfg3, cfg4 on one GPU) plus the multi-stream
# kernel trace of the bench, on one box and one build.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r02r}; mkdir -p $O
tools/profile_r02.sh $O/prof > $O/profile.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/trace.log 2>&1 &&
python tools/kernel_stats_by_stream.py $O/trace/run_kernel_trace.csv $O/kernel_stats_by_stream.csv
rc=$?
cat $O/bench.json $O/bench_cfg4.json; echo "refresh rc=$rc"; exit $rc
