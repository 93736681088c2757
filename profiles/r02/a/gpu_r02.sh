#!/bin/bash
# GPU-box recipe (round 2): GPU suite, smoke, bench (cfg2 + secondary cfg3),
# and the rocprofv3 kernel trace of the bench, summarised per stream.
# usage: tools/gpu_r02.sh <outdir> [pytest -k expression]
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r02}; K=${2:-}
mkdir -p $O
KARG=(); [ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/trace.log 2>&1 &&
python tools/kernel_stats_by_stream.py $O/trace/run_kernel_trace.csv $O/kernel_stats_by_stream.csv
rc=$?
tail -n 3 $O/pytest_gpu.log; cat $O/smoke.log $O/bench.json
echo "r02 rc=$rc"
exit $rc
