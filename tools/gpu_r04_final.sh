#!/bin/bash
# Round-4 validation of the final tree (GPU box): the GPU suite as the driver
# runs it, smoke(), the default bench line, and rocprofv3 --stats of the bench
# with serial launches (HM_BENCH_STREAMS=1) for the kernel-time agreement.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r04final}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
HM_BENCH_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/bench_serial.json 2> $O/serial.log
rc=$?
tail -2 $O/pytest_gpu.log; head -2 $O/serial/run_kernel_stats.csv 2>/dev/null
echo "final rc=$rc"
exit $rc
