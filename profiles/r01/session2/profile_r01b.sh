#!/bin/bash
# GPU-box recipe (round 1, second session): parity tests, bench, kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r01b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --workload cfg3 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log; cat $O/bench.json $O/bench_cfg3.json
echo "profile rc=$rc"
exit $rc
