#!/bin/bash
# GPU-box recipe: what the driver runs at round end (GPU suite, smoke, bench)
# plus the rocprofv3 kernel-trace summary of the same bench command, so the
# committed bench line and its profile come from one box and one build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --workload cfg3 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
rc=$?
tail -n 2 $O/pytest_gpu.log; cat $O/smoke.log $O/bench.json $O/bench_cfg3.json
echo "final rc=$rc"
exit $rc
