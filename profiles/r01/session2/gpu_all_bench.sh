#!/bin/bash
# GPU-box: whole GPU suite, smoke, bench (cfg2 + cfg3) and a kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/allb; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --workload cfg3 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
rc=$?
tail -4 $O/pytest_gpu.log; cat $O/smoke.log $O/bench.json $O/bench_cfg3.json; exit $rc
