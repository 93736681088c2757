#!/bin/bash
# GPU-box: whole GPU suite, bench, occupancy sweep and a kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/allc; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --workload cfg3 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err &&
timeout -k 10 300 python tools/occ_sweep.py > $O/occ_sweep.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log; cat $O/bench.json $O/bench_cfg3.json $O/occ_sweep.txt; exit $rc
