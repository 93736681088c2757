#!/bin/bash
# Round-3 chained-epoch layouts: their GPU tests, the parity and checked
# suites, the bench (cfg3 must not move) and the layout sweep.
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_chained_epochs.py tests/test_gpu_parity.py tests/test_gpu_checked.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --secondary cfg3 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python tools/layout_perf.py > $O/layout_perf.txt 2> $O/layout_perf.err
rc=$?; tail -4 $O/pytest.log; exit $rc
