#!/bin/bash
# Round-4 validation (GPU box): the new GPU tests first (enqueue overlap,
# table cap fallback, per-rank bench self-check), then the whole GPU suite as
# the driver runs it, smoke() and the default bench line.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r04a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_enqueue.py tests/test_gpu_bench_dist.py -x -vv -s --timeout 240 --timeout-method thread > $O/pytest_new.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/pytest_new.log $O/pytest_gpu.log 2>/dev/null
echo "final rc=$rc"
exit $rc
