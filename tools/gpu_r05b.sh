#!/bin/bash
# Round 5: the new GPU tests of the first milestone -- hm_scan_stats' frozen
# 144 bytes, the live mid_call_syncs counter and per-call table frees, and
# bench.py's single-process children (host merge on GPU 0 opened twice, RCCL
# merge on a 1-rank communicator), then smoke().
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  tests/test_abi.py tests/test_gpu_enqueue.py \
  "tests/test_gpu_bench_dist.py::test_bench_single_process_workload_on_one_gpu" > $O/pytest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?
tail -15 $O/pytest.log; tail -2 $O/smoke.log
echo "rc=$rc"
exit $rc
