#!/bin/bash
# Round 5: fused-launch task dispensing A/B (static first task, prefetch,
# grid per CU) on small requests, after the fused GPU tests with each flag.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u tools/fused_ab.py 25 0,1,2,3 2,3,4 > $O/ab.jsonl 2> $O/ab.err
rc=$?
tail -3 $O/pytest.log; cat $O/ab.jsonl
echo "rc=$rc"
exit $rc
