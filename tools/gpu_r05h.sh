#!/bin/bash
# Round 5: fused-launch task dispensing (HM_OPT_FUSED_FLAGS 1 = static first
# task + queue, 9 = + LDS dispenser, 4 = static stride, no queue) x grid x
# parts A/B on small requests, after the fused GPU tests; KFD queue counts.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05h}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_smoke.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/queue_count.py > $O/queue_count.jsonl 2> $O/queue_count.err &&
timeout -k 10 400 python -u tools/fused_ab.py 15 1,9,4 3,4,6 1,2 > $O/fused_ab.jsonl 2> $O/fused_ab.err
rc=$?
tail -3 $O/pytest.log; cut -c1-200 $O/queue_count.jsonl
echo "rc=$rc"
exit $rc
