#!/bin/bash
# Round 5: the fused small-request launch -- its GPU tests, the parity and
# checked suites that now run small ranges through it, the request-size
# curve and the small-request diagnosis fused vs per-segment, and a short
# bench line to confirm the per-segment kernels' rate after the task refactor.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_checked.py > $O/pytest.log 2>&1 &&
timeout -k 10 240 python -u tools/request_sizes.py > $O/request_sizes.jsonl 2> $O/rs.err &&
timeout -k 10 300 python -u tools/small_req_diag.py 15 1,0 4 0,2,3,4 > $O/diag.jsonl 2> $O/diag.err &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --secondary cfg3 > $O/bench.json 2> $O/bench.err
rc=$?
tail -5 $O/pytest.log; cat $O/request_sizes.jsonl; cut -c1-160 $O/diag.jsonl; cut -c1-300 $O/bench.json
echo "rc=$rc"
exit $rc
