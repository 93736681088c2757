#!/bin/bash
# Round 5: the fused launch's in-launch fold (HM_OPT_FUSED_FLAGS bit 4): the
# fused GPU tests, then an interleaved A/B of flags 1 (queue + static first
# task), 17 (+ in-launch fold) and 25 (+ LDS dispenser) on small requests,
# and a rocprofv3 kernel trace of config 1 with the fold in the launch.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05n}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_smoke.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/fused_ab.py 25 1,17,25 3 1 > $O/fused_ab.jsonl 2> $O/fused_ab.err
rc=$?
tail -3 $O/pytest.log; cat $O/fused_ab.jsonl
echo "rc=$rc"
exit $rc
