#!/bin/bash
# Round-4 check of the retire-until-close table growth and the new parity
# tests (long messages, chained shards cut at lane chunks), plus a 60-s soak.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r04c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_enqueue.py tests/test_gpu_chained_epochs.py tests/test_gpu_lengths.py \
  -x -v -s --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1 &&
HM_SOAK_SECONDS=60 HM_SOAK_SEED=4040 timeout -k 10 300 python -u -m pytest tests/test_gpu_soak.py -x -v -s \
  --timeout 250 --timeout-method thread > $O/soak_60s.log 2>&1
rc=$?
tail -3 $O/pytest_new.log; grep "soak done" $O/soak_60s.log
echo "final rc=$rc"
exit $rc
