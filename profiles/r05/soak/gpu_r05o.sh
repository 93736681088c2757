#!/bin/bash
# Round 5: long randomised soaks of the final tree, one per small-request
# path: the per-segment kernels (HM_SOAK_FUSED=0) and the fused launch.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05o}
mkdir -p $O
HM_SOAK_FUSED=0 HM_SOAK_SECONDS=400 HM_SOAK_SEED=7070 timeout -k 10 800 python -u -m pytest tests/test_gpu_soak.py -m gpu -x -v -s \
  --timeout 700 --timeout-method thread > $O/soak_per_segment_400s_seed7070.log 2>&1 &&
HM_SOAK_SECONDS=160 HM_SOAK_SEED=8080 timeout -k 10 400 python -u -m pytest tests/test_gpu_soak.py -m gpu -x -v -s \
  --timeout 350 --timeout-method thread > $O/soak_fused_160s_seed8080.log 2>&1
rc=$?
grep -h 'done' $O/*.log
echo "rc=$rc"
exit $rc
