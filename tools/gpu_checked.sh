#!/bin/bash
# GPU-box: checked-scan (coverage checksum) tests, then the full GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/checked; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_checked.py -x -v --timeout 300 --timeout-method thread > $O/pytest_checked.log 2>&1
rc=$?; tail -25 $O/pytest_checked.log; exit $rc
