#!/bin/bash
# GPU-box: the whole GPU suite (as the driver runs it at round end).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/all; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -40 $O/pytest_gpu.log; exit $rc
