#!/bin/bash
# GPU-box recipe: GPU suite on the current build, then interleaved one-process
# A/B runs of two library builds (tools/ab_libs.py) on given workloads.
# usage: tools/gpu_r02_ab.sh <outdir> <libA.so> <libB.so> [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
O=$1; A=$2; B=$3; K=${4:-}
mkdir -p $O
KARG=(); [ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread "${KARG[@]}" > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 7 $A $B > $O/ab_cfg2.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 7 $A $B -- bradfitz 100000000000 120000000000 > $O/ab_d12.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 7 $A $B -- bradfitz 1000000000000 1020000000000 > $O/ab_d13.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 7 $A $B -- bradfitz 100000000 999999999 > $O/ab_d9.txt 2>&1
rc=$?
tail -n 2 $O/pytest_gpu.log; cat $O/ab_*.txt; echo "ab rc=$rc"; exit $rc
