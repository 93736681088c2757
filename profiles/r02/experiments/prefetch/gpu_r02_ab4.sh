#!/bin/bash
# GPU-box recipe: interleaved A/B (both orders) of two builds on cfg2, a
# medium d=10 request (2^27 nonces) and cfg3, plus a GPU-suite subset on the
# current build.  usage: tools/gpu_r02_ab4.sh <outdir> <libA> <libB>
set -o pipefail
export TMPDIR=/tmp
O=$1; A=$2; B=$3; mkdir -p $O
M3=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "checked or golden or random or chained" > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 9 $A $B > $O/ab_cfg2_ab.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 9 $B $A > $O/ab_cfg2_ba.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 15 $A $B -- bradfitz 5000000000 5134217727 > $O/ab_med_ab.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 15 $B $A -- bradfitz 5000000000 5134217727 > $O/ab_med_ba.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 9 $A $B -- "$M3" 0 4294967295 > $O/ab_cfg3_ab.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 9 $B $A -- "$M3" 0 4294967295 > $O/ab_cfg3_ba.txt 2>&1
rc=$?; tail -n 1 $O/pytest_gpu.log; for f in $O/ab_*.txt; do echo $f; cat $f; done; exit $rc
