#!/bin/bash
# GPU-box recipe: the GPU suite on the current build, then an interleaved
# one-process A/B of library variants over request shapes (both orders):
# cfg2, a 2^27-nonce d = 10 request, 10^8-nonce requests (one segment, and
# [0, 10^8) over eight digit counts), cfg4's d = 12 segment and cfg3.
# usage: [SKIP_SUITE=1] tools/gpu_ab_shapes.sh <outdir> <lib.so>...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
L="$*"; R=""
for l in "$@"; do R="$l $R"; done
M3=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
ab() {  # name rounds [-- msg lo hi]
    local n=$1 k=$2; shift 2
    timeout -k 10 300 python -u tools/ab_libs.py $k $L "$@" > $O/ab_${n}_fwd.txt 2>&1 &&
    timeout -k 10 300 python -u tools/ab_libs.py $k $R "$@" > $O/ab_${n}_rev.txt 2>&1
}
{ [ -n "$SKIP_SUITE" ] || timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; } &&
ab cfg2 7 &&
ab r27 25 -- bradfitz 5000000000 5134217727 &&
ab e8one 25 -- bradfitz 1000000000 1099999999 &&
ab e8multi 25 -- bradfitz 0 99999999 &&
ab d12 5 -- bradfitz 100000000000 104999999999 &&
ab cfg3 5 -- "$M3" 0 4294967295
rc=$?; [ -f $O/pytest_gpu.log ] && tail -n 2 $O/pytest_gpu.log; for f in $O/ab_*.txt; do echo $f; cat $f; done; exit $rc
