#!/bin/bash
# A/B of libhipminer builds in one process per workload (GPU box):
#   bash tools/ab_run.sh build/ab/libX.so build/ab/libY.so ...
# cfg2 (bradfitz [0, 2^32)), the d=12 segment of cfg4, cfg3 (120-B message).
set -o pipefail
O=${AB_OUT:-gpurun_out/ab}; mkdir -p $O
M=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
timeout -k 10 200 python tools/ab_libs.py 6 "$@" > $O/cfg2.txt 2>&1 &&
timeout -k 10 200 python tools/ab_libs.py 6 "$@" -- bradfitz 100000000000 117179869183 > $O/d12.txt 2>&1 &&
timeout -k 10 200 python tools/ab_libs.py 6 "$@" -- "$M" 0 4294967295 > $O/cfg3.txt 2>&1
rc=$?; tail -n 4 $O/*.txt; exit $rc
