#!/bin/bash
# A/B of build/ab/libA.so vs libB.so on cfg2, the d=12 segment and cfg3 (GPU box).
set -o pipefail
O=gpurun_out/ab; mkdir -p $O
M=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
timeout -k 10 200 python tools/ab_libs.py 6 build/ab/libA.so build/ab/libB.so > $O/cfg2.txt 2>&1 &&
timeout -k 10 200 python tools/ab_libs.py 6 build/ab/libA.so build/ab/libB.so -- bradfitz 100000000000 117179869183 > $O/d12.txt 2>&1 &&
timeout -k 10 200 python tools/ab_libs.py 6 build/ab/libA.so build/ab/libB.so -- "$M" 0 4294967295 > $O/cfg3.txt 2>&1
rc=$?; tail -n 2 $O/*.txt; exit $rc
