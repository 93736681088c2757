#!/bin/bash
# GPU-box recipe: edge-tile trimming of the launch unit ranges.  GPU parity
# suite, then A/B (build/ab/lib_base.so = before, lib_trim.so = after) on the
# bench's weak-scaling shard of rank 3 of 8 (d=11, tiles of 10^8 nonces),
# cfg2, and cfg3's rank-3 shard.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/trim; mkdir -p $O
M=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python tools/ab_libs.py 6 build/ab/lib_base.so build/ab/lib_trim.so -- bradfitz 12884901888 17179869183 > $O/rank3.txt 2>&1 &&
timeout -k 10 200 python tools/ab_libs.py 6 build/ab/lib_base.so build/ab/lib_trim.so > $O/cfg2.txt 2>&1 &&
timeout -k 10 200 python tools/ab_libs.py 6 build/ab/lib_base.so build/ab/lib_trim.so -- "$M" 12884901888 17179869183 > $O/cfg3_rank3.txt 2>&1
rc=$?
tail -n 2 $O/pytest_gpu.log; tail -n 3 $O/*.txt
exit $rc
