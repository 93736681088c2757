#!/bin/bash
# GPU-box recipe: stream-order A/B (both orders, cfg2 and cfg3) + the
# multi-stream GPU tests.  usage: tools/gpu_r02_ab3.sh <outdir> <libA> <libB>
set -o pipefail
export TMPDIR=/tmp
O=$1; A=$2; B=$3; mkdir -p $O
M3=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "scan_many or streams or rccl or stats or golden_scans or full_2p32" > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 11 $A $B > $O/ab_cfg2_ab.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 11 $B $A > $O/ab_cfg2_ba.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 11 $A $B -- "$M3" 0 4294967295 > $O/ab_cfg3_ab.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 11 $B $A -- "$M3" 0 4294967295 > $O/ab_cfg3_ba.txt 2>&1
rc=$?; tail -n 1 $O/pytest_gpu.log; for f in $O/ab_*.txt; do echo $f; cat $f; done; exit $rc
