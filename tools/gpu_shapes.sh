#!/bin/bash
# GPU-box recipe: hm_scan wall vs kernel rate over assorted request shapes
# (tools/quick_scan.py, 5 calls each).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/shapes}; mkdir -p $O
M3=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
for spec in "bradfitz 0 999999999" "bradfitz 0 99999999" "bradfitz 18446744071562067966 18446744073709551614" "bradfitz 5000000000 5134217727" "bradfitz 123456789012 123556789011" "jonny_greenwood 0 4294967295" "$M3 18446744071562067966 18446744073709551614"; do
  set -- $spec
  timeout -k 10 120 python tools/quick_scan.py "$1" $2 $3 5 >> $O/shapes.txt 2>&1 || exit 1
done
echo ok
