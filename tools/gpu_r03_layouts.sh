#!/bin/bash
# Layout sweeps (round 3): every message length at d = 10, 12 and 16.
set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
for d in 10 12 16; do
  timeout -k 10 250 python tools/layout_perf.py $d --all > $O/layout_perf_d$d.txt 2> $O/layout_perf_d$d.err || exit 1
done
wc -l $O/*.txt
