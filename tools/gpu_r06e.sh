#!/bin/bash
# Round-6 run e: fused launch vs per-segment launches by request size
# (HM_OPT_FUSED 1/0), with the fused grid at 3 and 4 workgroups per CU:
# where the fused launch's 10-step tasks stop paying.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06e}
mkdir -p $O
A="timeout -k 10 200 python -u tools/ab_opts.py"
$A 200 f1:FUSED=1 f0:FUSED=0 f1g4:FUSED=1,GRID_PER_CU=4 -- bradfitz 0 10000001 > $O/ab_fused_1e7.jsonl 2> $O/ab.err &&
$A 100 f1:FUSED=1 f0:FUSED=0 f1g4:FUSED=1,GRID_PER_CU=4 -- bradfitz 0 29999999 > $O/ab_fused_3e7.jsonl 2>> $O/ab.err &&
$A 60 f1:FUSED=1 f0:FUSED=0 f1g4:FUSED=1,GRID_PER_CU=4 -- bradfitz 0 99999999 > $O/ab_fused_1e8.jsonl 2>> $O/ab.err &&
$A 60 f1:FUSED=1 f0:FUSED=0 -- bradfitz 1000000000 1130000000 > $O/ab_fused_1p3e8_d10.jsonl 2>> $O/ab.err &&
$A 200 f1:FUSED=1 f0:FUSED=0 -- bradfitz 0 3000000 > $O/ab_fused_3e6.jsonl 2>> $O/ab.err &&
$A 100 f1:FUSED=1 f0:FUSED=0 -- long120 0 99999999 > $O/ab_fused_long120_1e8.jsonl 2>> $O/ab.err &&
$A 200 f1:FUSED=1 f0:FUSED=0 -- long120 0 30000000 > $O/ab_fused_long120_3e7.jsonl 2>> $O/ab.err
rc=$?
for f in $O/ab_*.jsonl; do echo "== $f"; cut -c1-200 $f; done
echo "final rc=$rc"
exit $rc
