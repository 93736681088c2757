#!/bin/bash
# Round-6 run d: wave-priority equalisation in the fused launch
# (HM_OPT_FUSED_FLAGS bit 4): its dispensing test, the wave timeline, and an
# interleaved A/B on configs[0], 10^6 nonces and the 120-B message at 10^7.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -v -k "flags or trace" --timeout 200 --timeout-method thread > $O/pytest_fused.log 2>&1
prc=$?
tail -2 $O/pytest_fused.log
if [ $prc -gt 1 ]; then echo "pytest rc=$prc: stopping"; exit $prc; fi
T="timeout -k 10 120 python -u tools/fused_trace.py"
A="timeout -k 10 240 python -u tools/ab_opts.py"
$T --runs 3 --opt FUSED_FLAGS=17 > $O/trace_cfg1_prio.jsonl 2> $O/trace.err &&
$A 300 base:FUSED_FLAGS=1 prio:FUSED_FLAGS=17 prlds:FUSED_FLAGS=25 -- bradfitz 0 10000001 > $O/ab_prio_cfg1.jsonl 2> $O/ab.err &&
$A 300 base:FUSED_FLAGS=1 prio:FUSED_FLAGS=17 prlds:FUSED_FLAGS=25 -- long120 0 10000000 > $O/ab_prio_long120.jsonl 2>> $O/ab.err &&
$A 300 base:FUSED_FLAGS=1 prio:FUSED_FLAGS=17 prlds:FUSED_FLAGS=25 -- bradfitz 0 1000000 > $O/ab_prio_1e6.jsonl 2>> $O/ab.err &&
$A 100 base:FUSED_FLAGS=1 prio:FUSED_FLAGS=17 -- bradfitz 0 99999999 > $O/ab_prio_1e8.jsonl 2>> $O/ab.err
rc=$?
for f in $O/trace_*.jsonl $O/ab_*.jsonl; do echo "== $f"; cut -c1-400 $f; done
echo "final rc=$rc"
exit $rc
