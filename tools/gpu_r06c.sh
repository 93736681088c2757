#!/bin/bash
# Round-6 run c: the fused launch's wave timeline (HM_OPT_FUSED_TRACE) on
# configs[0]'s request, 10^6 nonces and the 120-B message at 10^7, under a
# few grid / tail / dispensing settings -- where the small request's time
# beyond its layouts' rate goes.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06c}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_fused.log 2>&1
prc=$?
tail -2 $O/pytest_fused.log
if [ $prc -gt 1 ]; then echo "pytest rc=$prc: stopping"; exit $prc; fi
T="timeout -k 10 120 python -u tools/fused_trace.py"
$T --runs 5 > $O/trace_cfg1.jsonl 2> $O/trace.err &&
$T --runs 3 --opt FUSED_TAIL=1 > $O/trace_cfg1_t1.jsonl 2>> $O/trace.err &&
$T --runs 3 --opt GRID_PER_CU=2 > $O/trace_cfg1_g2.jsonl 2>> $O/trace.err &&
$T --runs 3 --opt GRID_PER_CU=4 > $O/trace_cfg1_g4.jsonl 2>> $O/trace.err &&
$T --runs 3 --opt FUSED_FLAGS=9 > $O/trace_cfg1_lds.jsonl 2>> $O/trace.err &&
$T bradfitz 0 1000000 --runs 3 > $O/trace_1e6.jsonl 2>> $O/trace.err &&
$T long120 0 10000000 --runs 3 > $O/trace_long120.jsonl 2>> $O/trace.err
rc=$?
for f in $O/trace_*.jsonl; do echo "== $f"; cut -c1-420 $f; done
echo "final rc=$rc"
exit $rc
