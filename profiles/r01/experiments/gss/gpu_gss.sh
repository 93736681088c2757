#!/bin/bash
# GPU-box recipe: guided self-scheduling of the task queue (HM_OPT_GSS_K).
# GPU parity suite, interleaved A/B (HEAD-before build vs the new build at
# K = 0/2/4/8), and HBM traffic per launch (PMC FETCH_SIZE / WRITE_SIZE) at
# K = 0 and K = 4 on cfg2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/gss; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
AB_OUT=$O/ab bash tools/ab_run.sh build/ab/lib_base.so build/ab/lib_gss.so:0 build/ab/lib_gss.so:2 build/ab/lib_gss.so:4 build/ab/lib_gss.so:8 > $O/ab.log 2>&1 &&
P="timeout -s KILL 120 rocprofv3 --kernel-trace" &&
for k in 0 4; do
  HM_QS_GSS_K=$k $P --pmc FETCH_SIZE -d $O/k$k/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/k$k.fetch.log 2>&1 &&
  HM_QS_GSS_K=$k $P --pmc WRITE_SIZE -d $O/k$k/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/k$k.write.log 2>&1 || exit 1
done
rc=$?
tail -n 2 $O/pytest_gpu.log; tail -n 5 $O/ab/*.txt
exit $rc
