#!/bin/bash
# GPU-box profiling recipe for round 1 (run from the repo root under gpurun).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r01
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 &&
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_valu -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_valu.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_write.log 2>&1
rc=$?
cat $O/bench.json
echo "profile rc=$rc"
exit $rc
