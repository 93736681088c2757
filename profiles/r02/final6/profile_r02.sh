#!/bin/bash
# GPU-box recipe (round 2): PMC passes (one counter group per rocprofv3 run,
# MI355X_MICROARCH.md HBM/rocprofv3 section) for the cfg2 tiled and cfg3
# chained kernels, and a kernel trace of the bench with strictly serial
# launches (HM_BENCH_STREAMS=1) beside the default multi-stream trace.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r02p}
mkdir -p $O/cfg3
M=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
P="timeout -s KILL 90 rocprofv3 --kernel-trace"
$P --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_valu -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_write.log 2>&1 &&
$P --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/cfg3/pmc_valu -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/cfg3/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/cfg3/pmc_write -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_write.log 2>&1 &&
mkdir -p $O/cfg4 &&
$P --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/cfg4/pmc_valu -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 119999999999 1 > $O/cfg4/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/cfg4/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 119999999999 1 > $O/cfg4/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/cfg4/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 119999999999 1 > $O/cfg4/pmc_write.log 2>&1 &&
HM_BENCH_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_serial -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/trace_serial.log 2>&1
rc=$?
echo "profile rc=$rc"
exit $rc
