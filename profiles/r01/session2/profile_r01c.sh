#!/bin/bash
# GPU-box recipe (round 1, second session): PMC passes for the tiled (cfg2)
# and chained (cfg3) kernels, cfg3 bench + kernel trace.  One counter group
# per rocprofv3 run (MI355X_MICROARCH.md HBM/rocprofv3 section).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r01c
mkdir -p $O/cfg3
M=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
P="timeout -s KILL 240 rocprofv3 --kernel-trace"
$P --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_valu -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_write.log 2>&1 &&
$P --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/cfg3/pmc_valu -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/cfg3/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/cfg3/pmc_write -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_write.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg3 --no-cpu-baseline > $O/cfg3/bench.json 2> $O/cfg3/bench.err &&
$P --stats -d $O/cfg3/trace -o run --output-format csv -- python bench.py --workload cfg3 --steps 5 --warmup 1 --no-cpu-baseline > $O/cfg3/trace.log 2>&1
rc=$?
cat $O/cfg3/bench.json
echo "profile rc=$rc"
exit $rc
