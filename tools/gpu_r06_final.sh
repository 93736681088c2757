#!/bin/bash
# Round-6 final validation, part 1 (GPU box), after the last kernel change:
# the GPU suite as the driver runs it, smoke(), the PMC passes of the cfg2 /
# cfg3 / d = 12 dominant kernels summarised for the loaded code object
# (written to profiles/r06/pmc_summary.json on the box, so the bench line's
# `traffic` uses it, and to $O/summary), the default bench line, and
# rocprofv3 --stats of the bench with serial launches.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06final}
mkdir -p $O/cfg3 $O/cfg4
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
prc=$?
tail -3 $O/pytest_gpu.log
if [ $prc -gt 1 ]; then echo "pytest rc=$prc: stopping"; exit $prc; fi
M=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
P="timeout -s KILL 90 rocprofv3 --kernel-trace"
V="--pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
$P $V -d $O/pmc_valu -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 0 4294967295 1 > $O/pmc_write.log 2>&1 &&
$P $V -d $O/cfg3/pmc_valu -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/cfg3/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/cfg3/pmc_write -o run --output-format csv -- python tools/quick_scan.py "$M" 0 4294967295 1 > $O/cfg3/pmc_write.log 2>&1 &&
$P $V -d $O/cfg4/pmc_valu -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 299999999999 1 > $O/cfg4/pmc_valu.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/cfg4/pmc_fetch -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 299999999999 1 > $O/cfg4/pmc_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/cfg4/pmc_write -o run --output-format csv -- python tools/quick_scan.py bradfitz 100000000000 299999999999 1 > $O/cfg4/pmc_write.log 2>&1 &&
python tools/summarize_profile.py $O $O/summary > /dev/null &&
python tools/summarize_profile.py $O/cfg3 $O/summary > /dev/null &&
python tools/summarize_profile.py $O/cfg4 $O/summary > /dev/null &&
mkdir -p profiles/r06 && cp $O/summary/pmc_summary.json profiles/r06/pmc_summary.json &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
HM_BENCH_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/bench_serial.json 2> $O/serial.log
rc=$?
tail -2 $O/smoke.log; head -3 $O/serial/run_kernel_stats.csv 2>/dev/null; head -c 400 $O/bench.json
echo "final rc=$rc"
exit $rc
